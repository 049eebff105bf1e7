// natscore: small self-contained helpers (JSON, base64, SHA-256, NUID, sockets).
// No third-party dependencies: the image has no nats.c / nats-server / nats-py.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace natscore {

// ---------------------------------------------------------------------------
// Minimal JSON value (enough for INFO/CONNECT and the JetStream API subset)
// ---------------------------------------------------------------------------
struct Json {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<Json> a;
  std::vector<std::pair<std::string, Json>> o;

  static Json parse(const std::string& text);
  std::string dump() const;

  const Json* get(const std::string& k) const {
    if (t != OBJ) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  std::string str(const std::string& k, const std::string& d = "") const {
    auto* v = get(k);
    return v && v->t == STR ? v->s : d;
  }
  double num(const std::string& k, double d = 0) const {
    auto* v = get(k);
    return v && v->t == NUM ? v->n : d;
  }
  bool boolean(const std::string& k, bool d = false) const {
    auto* v = get(k);
    return v && v->t == BOOL ? v->b : d;
  }
  Json& set(const std::string& k, Json v) {
    if (t != OBJ) { t = OBJ; o.clear(); }
    for (auto& kv : o)
      if (kv.first == k) { kv.second = std::move(v); return kv.second; }
    o.emplace_back(k, std::move(v));
    return o.back().second;
  }
  static Json S(const std::string& v) { Json j; j.t = STR; j.s = v; return j; }
  static Json N(double v) { Json j; j.t = NUM; j.n = v; return j; }
  static Json B(bool v) { Json j; j.t = BOOL; j.b = v; return j; }
  static Json O() { Json j; j.t = OBJ; return j; }
  static Json A() { Json j; j.t = ARR; return j; }
};

std::string json_escape(const std::string& s);

// ---------------------------------------------------------------------------
// base64 (std + url alphabets), SHA-256, NUID
// ---------------------------------------------------------------------------
std::string b64encode(const std::string& in, bool url = false, bool pad = true);
std::string b64decode(const std::string& in);

class Sha256 {
 public:
  Sha256();
  void update(const void* data, size_t len);
  std::string digest();   // 32 raw bytes
 private:
  void block(const uint8_t* p);                 // scalar compression of one block
  void blocks(const uint8_t* p, size_t n);      // n blocks (SHA-NI when the CPU has it)
  uint32_t h_[8];
  uint8_t buf_[64];
  size_t blen_ = 0;
  uint64_t total_ = 0;
};

std::string nuid_next();          // 22-char base62 unique id

// ---------------------------------------------------------------------------
// NATS nkeys (ed25519 identities, base32 + CRC16 text form) and auth helpers
// ---------------------------------------------------------------------------
std::string base32_encode(const std::string& raw);               // RFC 4648, no padding
bool base32_decode(const std::string& s, std::string& raw);
uint16_t crc16_xmodem(const std::string& data);
constexpr uint8_t NKEY_PREFIX_SEED = 18 << 3, NKEY_PREFIX_USER = 20 << 3;
// "SU..." user seed -> raw 32-byte ed25519 private seed (false: malformed / bad checksum)
bool nkey_seed_raw(const std::string& seed, std::string& raw32);
std::string nkey_public(const std::string& raw32);               // "U..." public key of a seed
std::string nkey_sign(const std::string& raw32, const std::string& msg);    // 64-byte signature
bool nkey_verify(const std::string& pub, const std::string& msg, const std::string& sig);
std::string random_b64url(size_t nbytes);
bool ct_equal(const std::string& a, const std::string& b);      // constant-time compare
// creds file: the user JWT and the nkey seed between the BEGIN/END markers
bool parse_creds(const std::string& text, std::string& jwt, std::string& seed);

// ---------------------------------------------------------------------------
// Subject helpers
// ---------------------------------------------------------------------------
std::vector<std::string> split_tokens(const std::string& subj);
bool subject_matches(const std::string& pattern, const std::string& subject);
bool valid_subject(const std::string& s, bool allow_wildcards);

// ---------------------------------------------------------------------------
// sockets
// ---------------------------------------------------------------------------
int tcp_listen(const std::string& host, int port, int* bound_port);
int tcp_connect(const std::string& host, int port, int timeout_ms);
bool send_all(int fd, const char* p, size_t n);

}  // namespace natscore
