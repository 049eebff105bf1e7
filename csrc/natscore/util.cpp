#include "util.h"

#include <openssl/evp.h>
#include <openssl/rand.h>

#include <cpuid.h>
#include <immintrin.h>
#include <cstdlib>

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <mutex>
#include <random>
#include <sstream>

namespace natscore {

// ============================ JSON ==========================================
namespace {
struct JP {
  const std::string& s;
  size_t i = 0;
  explicit JP(const std::string& x) : s(x) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at " + std::to_string(i));
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) fail("bad \\u escape");
    uint32_t v = (uint32_t)std::stoul(s.substr(i, 4), nullptr, 16);
    i += 4;
    return v;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              i += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    if (i >= s.size()) fail("unterminated string");
    ++i;
    return out;
  }
  Json val(int depth = 0) {
    if (depth > 64) fail("too deep");
    ws();
    if (i >= s.size()) fail("eof");
    Json j;
    char c = s[i];
    if (c == '{') {
      j.t = Json::OBJ;
      ++i;
      ws();
      if (s[i] == '}') { ++i; return j; }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (s[i] != ':') fail("expected :");
        ++i;
        j.o.emplace_back(k, val(depth + 1));
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == '}') { ++i; break; }
        fail("expected , or }");
      }
    } else if (c == '[') {
      j.t = Json::ARR;
      ++i;
      ws();
      if (s[i] == ']') { ++i; return j; }
      while (true) {
        j.a.push_back(val(depth + 1));
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == ']') { ++i; break; }
        fail("expected , or ]");
      }
    } else if (c == '"') {
      j.t = Json::STR;
      j.s = str();
    } else if (s.compare(i, 4, "true") == 0) { j.t = Json::BOOL; j.b = true; i += 4; }
    else if (s.compare(i, 5, "false") == 0) { j.t = Json::BOOL; j.b = false; i += 5; }
    else if (s.compare(i, 4, "null") == 0) { j.t = Json::NUL; i += 4; }
    else {
      size_t st = i;
      while (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '-' || s[i] == '+' || s[i] == '.' ||
                              s[i] == 'e' || s[i] == 'E'))
        ++i;
      if (st == i) fail("unexpected character");
      j.t = Json::NUM;
      j.n = std::stod(s.substr(st, i - st));
    }
    return j;
  }
};
}  // namespace

Json Json::parse(const std::string& text) {
  JP p(text);
  Json j = p.val();
  p.ws();
  if (p.i != text.size()) p.fail("trailing data");
  return j;
}

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
    }
  }
  return o;
}

std::string Json::dump() const {
  switch (t) {
    case NUL: return "null";
    case BOOL: return b ? "true" : "false";
    case NUM: {
      if (std::isfinite(n) && n == std::floor(n) && std::fabs(n) < 9.007199254740992e15) {
        char buf[32];
        snprintf(buf, sizeof buf, "%lld", (long long)n);
        return buf;
      }
      char buf[64];
      snprintf(buf, sizeof buf, "%.17g", n);
      return buf;
    }
    case STR: return "\"" + json_escape(s) + "\"";
    case ARR: {
      std::string r = "[";
      for (size_t k = 0; k < a.size(); ++k) {
        if (k) r += ",";
        r += a[k].dump();
      }
      return r + "]";
    }
    case OBJ: {
      std::string r = "{";
      for (size_t k = 0; k < o.size(); ++k) {
        if (k) r += ",";
        r += "\"" + json_escape(o[k].first) + "\":" + o[k].second.dump();
      }
      return r + "}";
    }
  }
  return "null";
}

// ============================ base64 ========================================
static const char* B64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
static const char* B64U = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

std::string b64encode(const std::string& in, bool url, bool pad) {
  const char* tb = url ? B64U : B64;
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    out += tb[v >> 18]; out += tb[(v >> 12) & 63]; out += tb[(v >> 6) & 63]; out += tb[v & 63];
  }
  if (i + 1 == in.size()) {
    uint32_t v = (uint8_t)in[i] << 16;
    out += tb[v >> 18]; out += tb[(v >> 12) & 63];
    if (pad) out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    out += tb[v >> 18]; out += tb[(v >> 12) & 63]; out += tb[(v >> 6) & 63];
    if (pad) out += "=";
  }
  return out;
}

std::string b64decode(const std::string& in) {
  int8_t rev[256];
  memset(rev, -1, sizeof rev);
  for (int k = 0; k < 64; ++k) { rev[(uint8_t)B64[k]] = k; rev[(uint8_t)B64U[k]] = k; }
  std::string out;
  uint32_t acc = 0;
  int bits = 0;
  for (unsigned char c : in) {
    if (c == '=' || c == '\n' || c == '\r') continue;
    if (rev[c] < 0) throw std::runtime_error("bad base64");
    acc = (acc << 6) | rev[c];
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out += (char)((acc >> bits) & 0xFF);
    }
  }
  return out;
}

// ============================ SHA-256 =======================================
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

static inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

Sha256::Sha256() {
  const uint32_t init[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(h_, init, sizeof h_);
}

void Sha256::block(const uint8_t* p) {
  uint32_t w[64];
  for (int k = 0; k < 16; ++k) w[k] = (p[4 * k] << 24) | (p[4 * k + 1] << 16) | (p[4 * k + 2] << 8) | p[4 * k + 3];
  for (int k = 16; k < 64; ++k) {
    uint32_t s0 = ror(w[k - 15], 7) ^ ror(w[k - 15], 18) ^ (w[k - 15] >> 3);
    uint32_t s1 = ror(w[k - 2], 17) ^ ror(w[k - 2], 19) ^ (w[k - 2] >> 10);
    w[k] = w[k - 16] + s0 + w[k - 7] + s1;
  }
  uint32_t a = h_[0], b = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6], h = h_[7];
  for (int k = 0; k < 64; ++k) {
    uint32_t S1 = ror(e, 6) ^ ror(e, 11) ^ ror(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K256[k] + w[k];
    uint32_t S0 = ror(a, 2) ^ ror(a, 13) ^ ror(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h_[0] += a; h_[1] += b; h_[2] += c; h_[3] += d; h_[4] += e; h_[5] += f; h_[6] += g; h_[7] += h;
}

// x86 SHA extensions (SHA-NI): the compression function of n consecutive 64-byte blocks, ~10x the
// scalar code (model pulls hash multi-GB objects). State layout per the instruction set: ABEF / CDGH.
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_ni_blocks(uint32_t* h, const uint8_t* p, size_t n) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[0]), 0xB1);   // CDAB
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[4]), 0x1B);  // HGFE
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                          // ABEF
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                               // CDGH
  for (; n; --n, p += 64) {
    const __m128i abef = s0, cdgh = s1;
    __m128i w[4];
#pragma GCC unroll 16
    for (int i = 0; i < 16; ++i) {
      __m128i wi;
      if (i < 4) {
        wi = w[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), bswap);
      } else {   // words 4i..4i+3 from groups i-4 .. i-1
        __m128i m = _mm_sha256msg1_epu32(w[i & 3], w[(i + 1) & 3]);
        m = _mm_add_epi32(m, _mm_alignr_epi8(w[(i + 3) & 3], w[(i + 2) & 3], 4));
        wi = w[i & 3] = _mm_sha256msg2_epu32(m, w[(i + 3) & 3]);
      }
      const __m128i k = _mm_add_epi32(wi, _mm_loadu_si128((const __m128i*)&K256[4 * i]));
      s1 = _mm_sha256rnds2_epu32(s1, s0, k);
      s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(k, 0x0E));
    }
    s0 = _mm_add_epi32(s0, abef);
    s1 = _mm_add_epi32(s1, cdgh);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);                 // FEBA
  s1 = _mm_shuffle_epi32(s1, 0xB1);                // DCHG
  s0 = _mm_blend_epi16(t, s1, 0xF0);               // DCBA
  s1 = _mm_alignr_epi8(s1, t, 8);                  // HGFE
  _mm_storeu_si128((__m128i*)&h[0], s0);
  _mm_storeu_si128((__m128i*)&h[4], s1);
}

static bool cpu_has_sha() {
  unsigned a = 0, b = 0, c = 0, d = 0;
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  const bool sha = (b >> 29) & 1;
  __get_cpuid(1, &a, &b, &c, &d);
  return sha && ((c >> 19) & 1) && ((c >> 9) & 1);       // + SSE4.1, SSSE3
}
static const bool g_sha_ni = cpu_has_sha() && !getenv("NATSCORE_NO_SHA_NI");

void Sha256::blocks(const uint8_t* p, size_t n) {
  if (g_sha_ni) {
    sha256_ni_blocks(h_, p, n);
    return;
  }
  for (; n; --n, p += 64) block(p);
}

void Sha256::update(const void* data, size_t len) {
  const uint8_t* p = (const uint8_t*)data;
  total_ += len;
  if (blen_) {
    size_t take = std::min(len, 64 - blen_);
    memcpy(buf_ + blen_, p, take);
    blen_ += take; p += take; len -= take;
    if (blen_ == 64) { blocks(buf_, 1); blen_ = 0; }
  }
  if (len >= 64) {
    const size_t nb = len / 64;
    blocks(p, nb);
    p += 64 * nb;
    len -= 64 * nb;
  }
  if (len) { memcpy(buf_, p, len); blen_ = len; }
}

std::string Sha256::digest() {
  uint64_t bits = total_ * 8;
  uint8_t pad = 0x80;
  update(&pad, 1);
  uint8_t z = 0;
  while (blen_ != 56) update(&z, 1);
  uint8_t L[8];
  for (int k = 0; k < 8; ++k) L[k] = (uint8_t)(bits >> (56 - 8 * k));
  update(L, 8);
  std::string out(32, '\0');
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (char)(h_[k] >> 24); out[4 * k + 1] = (char)(h_[k] >> 16);
    out[4 * k + 2] = (char)(h_[k] >> 8); out[4 * k + 3] = (char)h_[k];
  }
  return out;
}

// ============================ NUID ==========================================
std::string nuid_next() {
  static const char* D = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz";
  static std::mutex mu;
  static std::mt19937_64 rng{std::random_device{}() ^
                             (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count()};
  static std::string pre;
  static uint64_t seq = 0, inc = 0;
  std::lock_guard<std::mutex> g(mu);
  if (pre.empty() || seq >= 839299365868340224ULL) {   // 62^10
    pre.clear();
    for (int k = 0; k < 12; ++k) pre += D[rng() % 62];
    seq = rng() % 839299365868340224ULL;
    inc = 33 + rng() % 300;
  }
  seq += inc;
  std::string s = pre;
  uint64_t v = seq;
  char tail[10];
  for (int k = 9; k >= 0; --k) { tail[k] = D[v % 62]; v /= 62; }
  s.append(tail, 10);
  return s;
}

// ============================ subjects ======================================
std::vector<std::string> split_tokens(const std::string& subj) {
  std::vector<std::string> t;
  size_t st = 0;
  for (size_t k = 0; k <= subj.size(); ++k) {
    if (k == subj.size() || subj[k] == '.') {
      t.push_back(subj.substr(st, k - st));
      st = k + 1;
    }
  }
  return t;
}

bool subject_matches(const std::string& pattern, const std::string& subject) {
  if (pattern == subject) return true;
  size_t pi = 0, si = 0;
  const size_t pn = pattern.size(), sn = subject.size();
  while (pi < pn && si < sn) {
    size_t pe = pattern.find('.', pi);
    if (pe == std::string::npos) pe = pn;
    size_t se = subject.find('.', si);
    if (se == std::string::npos) se = sn;
    const size_t pl = pe - pi;
    if (pl == 1 && pattern[pi] == '>') return true;
    if (!(pl == 1 && pattern[pi] == '*')) {
      if (pl != se - si || pattern.compare(pi, pl, subject, si, pl) != 0) return false;
    }
    pi = pe + 1;
    si = se + 1;
    if (pe == pn || se == sn) return pe == pn && se == sn;
  }
  return false;
}

bool valid_subject(const std::string& s, bool allow_wildcards) {
  if (s.empty() || s.front() == '.' || s.back() == '.') return false;
  auto toks = split_tokens(s);
  for (size_t k = 0; k < toks.size(); ++k) {
    auto& t = toks[k];
    if (t.empty()) return false;
    for (char c : t)
      if (c == ' ' || c == '\t' || c == '\r' || c == '\n') return false;
    if (!allow_wildcards && (t == "*" || t == ">")) return false;
    if (t == ">" && k + 1 != toks.size()) return false;
  }
  return true;
}

// ============================ sockets =======================================
int tcp_listen(const std::string& host, int port, int* bound_port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.empty() ? "127.0.0.1" : host.c_str(), &a.sin_addr) != 1) {
    ::close(fd);
    return -1;
  }
  if (::bind(fd, (sockaddr*)&a, sizeof a) < 0 || ::listen(fd, 512) < 0) {
    ::close(fd);
    return -1;
  }
  socklen_t l = sizeof a;
  getsockname(fd, (sockaddr*)&a, &l);
  if (bound_port) *bound_port = ntohs(a.sin_port);
  return fd;
}

int tcp_connect(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) { freeaddrinfo(res); return -1; }
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc < 0 && errno != EINPROGRESS) { ::close(fd); return -1; }
  if (rc < 0) {
    pollfd p{fd, POLLOUT, 0};
    if (poll(&p, 1, timeout_ms) <= 0) { ::close(fd); return -1; }
    int err = 0;
    socklen_t el = sizeof err;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el);
    if (err) { ::close(fd); return -1; }
  }
  fcntl(fd, F_SETFL, fl);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int big = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
  return fd;
}

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

}  // namespace natscore


// ============================== nkeys / auth ===============================
namespace natscore {

static const char B32[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZ234567";

std::string base32_encode(const std::string& raw) {
  std::string out;
  uint32_t buf = 0;
  int bits = 0;
  for (unsigned char c : raw) {
    buf = (buf << 8) | c;
    bits += 8;
    while (bits >= 5) {
      out += B32[(buf >> (bits - 5)) & 31];
      bits -= 5;
    }
  }
  if (bits > 0) out += B32[(buf << (5 - bits)) & 31];
  return out;
}

bool base32_decode(const std::string& s, std::string& raw) {
  raw.clear();
  uint32_t buf = 0;
  int bits = 0;
  for (char ch : s) {
    int v;
    if (ch >= 'A' && ch <= 'Z') v = ch - 'A';
    else if (ch >= '2' && ch <= '7') v = ch - '2' + 26;
    else if (ch == '=') break;
    else return false;
    buf = (buf << 5) | (uint32_t)v;
    bits += 5;
    if (bits >= 8) {
      raw += (char)((buf >> (bits - 8)) & 0xFF);
      bits -= 8;
    }
  }
  return true;
}

uint16_t crc16_xmodem(const std::string& data) {
  uint16_t crc = 0;
  for (unsigned char c : data) {
    crc ^= (uint16_t)c << 8;
    for (int i = 0; i < 8; ++i) crc = (crc & 0x8000) ? (uint16_t)((crc << 1) ^ 0x1021) : (uint16_t)(crc << 1);
  }
  return crc;
}

static bool nkey_unwrap(const std::string& text, std::string& body) {
  std::string raw;
  if (!base32_decode(text, raw) || raw.size() < 3) return false;
  body = raw.substr(0, raw.size() - 2);
  const uint16_t crc = (uint16_t)((unsigned char)raw[raw.size() - 2] | ((unsigned char)raw[raw.size() - 1] << 8));
  return crc16_xmodem(body) == crc;
}

static std::string nkey_wrap(const std::string& body) {
  const uint16_t crc = crc16_xmodem(body);
  return base32_encode(body + std::string(1, (char)(crc & 0xFF)) + std::string(1, (char)(crc >> 8)));
}

bool nkey_seed_raw(const std::string& seed, std::string& raw32) {
  std::string body;
  if (!nkey_unwrap(seed, body) || body.size() != 34) return false;
  const uint8_t b0 = (uint8_t)body[0], b1 = (uint8_t)body[1];
  if ((b0 & 0xF8) != NKEY_PREFIX_SEED) return false;
  const uint8_t kind = (uint8_t)(((b0 & 7) << 5) | ((b1 & 0xF8) >> 3));
  if (kind != NKEY_PREFIX_USER) return false;           // user seeds only ("SU...")
  raw32 = body.substr(2, 32);
  return true;
}

static EVP_PKEY* ed_priv(const std::string& raw32) {
  return EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, (const unsigned char*)raw32.data(), 32);
}

std::string nkey_public(const std::string& raw32) {
  EVP_PKEY* k = ed_priv(raw32);
  if (!k) throw std::runtime_error("nkey: bad seed");
  unsigned char pub[32];
  size_t n = sizeof pub;
  EVP_PKEY_get_raw_public_key(k, pub, &n);
  EVP_PKEY_free(k);
  return nkey_wrap(std::string(1, (char)NKEY_PREFIX_USER) + std::string((const char*)pub, 32));
}

std::string nkey_sign(const std::string& raw32, const std::string& msg) {
  EVP_PKEY* k = ed_priv(raw32);
  if (!k) throw std::runtime_error("nkey: bad seed");
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  unsigned char sig[64];
  size_t n = sizeof sig;
  const bool ok = EVP_DigestSignInit(ctx, nullptr, nullptr, nullptr, k) == 1 &&
                  EVP_DigestSign(ctx, sig, &n, (const unsigned char*)msg.data(), msg.size()) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(k);
  if (!ok) throw std::runtime_error("nkey: signing failed");
  return std::string((const char*)sig, n);
}

bool nkey_verify(const std::string& pub, const std::string& msg, const std::string& sig) {
  std::string body;
  if (!nkey_unwrap(pub, body) || body.size() != 33 || (uint8_t)body[0] != NKEY_PREFIX_USER || sig.size() != 64)
    return false;
  EVP_PKEY* k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, (const unsigned char*)body.data() + 1, 32);
  if (!k) return false;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  const bool ok = EVP_DigestVerifyInit(ctx, nullptr, nullptr, nullptr, k) == 1 &&
                  EVP_DigestVerify(ctx, (const unsigned char*)sig.data(), sig.size(), (const unsigned char*)msg.data(),
                                   msg.size()) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(k);
  return ok;
}

std::string random_b64url(size_t nbytes) {
  std::string r(nbytes, '\0');
  RAND_bytes((unsigned char*)&r[0], (int)nbytes);
  std::string s = b64encode(r, true);
  while (!s.empty() && s.back() == '=') s.pop_back();
  return s;
}

bool ct_equal(const std::string& a, const std::string& b) {
  unsigned char d = a.size() != b.size();
  for (size_t i = 0; i < std::min(a.size(), b.size()); ++i) d |= (unsigned char)(a[i] ^ b[i]);
  return d == 0;
}

static std::string between(const std::string& t, const std::string& begin) {
  size_t a = t.find(begin);
  if (a == std::string::npos) return "";
  a = t.find('\n', a);
  if (a == std::string::npos) return "";
  size_t b = t.find("---", a + 1);
  std::string s = t.substr(a + 1, (b == std::string::npos ? t.size() : b) - a - 1);
  std::string out;
  for (char c : s)
    if (!isspace((unsigned char)c)) out += c;
  return out;
}

bool parse_creds(const std::string& text, std::string& jwt, std::string& seed) {
  jwt = between(text, "BEGIN NATS USER JWT");
  seed = between(text, "BEGIN USER NKEY SEED");
  return !seed.empty();
}

}  // namespace natscore
