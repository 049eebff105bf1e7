// NATS client protocol: incremental parser + header codec.
// Wire contract per the public NATS protocol (INFO/CONNECT/PUB/HPUB/SUB/UNSUB/MSG/HMSG/
// PING/PONG/+OK/-ERR); headers are "NATS/1.0[ status[ text]]\r\nK: V\r\n...\r\n".
#pragma once
#include <functional>
#include <string>
#include <utility>
#include <vector>

namespace natscore {

struct Op {
  enum Kind { INFO, CONNECT, PUB, HPUB, SUB, UNSUB, MSG, HMSG, PING, PONG, OK, ERR } kind = PING;
  std::string subject, reply, queue, sid, arg;
  long max_msgs = 0;
  std::string hdr;       // raw header block (HPUB/HMSG), includes trailing \r\n\r\n
  std::string payload;   // message body (without headers)
};

class Parser {
 public:
  explicit Parser(size_t max_payload = 64ull << 20) : max_payload_(max_payload) {}
  // Feeds bytes; calls on_op for every complete op. Returns false on a protocol error (see error()).
  bool feed(const char* data, size_t n, const std::function<void(Op&)>& on_op);
  const std::string& error() const { return err_; }
  void reset() { buf_.clear(); off_ = 0; }

 private:
  bool parse_line(const std::string& line, Op& op, long& need_total, long& need_hdr);
  std::string buf_;
  size_t off_ = 0;
  size_t max_payload_;
  std::string err_;
};

struct Headers {
  int status = 0;                 // e.g. 503 no responders
  std::string description;
  std::vector<std::pair<std::string, std::string>> kv;
  std::string get(const std::string& k) const;
};

Headers parse_headers(const std::string& raw);
std::string build_headers(const std::vector<std::pair<std::string, std::string>>& kv, int status = 0,
                          const std::string& desc = "");

}  // namespace natscore
