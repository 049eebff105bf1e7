#include "proto.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>

namespace natscore {

namespace {
std::vector<std::string> fields(const std::string& s, size_t from) {
  std::vector<std::string> f;
  size_t i = from;
  while (i < s.size()) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
    size_t st = i;
    while (i < s.size() && s[i] != ' ' && s[i] != '\t') ++i;
    if (i > st) f.push_back(s.substr(st, i - st));
  }
  return f;
}

bool to_long(const std::string& s, long& v) {
  if (s.empty()) return false;
  char* e = nullptr;
  v = std::strtol(s.c_str(), &e, 10);
  return *e == 0 && v >= 0;
}

std::string upper(const std::string& s) {
  std::string r = s;
  for (auto& c : r) c = (char)std::toupper((unsigned char)c);
  return r;
}
}  // namespace

bool Parser::parse_line(const std::string& line, Op& op, long& need_total, long& need_hdr) {
  need_total = -1;
  need_hdr = 0;
  size_t sp = line.find_first_of(" \t");
  std::string verb = upper(line.substr(0, sp));
  std::string rest = sp == std::string::npos ? "" : line.substr(sp + 1);
  if (verb == "PING") { op.kind = Op::PING; return true; }
  if (verb == "PONG") { op.kind = Op::PONG; return true; }
  if (verb == "+OK") { op.kind = Op::OK; return true; }
  if (verb == "-ERR") { op.kind = Op::ERR; op.arg = rest; return true; }
  if (verb == "INFO") { op.kind = Op::INFO; op.arg = rest; return true; }
  if (verb == "CONNECT") { op.kind = Op::CONNECT; op.arg = rest; return true; }
  auto f = fields(line, sp == std::string::npos ? line.size() : sp);
  long a = 0, b = 0;
  if (verb == "PUB") {
    op.kind = Op::PUB;
    if (f.size() == 2 && to_long(f[1], a)) { op.subject = f[0]; }
    else if (f.size() == 3 && to_long(f[2], a)) { op.subject = f[0]; op.reply = f[1]; }
    else { err_ = "Unknown Protocol Operation"; return false; }
    need_total = a;
    return true;
  }
  if (verb == "HPUB") {
    op.kind = Op::HPUB;
    if (f.size() == 3 && to_long(f[1], a) && to_long(f[2], b)) { op.subject = f[0]; }
    else if (f.size() == 4 && to_long(f[2], a) && to_long(f[3], b)) { op.subject = f[0]; op.reply = f[1]; }
    else { err_ = "Unknown Protocol Operation"; return false; }
    if (a > b) { err_ = "bad header size"; return false; }
    need_hdr = a;
    need_total = b;
    return true;
  }
  if (verb == "MSG") {
    op.kind = Op::MSG;
    if (f.size() == 3 && to_long(f[2], a)) { op.subject = f[0]; op.sid = f[1]; }
    else if (f.size() == 4 && to_long(f[3], a)) { op.subject = f[0]; op.sid = f[1]; op.reply = f[2]; }
    else { err_ = "bad MSG"; return false; }
    need_total = a;
    return true;
  }
  if (verb == "HMSG") {
    op.kind = Op::HMSG;
    if (f.size() == 4 && to_long(f[2], a) && to_long(f[3], b)) { op.subject = f[0]; op.sid = f[1]; }
    else if (f.size() == 5 && to_long(f[3], a) && to_long(f[4], b)) {
      op.subject = f[0]; op.sid = f[1]; op.reply = f[2];
    } else { err_ = "bad HMSG"; return false; }
    if (a > b) { err_ = "bad header size"; return false; }
    need_hdr = a;
    need_total = b;
    return true;
  }
  if (verb == "SUB") {
    op.kind = Op::SUB;
    if (f.size() == 2) { op.subject = f[0]; op.sid = f[1]; }
    else if (f.size() == 3) { op.subject = f[0]; op.queue = f[1]; op.sid = f[2]; }
    else { err_ = "Unknown Protocol Operation"; return false; }
    return true;
  }
  if (verb == "UNSUB") {
    op.kind = Op::UNSUB;
    if (f.size() == 1) { op.sid = f[0]; }
    else if (f.size() == 2 && to_long(f[1], a)) { op.sid = f[0]; op.max_msgs = a; }
    else { err_ = "Unknown Protocol Operation"; return false; }
    return true;
  }
  err_ = "Unknown Protocol Operation";
  return false;
}

bool Parser::feed(const char* data, size_t n, const std::function<void(Op&)>& on_op) {
  buf_.append(data, n);
  while (true) {
    size_t eol = buf_.find("\r\n", off_);
    if (eol == std::string::npos) {
      if (buf_.size() - off_ > 64 * 1024) { err_ = "Maximum Control Line Exceeded"; return false; }
      break;
    }
    std::string line = buf_.substr(off_, eol - off_);
    Op op;
    long need_total = -1, need_hdr = 0;
    if (!parse_line(line, op, need_total, need_hdr)) return false;
    if (need_total >= 0) {
      if ((size_t)need_total > max_payload_) { err_ = "Maximum Payload Violation"; return false; }
      size_t body = eol + 2;
      if (buf_.size() < body + (size_t)need_total + 2) break;   // wait for the payload
      if (buf_.compare(body + need_total, 2, "\r\n") != 0) { err_ = "bad payload terminator"; return false; }
      op.hdr = buf_.substr(body, need_hdr);
      op.payload = buf_.substr(body + need_hdr, need_total - need_hdr);
      off_ = body + need_total + 2;
    } else {
      off_ = eol + 2;
    }
    on_op(op);
  }
  if (off_ > (1 << 20) || off_ == buf_.size()) {
    buf_.erase(0, off_);
    off_ = 0;
  }
  return true;
}

std::string Headers::get(const std::string& k) const {
  for (auto& p : kv) {
    if (p.first.size() != k.size()) continue;
    bool eq = true;
    for (size_t i = 0; i < k.size(); ++i)
      if (std::tolower((unsigned char)p.first[i]) != std::tolower((unsigned char)k[i])) { eq = false; break; }
    if (eq) return p.second;
  }
  return "";
}

Headers parse_headers(const std::string& raw) {
  Headers h;
  size_t eol = raw.find("\r\n");
  std::string first = raw.substr(0, eol);
  if (first.rfind("NATS/1.0", 0) == 0) {
    std::string rest = first.substr(8);
    size_t i = rest.find_first_not_of(' ');
    if (i != std::string::npos) {
      rest = rest.substr(i);
      h.status = std::atoi(rest.substr(0, 3).c_str());
      if (rest.size() > 4) h.description = rest.substr(4);
    }
  }
  size_t pos = eol == std::string::npos ? raw.size() : eol + 2;
  while (pos < raw.size()) {
    size_t e = raw.find("\r\n", pos);
    if (e == std::string::npos) e = raw.size();
    std::string l = raw.substr(pos, e - pos);
    pos = e + 2;
    if (l.empty()) break;
    size_t c = l.find(':');
    if (c == std::string::npos) continue;
    std::string k = l.substr(0, c), v = l.substr(c + 1);
    size_t vs = v.find_first_not_of(' ');
    v = vs == std::string::npos ? "" : v.substr(vs);
    h.kv.emplace_back(k, v);
  }
  return h;
}

std::string build_headers(const std::vector<std::pair<std::string, std::string>>& kv, int status,
                          const std::string& desc) {
  std::string s = "NATS/1.0";
  if (status) {
    s += " " + std::to_string(status);
    if (!desc.empty()) s += " " + desc;
  }
  s += "\r\n";
  for (auto& p : kv) s += p.first + ": " + p.second + "\r\n";
  s += "\r\n";
  return s;
}

}  // namespace natscore
