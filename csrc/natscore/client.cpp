#include "client.h"

#include <sys/socket.h>
#include <unistd.h>

#include <chrono>

namespace natscore {

Client::Client() {}

Client::~Client() { close(); }

static std::string pct_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o += (char)std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
      i += 2;
    } else {
      o += s[i];
    }
  }
  return o;
}

// nats://[user:pass@ | token@]host[:port]: URL credentials fill the options the caller left empty
static void parse_url(const std::string& url, std::string& host, int& port, ClientOptions& opt) {
  std::string u = url;
  auto p = u.find("://");
  if (p != std::string::npos) {
    if (u.compare(0, p, "tls") == 0) opt.tls.enable = true;
    u = u.substr(p + 3);
  }
  auto at = u.rfind('@');
  if (at != std::string::npos) {
    const std::string ui = u.substr(0, at);
    const auto c = ui.find(':');
    if (c != std::string::npos) {
      if (opt.user.empty()) opt.user = pct_decode(ui.substr(0, c));
      if (opt.pass.empty()) opt.pass = pct_decode(ui.substr(c + 1));
    } else if (opt.token.empty()) {
      opt.token = pct_decode(ui);
    }
    u = u.substr(at + 1);
  }
  auto sl = u.find('/');
  if (sl != std::string::npos) u = u.substr(0, sl);
  auto c = u.rfind(':');
  if (c != std::string::npos) {
    host = u.substr(0, c);
    port = std::atoi(u.substr(c + 1).c_str());
  } else {
    host = u;
    port = 4222;
  }
  if (host.empty() || host == "localhost") host = "127.0.0.1";
}

bool Client::dial() {
  int fd = tcp_connect(host_, port_, opt_.connect_timeout_ms);
  if (fd < 0) return false;
  std::shared_ptr<TlsConn> tls;
  auto tls_up = [&]() {
    tls = std::make_shared<TlsConn>();
    std::string err;
    if (tls->handshake(fd, host_, opt_.tls, opt_.connect_timeout_ms, err)) return true;
    std::lock_guard<std::mutex> g(mu_);
    last_err_ = err;
    return false;
  };
  if (opt_.tls.first && !tls_up()) { ::close(fd); return false; }   // handshake_first: TLS before INFO
  // read INFO line synchronously
  std::string line;
  char ch;
  while (true) {
    const long n = tls ? tls->read(&ch, 1, closing_) : (long)::recv(fd, &ch, 1, 0);
    if (n <= 0) { ::close(fd); return false; }
    line += ch;
    if (line.size() >= 2 && line.compare(line.size() - 2, 2, "\r\n") == 0) break;
    if (line.size() > 65536) { ::close(fd); return false; }
  }
  if (line.rfind("INFO ", 0) != 0) { ::close(fd); return false; }
  std::string nonce;
  bool tls_required = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    info_ = line.substr(5, line.size() - 7);
    try {
      Json j = Json::parse(info_);
      max_payload_ = (size_t)j.num("max_payload", 1 << 20);
      nonce = j.str("nonce");
      tls_required = j.boolean("tls_required", false);
    } catch (...) {
    }
  }
  // the NATS upgrade: the client asked for TLS or the server requires it -> handshake after INFO
  if (!tls && (opt_.tls.enable || tls_required) && !tls_up()) { ::close(fd); return false; }
  Json c = Json::O();
  if (!opt_.token.empty()) c.set("auth_token", Json::S(opt_.token));
  if (!opt_.user.empty()) {
    c.set("user", Json::S(opt_.user));
    c.set("pass", Json::S(opt_.pass));
  }
  if (!opt_.jwt.empty()) c.set("jwt", Json::S(opt_.jwt));
  if (!opt_.nkey_seed.empty()) {
    std::string raw;
    if (!nkey_seed_raw(opt_.nkey_seed, raw)) {
      ::close(fd);
      throw std::runtime_error("nats: invalid nkey seed");
    }
    if (opt_.jwt.empty()) c.set("nkey", Json::S(nkey_public(raw)));
    c.set("sig", Json::S(b64encode(nkey_sign(raw, nonce), true, false)));
  }
  c.set("verbose", Json::B(opt_.verbose));
  c.set("pedantic", Json::B(false));
  c.set("tls_required", Json::B(tls != nullptr));
  c.set("name", Json::S(opt_.name));
  c.set("lang", Json::S("cpp-natscore"));
  c.set("version", Json::S("0.1.0"));
  c.set("protocol", Json::N(1));
  c.set("headers", Json::B(true));
  c.set("no_responders", Json::B(true));
  std::string hello = "CONNECT " + c.dump() + "\r\nPING\r\n";
  // re-establish subscriptions
  {
    std::lock_guard<std::mutex> g(mu_);
    // PING/PONG accounting: PINGs of a previous connection will never be answered (release their
    // waiters), and the handshake PING above counts like any flush PING -- otherwise its PONG runs
    // pongs_recv_ one ahead and the next flush() returns before the server has seen what preceded it
    pongs_recv_ = pings_sent_;
    ++pings_sent_;
    pong_cv_.notify_all();
    for (auto& kv : subs_) {
      if (kv.second->closed) continue;
      hello += "SUB " + kv.second->subject + (kv.second->queue.empty() ? "" : " " + kv.second->queue) + " " +
               std::to_string(kv.first) + "\r\n";
      if (kv.second->max > 0) {
        long left = kv.second->max - kv.second->delivered;
        if (left > 0) hello += "UNSUB " + std::to_string(kv.first) + " " + std::to_string(left) + "\r\n";
      }
    }
  }
  if (!(tls ? tls->write_all(hello.data(), hello.size()) : send_all(fd, hello.data(), hello.size()))) {
    ::close(fd);
    return false;
  }
  {
    std::lock_guard<std::mutex> g(wmu_);
    fd_ = fd;
    tls_ = tls;
  }
  connected_ = true;
  return true;
}

void Client::connect(const std::string& url, ClientOptions opt) {
  if (connected_) throw std::runtime_error("already connected");
  opt_ = opt;
  parse_url(url, host_, port_, opt_);
  // a configured CA bundle or client certificate makes TLS REQUIRED (nats.go: RootCAs / ClientCert imply
  // Secure): never wait for a plaintext INFO's tls_required, which a man in the middle can strip before the
  // client sends its credentials in the clear
  if (!opt_.tls.ca.empty() || !opt_.tls.cert.empty() || !opt_.tls.key.empty()) opt_.tls.enable = true;
  closing_ = false;
  dead_ = false;
  if (!dial()) {
    std::lock_guard<std::mutex> g(mu_);
    throw ConnectionClosedError("nats: cannot connect to " + url + (last_err_.empty() ? "" : ": " + last_err_));
  }
  rth_ = std::thread([this] { reader(); });
  try {
    flush(opt_.connect_timeout_ms);
  } catch (...) {
    std::string e;
    {
      std::lock_guard<std::mutex> g(mu_);
      e = last_err_;
    }
    close();
    if (!e.empty()) throw ConnectionClosedError("nats: " + e);
    throw;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (!last_err_.empty() && last_err_.find("Authorization") != std::string::npos) {
    const std::string e = last_err_;
    throw ConnectionClosedError("nats: " + e);
  }
}

void Client::close() {
  if (closing_.exchange(true)) {
    if (rth_.joinable() && std::this_thread::get_id() != rth_.get_id()) rth_.join();
    return;
  }
  connected_ = false;
  {
    std::lock_guard<std::mutex> g(wmu_);
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
  }
  if (rth_.joinable()) rth_.join();
  {
    std::lock_guard<std::mutex> g(wmu_);
    tls_.reset();
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  fail_all("connection closed");
}

void Client::fail_all(const std::string& why) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : subs_) {
    kv.second->closed = true;
    kv.second->cv.notify_all();
  }
  for (auto& kv : pending_) kv.second->done = true;
  resp_cv_.notify_all();
  pong_cv_.notify_all();
  (void)why;
}

void Client::write_raw(const std::string& s) {
  std::lock_guard<std::mutex> g(wmu_);
  if (fd_ < 0 || !connected_) throw ConnectionClosedError("nats: connection closed");
  if (!(tls_ ? tls_->write_all(s.data(), s.size()) : send_all(fd_, s.data(), s.size()))) {
    connected_ = false;
    ::shutdown(fd_, SHUT_RDWR);
    throw ConnectionClosedError("nats: write failed");
  }
}

void Client::publish(const std::string& subject, const std::string& data, const std::string& reply,
                     const std::string& hdr) {
  if (data.size() + hdr.size() > max_payload_) throw std::runtime_error("nats: maximum payload exceeded");
  std::string m;
  m.reserve(data.size() + hdr.size() + subject.size() + reply.size() + 48);
  if (hdr.empty()) {
    m = "PUB " + subject + (reply.empty() ? "" : " " + reply) + " " + std::to_string(data.size()) + "\r\n";
  } else {
    m = "HPUB " + subject + (reply.empty() ? "" : " " + reply) + " " + std::to_string(hdr.size()) + " " +
        std::to_string(hdr.size() + data.size()) + "\r\n" + hdr;
  }
  m += data;
  m += "\r\n";
  write_raw(m);
  out_msgs_++;
  out_bytes_ += data.size();
}

int64_t Client::subscribe(const std::string& subject, const std::string& queue) {
  if (!valid_subject(subject, true)) throw std::runtime_error("nats: invalid subject '" + subject + "'");
  int64_t sid;
  {
    std::lock_guard<std::mutex> g(mu_);
    sid = next_sid_++;
    auto s = std::make_shared<Sub>();
    s->subject = subject;
    s->queue = queue;
    subs_[sid] = s;
  }
  write_raw("SUB " + subject + (queue.empty() ? "" : " " + queue) + " " + std::to_string(sid) + "\r\n");
  return sid;
}

void Client::unsubscribe(int64_t sid, long max_msgs) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = subs_.find(sid);
    if (it == subs_.end()) return;
    if (max_msgs > 0) {
      it->second->max = max_msgs;
    } else {
      it->second->closed = true;
      it->second->cv.notify_all();
      subs_.erase(it);
    }
  }
  try {
    write_raw("UNSUB " + std::to_string(sid) + (max_msgs > 0 ? " " + std::to_string(max_msgs) : "") + "\r\n");
  } catch (...) {
  }
}

Msg Client::next_msg(int64_t sid, int timeout_ms) {
  std::unique_lock<std::mutex> g(mu_);
  auto it = subs_.find(sid);
  if (it == subs_.end()) throw std::runtime_error("nats: invalid subscription");
  auto s = it->second;
  auto ready = [&] { return !s->q.empty() || s->closed || closing_; };
  if (timeout_ms < 0) s->cv.wait(g, ready);
  else if (!s->cv.wait_for(g, std::chrono::milliseconds(timeout_ms), ready)) throw TimeoutError("nats: timeout");
  if (s->q.empty()) {
    if (s->closed && s->max > 0) subs_.erase(sid);   // auto-unsubscribed and fully drained
    throw ConnectionClosedError("nats: subscription closed");
  }
  Msg m = std::move(s->q.front());
  s->q.pop_front();
  if (s->q.empty() && s->closed && s->max > 0) subs_.erase(sid);
  return m;
}

void Client::set_auto_reply(int64_t sid, std::shared_ptr<const std::string> body) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = subs_.find(sid);
  if (it == subs_.end()) throw std::runtime_error("nats: unknown subscription");
  it->second->auto_reply = std::move(body);
}

uint64_t Client::auto_replied(int64_t sid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = subs_.find(sid);
  return it == subs_.end() ? 0 : it->second->auto_replied;
}

int Client::pending(int64_t sid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = subs_.find(sid);
  return it == subs_.end() ? 0 : (int)it->second->q.size();
}

Msg Client::request(const std::string& subject, const std::string& data, int timeout_ms, const std::string& hdr) {
  {
    // the muxed inbox SUB must be on the wire before any request that uses it
    std::lock_guard<std::mutex> sg(resp_setup_mu_);
    if (resp_sid_ == 0) {
      int64_t sid;
      {
        std::lock_guard<std::mutex> g(mu_);
        resp_prefix_ = new_inbox() + ".";
        sid = next_sid_++;
        auto s = std::make_shared<Sub>();
        s->subject = resp_prefix_ + "*";
        subs_[sid] = s;
      }
      write_raw("SUB " + resp_prefix_ + "* " + std::to_string(sid) + "\r\n");
      std::lock_guard<std::mutex> g(mu_);
      resp_sid_ = sid;
    }
  }
  std::string token;
  auto p = std::make_shared<Pending>();
  {
    std::lock_guard<std::mutex> g(mu_);
    token = std::to_string(next_token_++);
    pending_[token] = p;
  }
  try {
    publish(subject, data, resp_prefix_ + token, hdr);
  } catch (...) {
    std::lock_guard<std::mutex> g(mu_);
    pending_.erase(token);
    throw;
  }
  std::unique_lock<std::mutex> g(mu_);
  bool ok = resp_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms < 0 ? 1 << 30 : timeout_ms),
                              [&] { return p->done || closing_; });
  pending_.erase(token);
  if (!ok) throw TimeoutError("nats: timeout");
  if (!p->done) throw ConnectionClosedError("nats: connection closed");
  if (p->msg.status == 503) throw NoRespondersError("nats: no responders available for request");
  if (p->msg.subject.empty()) throw ConnectionClosedError("nats: connection lost during request");
  return p->msg;
}

void Client::flush(int timeout_ms) {
  uint64_t target;
  {
    std::lock_guard<std::mutex> g(mu_);
    target = ++pings_sent_;
  }
  write_raw("PING\r\n");
  std::unique_lock<std::mutex> g(mu_);
  if (!pong_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms),
                         [&] { return pongs_recv_ >= target || closing_ || dead_; }))
    throw TimeoutError("nats: flush timeout");
  if (pongs_recv_ < target && dead_) throw ConnectionClosedError("nats: connection closed");
}

void Client::on_op(Op& op) {
  switch (op.kind) {
    case Op::PING:
      try { write_raw("PONG\r\n"); } catch (...) {}
      break;
    case Op::PONG: {
      std::lock_guard<std::mutex> g(mu_);
      pongs_recv_++;
      pong_cv_.notify_all();
      break;
    }
    case Op::MSG:
    case Op::HMSG: {
      in_msgs_++;
      in_bytes_ += op.payload.size();
      Msg m;
      m.subject = std::move(op.subject);
      m.reply = std::move(op.reply);
      m.data = std::move(op.payload);
      m.hdr = std::move(op.hdr);
      m.sid = std::atoll(op.sid.c_str());
      if (!m.hdr.empty()) m.status = parse_headers(m.hdr).status;
      std::shared_ptr<const std::string> auto_body;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (m.sid == resp_sid_ && resp_sid_ != 0) {
          auto tok = m.subject.substr(resp_prefix_.size());
          auto it = pending_.find(tok);
          if (it != pending_.end()) {
            it->second->msg = std::move(m);
            it->second->done = true;
            resp_cv_.notify_all();
          }
          break;
        }
        auto it = subs_.find(m.sid);
        if (it == subs_.end() || it->second->closed) break;
        auto& s = it->second;
        if (s->auto_reply && !m.reply.empty()) {
          auto_body = s->auto_reply;        // answered below, outside the subscription lock
          s->auto_replied++;
        } else {
          s->delivered++;
          s->q.push_back(std::move(m));
          s->cv.notify_one();
          if (s->max > 0 && s->delivered >= s->max) s->closed = true;   // queued messages stay drainable
        }
      }
      if (auto_body) {
        try {
          publish(m.reply, *auto_body);
        } catch (...) {       // a reply that cannot be written is the requester's timeout, as for any responder
        }
      }
      break;
    }
    case Op::INFO: {
      std::lock_guard<std::mutex> g(mu_);
      info_ = op.arg;
      break;
    }
    case Op::ERR: {
      std::lock_guard<std::mutex> g(mu_);
      last_err_ = op.arg;
      break;
    }
    default: break;
  }
}

void Client::reader() {
  char buf[256 * 1024];
  while (!closing_) {
    Parser p;
    int fd;
    std::shared_ptr<TlsConn> tls;
    {
      std::lock_guard<std::mutex> g(wmu_);
      fd = fd_;
      tls = tls_;
    }
    while (!closing_) {
      const long n = tls ? tls->read(buf, sizeof buf, closing_) : (long)::recv(fd, buf, sizeof buf, 0);
      if (n <= 0) break;
      if (!p.feed(buf, (size_t)n, [&](Op& op) { on_op(op); })) break;
    }
    connected_ = false;
    if (closing_ || !opt_.allow_reconnect) break;
    // reconnect with back-off; in-flight requests fail fast, subscriptions are re-sent by dial()
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : pending_) kv.second->done = true;
      resp_cv_.notify_all();
    }
    {
      std::lock_guard<std::mutex> g(wmu_);
      tls_.reset();
      ::close(fd_);
      fd_ = -1;
    }
    tls.reset();
    bool ok = false;
    for (int a = 0; !closing_ && (opt_.max_reconnect < 0 || a < opt_.max_reconnect); ++a) {
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min(opt_.reconnect_wait_ms * (1 << std::min(a, 4)),
                                                                     2000)));
      if (dial()) {
        ok = true;
        reconnects_++;
        break;
      }
    }
    if (!ok) break;
  }
  connected_ = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    dead_ = true;
  }
  fail_all("reader exit");
}

std::string Client::stats_json() {
  Json j = Json::O();
  j.set("in_msgs", Json::N((double)in_msgs_));
  j.set("out_msgs", Json::N((double)out_msgs_));
  j.set("in_bytes", Json::N((double)in_bytes_));
  j.set("out_bytes", Json::N((double)out_bytes_));
  j.set("reconnects", Json::N((double)reconnects_));
  j.set("connected", Json::B(connected_));
  return j.dump();
}

}  // namespace natscore
