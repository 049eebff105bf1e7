#include "server.h"

#include <dirent.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <ctime>
#include <fstream>

namespace natscore {

namespace {
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
}  // namespace

std::string rfc3339(int64_t ns);   // defined in objstore.cpp

struct Server::Conn {
  int fd = -1;
  uint64_t id = 0;
  std::mutex wmu;
  std::atomic<bool> alive{true};
  bool headers = false, no_responders = false, verbose = false, echo = true;
  bool authed = false;
  std::string nonce;
  std::thread th;
  bool write(const std::string& s) {
    std::lock_guard<std::mutex> g(wmu);
    if (!alive) return false;
    if (!send_all(fd, s.data(), s.size())) {
      alive = false;
      ::shutdown(fd, SHUT_RDWR);   // unblock the reader so the connection can be reaped
      return false;
    }
    return true;
  }
};

struct Server::Sub {
  std::shared_ptr<Conn> conn;
  std::string subject, queue, sid;
  long max = 0;
  std::atomic<long> delivered{0};
};

Server::Server(ServerOptions o) : opt_(std::move(o)) { server_id_ = "N" + nuid_next(); }

Server::~Server() { stop(); }

int Server::start() {
  if (running_) return port_;
  if (!opt_.store_dir.empty()) {
    mkdir(opt_.store_dir.c_str(), 0755);
    load_store();
  }
  lfd_ = tcp_listen(opt_.host, opt_.port, &port_);
  if (lfd_ < 0) throw std::runtime_error("natscore server: cannot listen on " + opt_.host + ":" +
                                         std::to_string(opt_.port));
  running_ = true;
  accept_th_ = std::thread([this] { accept_loop(); });
  return port_;
}

void Server::stop() {
  if (!running_.exchange(false)) return;
  stop_consumers("");
  ::shutdown(lfd_, SHUT_RDWR);
  ::close(lfd_);
  if (accept_th_.joinable()) accept_th_.join();
  std::vector<std::shared_ptr<Conn>> cs;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs = conns_;
  }
  for (auto& c : cs) {
    c->alive = false;
    ::shutdown(c->fd, SHUT_RDWR);
  }
  for (auto& c : cs)
    if (c->th.joinable()) c->th.join();
  std::lock_guard<std::mutex> g(mu_);
  for (auto& c : conns_) ::close(c->fd);
  conns_.clear();
  subs_.clear();
}

void Server::set_fault(double drop_rate, int delay_ms) {
  drop_rate_ = drop_rate;
  delay_ms_ = delay_ms;
}

void Server::disconnect_all() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& c : conns_) ::shutdown(c->fd, SHUT_RDWR);
}

std::string Server::stats_json() {
  Json j = Json::O();
  size_t nc, ns;
  {
    std::lock_guard<std::mutex> g(mu_);
    nc = conns_.size();
    ns = subs_.size();
  }
  j.set("server_id", Json::S(server_id_));
  j.set("port", Json::N(port_));
  j.set("connections", Json::N((double)nc));
  j.set("subscriptions", Json::N((double)ns));
  j.set("in_msgs", Json::N((double)in_msgs_));
  j.set("out_msgs", Json::N((double)out_msgs_));
  j.set("in_bytes", Json::N((double)in_bytes_));
  j.set("out_bytes", Json::N((double)out_bytes_));
  std::lock_guard<std::mutex> g(js_mu_);
  j.set("streams", Json::N((double)streams_.size()));
  return j.dump();
}

void Server::accept_loop() {
  while (running_) {
    int fd = ::accept(lfd_, nullptr, nullptr);
    if (fd < 0) {
      if (!running_) break;
      continue;
    }
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    c->id = next_cid_++;
    std::vector<std::shared_ptr<Conn>> dead;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto it = conns_.begin(); it != conns_.end();) {
        if (!(*it)->alive) { dead.push_back(*it); it = conns_.erase(it); }
        else ++it;
      }
      conns_.push_back(c);
    }
    for (auto& d : dead) {      // reap finished connection threads
      if (d->th.joinable()) d->th.join();
      ::close(d->fd);
    }
    Json info = Json::O();
    info.set("server_id", Json::S(server_id_));
    info.set("server_name", Json::S(opt_.server_name));
    info.set("version", Json::S("2.10.12-natscore"));
    info.set("proto", Json::N(1));
    info.set("host", Json::S(opt_.host));
    info.set("port", Json::N(port_));
    info.set("headers", Json::B(true));
    info.set("max_payload", Json::N((double)opt_.max_payload));
    info.set("jetstream", Json::B(opt_.jetstream));
    info.set("client_id", Json::N((double)c->id));
    if (opt_.auth_required()) {
      info.set("auth_required", Json::B(true));
      c->nonce = random_b64url(11);
      info.set("nonce", Json::S(c->nonce));
    } else {
      c->authed = true;
    }
    c->write("INFO " + info.dump() + "\r\n");
    c->th = std::thread([this, c] { conn_loop(c); });
  }
}

void Server::conn_loop(std::shared_ptr<Conn> c) {
  Parser p(opt_.max_payload);
  char buf[256 * 1024];
  while (c->alive && running_) {
    ssize_t n = ::recv(c->fd, buf, sizeof buf, 0);
    if (n <= 0) break;
    bool ok = p.feed(buf, (size_t)n, [&](Op& op) { handle(c, op); });
    if (!ok) {
      c->write("-ERR '" + p.error() + "'\r\n");
      break;
    }
  }
  c->alive = false;
  ::shutdown(c->fd, SHUT_RDWR);
  std::lock_guard<std::mutex> g(mu_);
  subs_.erase(std::remove_if(subs_.begin(), subs_.end(), [&](const std::shared_ptr<Sub>& s) { return s->conn == c; }),
              subs_.end());
  // the Conn object stays in conns_ until stop() (its thread handle must be joined there)
}

bool Server::authorize(const Conn& c, const Json& j) {
  if (!opt_.auth_required()) return true;
  if (!opt_.auth_token.empty() && ct_equal(j.str("auth_token"), opt_.auth_token)) return true;
  const std::string user = j.str("user");
  if (!user.empty())
    for (auto& up : opt_.users)
      if (up.first == user && ct_equal(j.str("pass"), up.second)) return true;
  const std::string nk = j.str("nkey");
  if (!nk.empty() && std::find(opt_.nkeys.begin(), opt_.nkeys.end(), nk) != opt_.nkeys.end()) {
    std::string sig;
    std::string b = j.str("sig");
    while (b.size() % 4) b += '=';
    for (char& ch : b) {                      // base64url -> base64
      if (ch == '-') ch = '+';
      else if (ch == '_') ch = '/';
    }
    try {
      sig = b64decode(b);
    } catch (...) {
      return false;
    }
    return nkey_verify(nk, c.nonce, sig);
  }
  return false;
}

void Server::handle(const std::shared_ptr<Conn>& c, Op& op) {
  if (!c->authed && op.kind != Op::CONNECT && op.kind != Op::PING && op.kind != Op::PONG) {
    c->write("-ERR 'Authorization Violation'\r\n");
    c->alive = false;
    ::shutdown(c->fd, SHUT_RDWR);
    return;
  }
  switch (op.kind) {
    case Op::CONNECT: {
      try {
        Json j = Json::parse(op.arg);
        c->headers = j.boolean("headers", false);
        c->no_responders = j.boolean("no_responders", false);
        c->verbose = j.boolean("verbose", false);
        c->echo = j.boolean("echo", true);
        if (!c->authed) {
          if (!authorize(*c, j)) {
            c->write("-ERR 'Authorization Violation'\r\n");
            c->alive = false;
            ::shutdown(c->fd, SHUT_RDWR);
            return;
          }
          c->authed = true;
        }
      } catch (...) {
        c->write("-ERR 'Invalid CONNECT'\r\n");
        return;
      }
      if (c->verbose) c->write("+OK\r\n");
      break;
    }
    case Op::PING: c->write("PONG\r\n"); break;
    case Op::PONG: break;
    case Op::SUB: {
      if (!valid_subject(op.subject, true)) {
        c->write("-ERR 'Invalid Subject'\r\n");
        return;
      }
      auto s = std::make_shared<Sub>();
      s->conn = c;
      s->subject = op.subject;
      s->queue = op.queue;
      s->sid = op.sid;
      std::lock_guard<std::mutex> g(mu_);
      subs_.push_back(s);
      if (c->verbose) c->write("+OK\r\n");
      break;
    }
    case Op::UNSUB: {
      std::lock_guard<std::mutex> g(mu_);
      for (auto it = subs_.begin(); it != subs_.end(); ++it) {
        if ((*it)->conn == c && (*it)->sid == op.sid) {
          if (op.max_msgs > 0 && (*it)->delivered < op.max_msgs) (*it)->max = op.max_msgs;
          else subs_.erase(it);
          break;
        }
      }
      if (c->verbose) c->write("+OK\r\n");
      break;
    }
    case Op::PUB:
    case Op::HPUB: {
      if (!valid_subject(op.subject, false)) {
        c->write("-ERR 'Invalid Publish Subject'\r\n");
        return;
      }
      in_msgs_++;
      in_bytes_ += op.payload.size() + op.hdr.size();
      if (c->verbose) c->write("+OK\r\n");
      const double dr = drop_rate_;
      if (dr > 0) {
        std::uniform_real_distribution<double> u(0, 1);
        double x;
        {
          std::lock_guard<std::mutex> g(mu_);
          x = u(rng_);
        }
        if (x < dr) return;   // fault injection: message lost in transit
      }
      const int dl = delay_ms_;
      if (dl > 0) std::this_thread::sleep_for(std::chrono::milliseconds(dl));
      route(op.subject, op.reply, op.hdr, op.payload, c.get());
      break;
    }
    default: break;
  }
}

void Server::respond(const std::string& reply, const std::string& body) {
  if (!reply.empty()) route(reply, "", "", body, nullptr);
}

void Server::route(const std::string& subj, const std::string& reply, const std::string& hdr,
                   const std::string& payload, Conn* from) {
  bool handled = false;
  if (opt_.jetstream) {
    if (subj.rfind("$JS.API.", 0) == 0) {
      handled = js_handle(subj, reply, hdr, payload);
    } else if (subj.rfind("$JS.FC.", 0) == 0) {
      // a consumer's flow-control request answered by its subscriber: release the next window
      std::vector<std::shared_ptr<Consumer>> cs;
      {
        std::lock_guard<std::mutex> g(js_mu_);
        for (auto& kv : consumers_) cs.push_back(kv.second);
      }
      for (auto& c : cs) {
        std::lock_guard<std::mutex> g(c->m);
        if (c->fc_wait == subj) {
          c->fc_wait.clear();
          c->cv.notify_all();
        }
      }
      return;
    } else {
      handled = js_capture(subj, reply, hdr, payload);
    }
  }
  std::vector<std::shared_ptr<Sub>> targets;
  {
    std::lock_guard<std::mutex> g(mu_);
    std::map<std::string, std::vector<std::shared_ptr<Sub>>> groups;
    for (auto& s : subs_) {
      if (!s->conn->alive || !subject_matches(s->subject, subj)) continue;
      if (from && !s->conn->echo && s->conn.get() == from) continue;
      if (s->queue.empty()) targets.push_back(s);
      else groups[s->queue].push_back(s);
    }
    for (auto& kv : groups) {
      std::uniform_int_distribution<size_t> d(0, kv.second.size() - 1);
      targets.push_back(kv.second[d(rng_)]);
    }
  }
  for (auto& s : targets) {
    std::string m;
    const bool h = !hdr.empty() && s->conn->headers;
    const size_t total = (h ? hdr.size() : 0) + payload.size();
    m.reserve(total + subj.size() + reply.size() + 64);
    if (h) {
      m = "HMSG " + subj + " " + s->sid + (reply.empty() ? "" : " " + reply) + " " + std::to_string(hdr.size()) +
          " " + std::to_string(total) + "\r\n";
      m += hdr;
    } else {
      m = "MSG " + subj + " " + s->sid + (reply.empty() ? "" : " " + reply) + " " + std::to_string(payload.size()) +
          "\r\n";
    }
    m += payload;
    m += "\r\n";
    if (s->conn->write(m)) {
      out_msgs_++;
      out_bytes_ += total;
    }
    long d = ++s->delivered;
    if (s->max > 0 && d >= s->max) {
      std::lock_guard<std::mutex> g(mu_);
      subs_.erase(std::remove(subs_.begin(), subs_.end(), s), subs_.end());
    }
  }
  if (targets.empty() && !handled && !reply.empty() && from && from->headers && from->no_responders)
    route(reply, "", "NATS/1.0 503\r\n\r\n", "", nullptr);
}

// ============================ JetStream subset ================================

Json Server::stream_info(const Stream& s) {
  Json j = Json::O();
  j.set("config", s.config);
  j.set("created", Json::S(rfc3339(s.created_ns)));
  Json st = Json::O();
  st.set("messages", Json::N((double)s.msgs.size()));
  st.set("bytes", Json::N((double)s.bytes));
  st.set("first_seq", Json::N(s.msgs.empty() ? (double)(s.last_seq + 1) : (double)s.msgs.begin()->first));
  st.set("last_seq", Json::N((double)s.last_seq));
  uint64_t nc = 0;
  for (auto& kv : consumers_)
    if (kv.second->stream == s.name) ++nc;
  st.set("consumer_count", Json::N((double)nc));
  j.set("state", st);
  return j;
}

static std::string js_error(int code, int err_code, const std::string& desc, const std::string& type) {
  Json j = Json::O();
  j.set("type", Json::S(type));
  Json e = Json::O();
  e.set("code", Json::N(code));
  e.set("err_code", Json::N(err_code));
  e.set("description", Json::S(desc));
  j.set("error", e);
  return j.dump();
}

void Server::store_msg(Stream& s, const std::string& subj, const std::string& hdr, const std::string& data,
                       bool log) {
  StoredMsg m{++s.last_seq, subj, hdr, data, now_ns()};
  s.bytes += subj.size() + hdr.size() + data.size();
  auto it = s.msgs.emplace(m.seq, std::move(m)).first;
  if (log) persist(s, 'M', &it->second, "");
}

void Server::purge(Stream& s, const std::string& filter, uint64_t* n, bool log) {
  uint64_t cnt = 0;
  for (auto it = s.msgs.begin(); it != s.msgs.end();) {
    if (filter.empty() || subject_matches(filter, it->second.subject)) {
      s.bytes -= it->second.subject.size() + it->second.hdr.size() + it->second.data.size();
      it = s.msgs.erase(it);
      ++cnt;
    } else {
      ++it;
    }
  }
  if (n) *n = cnt;
  if (log) persist(s, 'P', nullptr, filter);
}

bool Server::js_capture(const std::string& subj, const std::string& reply, const std::string& hdr,
                        const std::string& payload) {
  std::string ack;
  {
    std::lock_guard<std::mutex> g(js_mu_);
    for (auto& kv : streams_) {
      Stream& s = *kv.second;
      bool match = false;
      for (auto& p : s.subjects)
        if (subject_matches(p, subj)) { match = true; break; }
      if (!match) continue;
      if (!hdr.empty()) {
        Headers h = parse_headers(hdr);
        if (h.get("Nats-Rollup") == "sub") {
          // rollup replaces every earlier message on this exact subject
          for (auto it = s.msgs.begin(); it != s.msgs.end();) {
            if (it->second.subject == subj) {
              s.bytes -= it->second.subject.size() + it->second.hdr.size() + it->second.data.size();
              it = s.msgs.erase(it);
            } else {
              ++it;
            }
          }
          persist(s, 'P', nullptr, subj);
        }
      }
      store_msg(s, subj, hdr, payload, true);
      js_cv_.notify_all();
      Json a = Json::O();
      a.set("stream", Json::S(s.name));
      a.set("seq", Json::N((double)s.last_seq));
      ack = a.dump();
      break;
    }
  }
  if (ack.empty()) return false;
  respond(reply, ack);
  return true;
}

bool Server::js_handle(const std::string& subj, const std::string& reply, const std::string& hdr,
                       const std::string& payload) {
  (void)hdr;
  const std::string api = subj.substr(8);   // after "$JS.API."
  auto tail = [&](const std::string& pre) -> std::string {
    return api.rfind(pre, 0) == 0 ? api.substr(pre.size()) : std::string();
  };
  Json req;
  if (!payload.empty()) {
    try {
      req = Json::parse(payload);
    } catch (...) {
      respond(reply, js_error(400, 10025, "bad request", "io.nats.jetstream.api.v1.error"));
      return true;
    }
  }
  std::string out;
  {
    std::lock_guard<std::mutex> g(js_mu_);
    if (api == "INFO") {
      Json j = Json::O();
      j.set("type", Json::S("io.nats.jetstream.api.v1.account_info_response"));
      uint64_t bytes = 0;
      for (auto& kv : streams_) bytes += kv.second->bytes;
      j.set("memory", Json::N(opt_.store_dir.empty() ? (double)bytes : 0));
      j.set("storage", Json::N(opt_.store_dir.empty() ? 0 : (double)bytes));
      j.set("streams", Json::N((double)streams_.size()));
      j.set("consumers", Json::N(0));
      out = j.dump();
    } else if (!tail("STREAM.CREATE.").empty() || !tail("STREAM.UPDATE.").empty()) {
      const bool create = !tail("STREAM.CREATE.").empty();
      std::string name = create ? tail("STREAM.CREATE.") : tail("STREAM.UPDATE.");
      if (req.str("name", name) != name) {
        out = js_error(400, 10058, "stream name in subject does not match request",
                       "io.nats.jetstream.api.v1.stream_create_response");
      } else {
        auto it = streams_.find(name);
        bool did = false;
        if (it == streams_.end()) {
          if (!create) {
            out = js_error(404, 10059, "stream not found", "io.nats.jetstream.api.v1.stream_update_response");
          } else {
            auto s = std::make_unique<Stream>();
            s->name = name;
            s->created_ns = now_ns();
            it = streams_.emplace(name, std::move(s)).first;
            did = true;
          }
        }
        if (out.empty()) {
          Stream& s = *it->second;
          Json cfg = req.t == Json::OBJ ? req : Json::O();
          cfg.set("name", Json::S(name));
          s.subjects.clear();
          if (auto* sj = cfg.get("subjects"))
            for (auto& v : sj->a)
              if (v.t == Json::STR) s.subjects.push_back(v.s);
          if (s.subjects.empty()) {
            s.subjects.push_back(name);
            Json arr = Json::A();
            arr.a.push_back(Json::S(name));
            cfg.set("subjects", arr);
          }
          s.config = cfg;
          persist_config(s);
          Json j = stream_info(s);
          j.set("type", Json::S(create ? "io.nats.jetstream.api.v1.stream_create_response"
                                       : "io.nats.jetstream.api.v1.stream_update_response"));
          j.set("did_create", Json::B(did));
          out = j.dump();
        }
      }
    } else if (!tail("STREAM.INFO.").empty()) {
      auto it = streams_.find(tail("STREAM.INFO."));
      if (it == streams_.end()) {
        out = js_error(404, 10059, "stream not found", "io.nats.jetstream.api.v1.stream_info_response");
      } else {
        Json j = stream_info(*it->second);
        j.set("type", Json::S("io.nats.jetstream.api.v1.stream_info_response"));
        out = j.dump();
      }
    } else if (api == "STREAM.NAMES" || api == "STREAM.LIST") {
      Json j = Json::O();
      j.set("type", Json::S(api == "STREAM.NAMES" ? "io.nats.jetstream.api.v1.stream_names_response"
                                                  : "io.nats.jetstream.api.v1.stream_list_response"));
      Json arr = Json::A();
      for (auto& kv : streams_) arr.a.push_back(api == "STREAM.NAMES" ? Json::S(kv.first) : stream_info(*kv.second));
      j.set("total", Json::N((double)streams_.size()));
      j.set("offset", Json::N(0));
      j.set("limit", Json::N(1024));
      j.set("streams", arr);
      out = j.dump();
    } else if (!tail("STREAM.DELETE.").empty()) {
      auto it = streams_.find(tail("STREAM.DELETE."));
      if (it == streams_.end()) {
        out = js_error(404, 10059, "stream not found", "io.nats.jetstream.api.v1.stream_delete_response");
      } else {
        persist(*it->second, 'X', nullptr, "");
        streams_.erase(it);
        out = "{\"type\":\"io.nats.jetstream.api.v1.stream_delete_response\",\"success\":true}";
      }
    } else if (!tail("STREAM.PURGE.").empty()) {
      auto it = streams_.find(tail("STREAM.PURGE."));
      if (it == streams_.end()) {
        out = js_error(404, 10059, "stream not found", "io.nats.jetstream.api.v1.stream_purge_response");
      } else {
        uint64_t n = 0;
        purge(*it->second, req.str("filter"), &n, true);
        out = "{\"type\":\"io.nats.jetstream.api.v1.stream_purge_response\",\"success\":true,\"purged\":" +
              std::to_string(n) + "}";
      }
    } else if (!tail("STREAM.MSG.GET.").empty()) {
      auto it = streams_.find(tail("STREAM.MSG.GET."));
      const std::string T = "io.nats.jetstream.api.v1.stream_msg_get_response";
      if (it == streams_.end()) {
        out = js_error(404, 10059, "stream not found", T);
      } else {
        Stream& s = *it->second;
        const StoredMsg* found = nullptr;
        const std::string last = req.str("last_by_subj"), next = req.str("next_by_subj");
        const uint64_t seq = (uint64_t)req.num("seq", 0);
        if (!last.empty()) {
          for (auto r = s.msgs.rbegin(); r != s.msgs.rend(); ++r)
            if (subject_matches(last, r->second.subject)) { found = &r->second; break; }
        } else if (!next.empty()) {
          for (auto f = s.msgs.lower_bound(seq); f != s.msgs.end(); ++f)
            if (subject_matches(next, f->second.subject)) { found = &f->second; break; }
        } else {
          auto f = s.msgs.find(seq);
          if (f != s.msgs.end()) found = &f->second;
        }
        if (!found) {
          out = js_error(404, 10037, "no message found", T);
        } else {
          Json m = Json::O();
          m.set("subject", Json::S(found->subject));
          m.set("seq", Json::N((double)found->seq));
          if (!found->hdr.empty()) m.set("hdrs", Json::S(b64encode(found->hdr)));
          m.set("data", Json::S(b64encode(found->data)));
          m.set("time", Json::S(rfc3339(found->time_ns)));
          Json j = Json::O();
          j.set("type", Json::S(T));
          j.set("message", m);
          out = j.dump();
        }
      }
    } else if (!tail("STREAM.MSG.DELETE.").empty()) {
      auto it = streams_.find(tail("STREAM.MSG.DELETE."));
      if (it == streams_.end()) {
        out = js_error(404, 10059, "stream not found", "io.nats.jetstream.api.v1.stream_msg_delete_response");
      } else {
        Stream& s = *it->second;
        uint64_t seq = (uint64_t)req.num("seq", 0);
        auto f = s.msgs.find(seq);
        if (f == s.msgs.end()) {
          out = js_error(400, 10057, "no message found", "io.nats.jetstream.api.v1.stream_msg_delete_response");
        } else {
          s.bytes -= f->second.subject.size() + f->second.hdr.size() + f->second.data.size();
          s.msgs.erase(f);
          persist(s, 'D', nullptr, std::to_string(seq));
          out = "{\"type\":\"io.nats.jetstream.api.v1.stream_msg_delete_response\",\"success\":true}";
        }
      }
    } else if (!tail("CONSUMER.CREATE.").empty() || !tail("CONSUMER.DURABLE.CREATE.").empty()) {
      // CONSUMER.CREATE.<stream>[.<name>[.<filter>]] (nats.go >= 2.9) | DURABLE.CREATE.<stream>.<name>
      std::string rest = !tail("CONSUMER.CREATE.").empty() ? tail("CONSUMER.CREATE.") : tail("CONSUMER.DURABLE.CREATE.");
      const size_t d1 = rest.find('.');
      const std::string sname = rest.substr(0, d1);
      std::string cname;
      if (d1 != std::string::npos) {
        const std::string r2 = rest.substr(d1 + 1);
        cname = r2.substr(0, r2.find('.'));
      }
      out = consumer_create(sname, cname, req);
    } else if (!tail("CONSUMER.DELETE.").empty() || !tail("CONSUMER.INFO.").empty()) {
      const bool del = !tail("CONSUMER.DELETE.").empty();
      const std::string key = del ? tail("CONSUMER.DELETE.") : tail("CONSUMER.INFO.");
      auto it = consumers_.find(key);
      if (it == consumers_.end()) {
        out = js_error(404, 10014, "consumer not found", del ? "io.nats.jetstream.api.v1.consumer_delete_response"
                                                            : "io.nats.jetstream.api.v1.consumer_info_response");
      } else if (del) {
        it->second->stop = true;
        it->second->cv.notify_all();
        js_cv_.notify_all();
        out = "{\"type\":\"io.nats.jetstream.api.v1.consumer_delete_response\",\"success\":true}";
      } else {
        Json j = consumer_info(*it->second);
        j.set("type", Json::S("io.nats.jetstream.api.v1.consumer_info_response"));
        out = j.dump();
      }
    } else {
      out = js_error(501, 10000, "not supported by the embedded server: " + api, "io.nats.jetstream.api.v1.error");
    }
  }
  respond(reply, out);
  return true;
}

// ---- push consumers (caller holds js_mu_ for create/info) ---------------------------------------
Json Server::consumer_info(const Consumer& c) {
  Json j = Json::O();
  j.set("stream_name", Json::S(c.stream));
  j.set("name", Json::S(c.name));
  j.set("created", Json::S(rfc3339(c.created_ns)));
  Json cfg = Json::O();
  cfg.set("deliver_subject", Json::S(c.deliver));
  if (!c.filter.empty()) cfg.set("filter_subject", Json::S(c.filter));
  cfg.set("ack_policy", Json::S("none"));
  cfg.set("flow_control", Json::B(c.flow_control));
  if (c.heartbeat_ns) cfg.set("idle_heartbeat", Json::N((double)c.heartbeat_ns));
  j.set("config", cfg);
  Json dl = Json::O();
  dl.set("consumer_seq", Json::N((double)c.delivered));
  dl.set("stream_seq", Json::N((double)(c.next_seq ? c.next_seq - 1 : 0)));
  j.set("delivered", dl);
  j.set("num_pending", Json::N(0));
  j.set("push_bound", Json::B(true));
  return j;
}

std::string Server::consumer_create(const std::string& sname, const std::string& cname, const Json& req) {
  const std::string type = "io.nats.jetstream.api.v1.consumer_create_response";
  auto sit = streams_.find(sname);
  if (sit == streams_.end()) return js_error(404, 10059, "stream not found", type);
  const Json* cfg = req.get("config");
  if (!cfg) return js_error(400, 10025, "consumer config required", type);
  auto c = std::make_shared<Consumer>();
  c->stream = sname;
  c->name = !cname.empty() ? cname : (!cfg->str("name").empty() ? cfg->str("name")
                                                                 : (!cfg->str("durable_name").empty() ? cfg->str("durable_name")
                                                                                                      : nuid_next()));
  c->deliver = cfg->str("deliver_subject");
  if (c->deliver.empty()) return js_error(400, 10137, "pull consumers are not supported by the embedded server", type);
  c->filter = cfg->str("filter_subject");
  if (c->filter.empty()) {
    const Json* fs = cfg->get("filter_subjects");
    if (fs && fs->a.size() == 1) c->filter = fs->a[0].s;
    else if (fs && fs->a.size() > 1) return js_error(400, 10136, "multiple filter subjects are not supported", type);
  }
  const std::string ack = cfg->str("ack_policy");
  if (!ack.empty() && ack != "none") return js_error(400, 10138, "only ack_policy none is supported", type);
  Stream& s = *sit->second;
  const std::string pol = cfg->str("deliver_policy");
  if (pol.empty() || pol == "all") c->next_seq = s.msgs.empty() ? s.last_seq + 1 : s.msgs.begin()->first;
  else if (pol == "by_start_sequence") c->next_seq = std::max<uint64_t>(1, (uint64_t)cfg->num("opt_start_seq", 1));
  else if (pol == "new") c->next_seq = s.last_seq + 1;
  else if (pol == "last") c->next_seq = s.msgs.empty() ? s.last_seq + 1 : s.msgs.rbegin()->first;
  else return js_error(400, 10025, "deliver_policy " + pol + " is not supported", type);
  c->flow_control = cfg->boolean("flow_control", false);
  c->heartbeat_ns = (int64_t)cfg->num("idle_heartbeat", 0);
  c->created_ns = now_ns();
  const std::string key = sname + "." + c->name;
  auto old = consumers_.find(key);
  if (old != consumers_.end()) {
    old->second->stop = true;
    old->second->cv.notify_all();
  }
  consumers_[key] = c;
  for (auto it = consumer_threads_.begin(); it != consumer_threads_.end();) {   // reap finished deliveries
    if ((*it)->done) {
      if ((*it)->th.joinable()) (*it)->th.join();
      it = consumer_threads_.erase(it);
    } else {
      ++it;
    }
  }
  c->th = std::thread([this, c] { consumer_loop(c); });
  consumer_threads_.push_back(c);
  Json j = consumer_info(*c);
  j.set("type", Json::S(type));
  return j.dump();
}

bool Server::has_interest(const std::string& subj) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& s : subs_)
    if (s->conn->alive && subject_matches(s->subject, subj)) return true;
  return false;
}

void Server::stop_consumers(const std::string& stream) {
  std::vector<std::shared_ptr<Consumer>> join;
  {
    std::lock_guard<std::mutex> g(js_mu_);
    for (auto it = consumers_.begin(); it != consumers_.end();) {
      if (stream.empty() || it->second->stream == stream) it = consumers_.erase(it);
      else ++it;
    }
    for (auto it = consumer_threads_.begin(); it != consumer_threads_.end();) {
      if (stream.empty() || (*it)->stream == stream) {
        (*it)->stop = true;
        (*it)->cv.notify_all();
        join.push_back(*it);
        it = consumer_threads_.erase(it);
      } else {
        ++it;
      }
    }
    js_cv_.notify_all();
  }
  for (auto& c : join)
    if (c->th.joinable()) c->th.join();
}

// Delivery: every stored message on the filter, in stream order, raw payload + original headers, reply
// subject "$JS.ACK.<stream>.<consumer>.<delivered>.<stream seq>.<consumer seq>.<ts>.<pending>" (the
// metadata nats.go ordered consumers check for gaps). Flow control: after each FC_WINDOW bytes a
// "100 FlowControl Request" status message is sent and delivery waits until the subscriber answers it,
// so a slow consumer (disk-bound pull) never makes the server queue an unbounded amount of data. Idle
// consumers send "100 Idle Heartbeat"; a consumer whose deliver subject lost all interest ends itself.
void Server::consumer_loop(std::shared_ptr<Consumer> c) {
  constexpr uint64_t FC_WINDOW = 32ull << 20;
  uint64_t since_fc = 0, fc_n = 0;
  auto last_activity = std::chrono::steady_clock::now();
  auto last_interest = last_activity;
  while (!c->stop && running_) {
    StoredMsg m;
    bool have = false;
    uint64_t pending = 0;
    {
      std::unique_lock<std::mutex> g(js_mu_);
      auto sit = streams_.find(c->stream);
      if (sit == streams_.end()) break;
      Stream& s = *sit->second;
      for (auto it = s.msgs.lower_bound(c->next_seq); it != s.msgs.end(); ++it) {
        if (!c->filter.empty() && !subject_matches(c->filter, it->second.subject)) continue;
        m = it->second;
        have = true;
        break;
      }
      if (have) {
        c->next_seq = m.seq + 1;
        pending = s.last_seq > m.seq ? s.last_seq - m.seq : 0;   // upper bound (ignores the filter)
      } else {
        c->next_seq = s.last_seq + 1;
        js_cv_.wait_for(g, std::chrono::milliseconds(200));
      }
    }
    const auto now = std::chrono::steady_clock::now();
    if (!have) {
      if (c->heartbeat_ns > 0 && now - last_activity >= std::chrono::nanoseconds(c->heartbeat_ns)) {
        route(c->deliver, "", "NATS/1.0 100 Idle Heartbeat\r\nNats-Last-Consumer: " + std::to_string(c->delivered) +
                                  "\r\nNats-Last-Stream: " + std::to_string(c->next_seq - 1) + "\r\n\r\n",
              "", nullptr);
        last_activity = now;
      }
      if (has_interest(c->deliver)) last_interest = now;
      else if (now - last_interest > std::chrono::seconds(5)) break;    // ephemeral consumer abandoned
      continue;
    }
    ++c->delivered;
    const std::string ack = "$JS.ACK." + c->stream + "." + c->name + ".1." + std::to_string(m.seq) + "." +
                            std::to_string(c->delivered) + "." + std::to_string(m.time_ns) + "." +
                            std::to_string(pending);
    route(c->deliver, ack, m.hdr, m.data, nullptr);
    last_activity = now;
    since_fc += m.data.size() + m.hdr.size();
    if (c->flow_control && since_fc >= FC_WINDOW) {
      since_fc = 0;
      const std::string fc = "$JS.FC." + c->stream + "." + c->name + "." + std::to_string(++fc_n);
      {
        std::lock_guard<std::mutex> g(c->m);
        c->fc_wait = fc;
      }
      route(c->deliver, fc, "NATS/1.0 100 FlowControl Request\r\n\r\n", "", nullptr);
      std::unique_lock<std::mutex> g(c->m);
      for (int waited = 0; !c->fc_wait.empty() && !c->stop && running_; ++waited) {
        c->cv.wait_for(g, std::chrono::milliseconds(100));
        if (waited % 50 == 49) {                       // every 5 s: give up if nobody listens any more
          g.unlock();
          const bool alive = has_interest(c->deliver);
          g.lock();
          if (!alive) {
            c->stop = true;
            break;
          }
        }
      }
    }
  }
  std::lock_guard<std::mutex> g(js_mu_);
  auto it = consumers_.find(c->stream + "." + c->name);
  if (it != consumers_.end() && it->second == c) consumers_.erase(it);
  c->done = true;
}

// ---- persistence: <store_dir>/<stream>.cfg (JSON) + <stream>.log (binary records) ----
static void put_u64(std::string& b, uint64_t v) { b.append((const char*)&v, 8); }
static void put_str(std::string& b, const std::string& s) {
  put_u64(b, s.size());
  b += s;
}

void Server::persist_config(const Stream& s) {
  if (opt_.store_dir.empty()) return;
  std::ofstream f(opt_.store_dir + "/" + s.name + ".cfg", std::ios::trunc);
  f << s.config.dump();
}

void Server::persist(const Stream& s, char kind, const StoredMsg* m, const std::string& arg) {
  if (opt_.store_dir.empty()) return;
  const std::string base = opt_.store_dir + "/" + s.name;
  if (kind == 'X') {
    ::unlink((base + ".cfg").c_str());
    ::unlink((base + ".log").c_str());
    return;
  }
  std::string rec(1, kind);
  if (m) {
    put_u64(rec, m->seq);
    put_u64(rec, (uint64_t)m->time_ns);
    put_str(rec, m->subject);
    put_str(rec, m->hdr);
    put_str(rec, m->data);
  } else {
    put_str(rec, arg);
  }
  FILE* f = fopen((base + ".log").c_str(), "ab");
  if (f) {
    fwrite(rec.data(), 1, rec.size(), f);
    fclose(f);
  }
}

void Server::load_store() {
  std::string cmd_dir = opt_.store_dir;
  // enumerate *.cfg files
  std::vector<std::string> names;
  if (auto* d = opendir(cmd_dir.c_str())) {
    while (auto* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.size() > 4 && n.substr(n.size() - 4) == ".cfg") names.push_back(n.substr(0, n.size() - 4));
    }
    closedir(d);
  }
  for (auto& name : names) {
    std::ifstream cf(cmd_dir + "/" + name + ".cfg");
    std::string txt((std::istreambuf_iterator<char>(cf)), std::istreambuf_iterator<char>());
    auto s = std::make_unique<Stream>();
    s->name = name;
    s->created_ns = now_ns();
    try {
      s->config = Json::parse(txt);
    } catch (...) {
      continue;
    }
    if (auto* sj = s->config.get("subjects"))
      for (auto& v : sj->a) s->subjects.push_back(v.s);
    FILE* f = fopen((cmd_dir + "/" + name + ".log").c_str(), "rb");
    if (f) {
      auto rd64 = [&](uint64_t& v) { return fread(&v, 8, 1, f) == 1; };
      auto rds = [&](std::string& out) {
        uint64_t n;
        if (!rd64(n)) return false;
        out.resize(n);
        return n == 0 || fread(&out[0], 1, n, f) == n;
      };
      int kind;
      while ((kind = fgetc(f)) != EOF) {
        if (kind == 'M') {
          StoredMsg m;
          uint64_t t;
          if (!rd64(m.seq) || !rd64(t) || !rds(m.subject) || !rds(m.hdr) || !rds(m.data)) break;
          m.time_ns = (int64_t)t;
          s->last_seq = std::max(s->last_seq, m.seq);
          s->bytes += m.subject.size() + m.hdr.size() + m.data.size();
          s->msgs.emplace(m.seq, std::move(m));
        } else if (kind == 'P') {
          std::string filt;
          if (!rds(filt)) break;
          purge(*s, filt, nullptr, false);
        } else if (kind == 'D') {
          std::string a;
          if (!rds(a)) break;
          auto it = s->msgs.find(std::stoull(a));
          if (it != s->msgs.end()) {
            s->bytes -= it->second.subject.size() + it->second.hdr.size() + it->second.data.size();
            s->msgs.erase(it);
          }
        } else {
          break;
        }
      }
      fclose(f);
    }
    streams_.emplace(name, std::move(s));
  }
}

}  // namespace natscore
