// NATS client: pub/sub/queue-sub/unsub, headers, muxed-inbox request-reply (nats.go style:
// one `_INBOX.<nuid>.*` subscription, per-request token), no-responders detection,
// flush (PING/PONG), automatic reconnect with back-off and re-subscription.
// All blocking calls are safe to run with the Python GIL released.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "proto.h"
#include "tls.h"
#include "util.h"

namespace natscore {

struct Msg {
  std::string subject, reply, data, hdr;
  int64_t sid = 0;
  int status = 0;     // from the header status line (e.g. 503 = no responders)
};

struct ClientOptions {
  std::string name = "natscore";
  int connect_timeout_ms = 2000;
  bool allow_reconnect = true;
  int max_reconnect = 60;            // attempts (-1 = forever)
  int reconnect_wait_ms = 250;
  bool verbose = false;
  // authentication (CONNECT fields): token, user/password, an nkey seed ("SU..." signing the server
  // nonce) and/or a user JWT (from a .creds file, also signed with its seed)
  std::string token, user, pass, nkey_seed, jwt;
  TlsOptions tls;                    // TLS (tls.h); a tls:// URL sets tls.enable
};

class TimeoutError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};
class NoRespondersError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};
class ConnectionClosedError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Client {
 public:
  Client();
  ~Client();
  void connect(const std::string& url, ClientOptions opt = ClientOptions());
  void close();
  bool connected() const { return connected_; }

  void publish(const std::string& subject, const std::string& data, const std::string& reply = "",
               const std::string& hdr = "");
  int64_t subscribe(const std::string& subject, const std::string& queue = "");
  void unsubscribe(int64_t sid, long max_msgs = 0);
  // Blocks up to timeout_ms (<0 = forever). Throws TimeoutError / ConnectionClosedError.
  Msg next_msg(int64_t sid, int timeout_ms);
  int pending(int64_t sid);
  // Static responder: every message of `sid` that carries a reply subject is answered with `body` from the
  // reader thread -- no next_msg consumer, no Python on the path (a cached read-only reply such as the
  // list_models registry listing, kept current by its owner). A null body turns it off; messages without a
  // reply subject still queue.
  void set_auto_reply(int64_t sid, std::shared_ptr<const std::string> body);
  uint64_t auto_replied(int64_t sid);
  Msg request(const std::string& subject, const std::string& data, int timeout_ms, const std::string& hdr = "");
  void flush(int timeout_ms);
  std::string new_inbox() { return "_INBOX." + nuid_next(); }
  std::string server_info() {
    std::lock_guard<std::mutex> g(mu_);
    return info_;
  }
  size_t max_payload() const { return max_payload_; }
  std::string stats_json();
  std::string tls_cipher() {
    std::lock_guard<std::mutex> g(wmu_);
    return tls_ ? tls_->cipher() : "";
  }

 private:
  struct Sub {
    std::string subject, queue;
    std::deque<Msg> q;
    std::condition_variable cv;
    long max = 0, delivered = 0;
    bool closed = false;
    std::shared_ptr<const std::string> auto_reply;   // set_auto_reply
    uint64_t auto_replied = 0;
  };
  struct Pending {
    Msg msg;
    bool done = false;
  };
  bool dial();
  void reader();
  void on_op(Op& op);
  void write_raw(const std::string& s);
  void fail_all(const std::string& why);

  std::string host_;
  int port_ = 4222;
  ClientOptions opt_;
  int fd_ = -1;
  std::shared_ptr<TlsConn> tls_;       // set when the connection runs over TLS (guarded by wmu_)
  std::atomic<bool> connected_{false}, closing_{false};
  std::atomic<bool> dead_{false};      // the reader gave up (connection lost, no reconnect left)
  std::thread rth_;
  std::mutex wmu_;
  std::mutex mu_;
  std::map<int64_t, std::shared_ptr<Sub>> subs_;
  int64_t next_sid_ = 1;
  std::string info_;
  std::string last_err_;               // last -ERR text from the server (e.g. 'Authorization Violation')
  size_t max_payload_ = 1 << 20;
  // request/reply
  std::mutex resp_setup_mu_;
  std::string resp_prefix_;
  int64_t resp_sid_ = 0;
  std::map<std::string, std::shared_ptr<Pending>> pending_;
  uint64_t next_token_ = 1;
  std::condition_variable resp_cv_;
  // flush
  std::condition_variable pong_cv_;
  uint64_t pings_sent_ = 0, pongs_recv_ = 0;
  std::atomic<uint64_t> in_msgs_{0}, out_msgs_{0}, in_bytes_{0}, out_bytes_{0}, reconnects_{0};
};

}  // namespace natscore
