// Embedded NATS server (tests, single-box benchmarks, the GPU box which has no
// nats-server binary): core pub/sub with `*`/`>` wildcards, queue groups, request-reply
// with no-responders (503) status, headers, max_payload enforcement, PING/PONG, and a
// JetStream subset sufficient for the Object Store (streams, publish acks, rollup,
// purge, direct message get incl. next_by_subj, optional file persistence) and the
// ephemeral push consumers nats.go's ObjectStore.Get uses (ordered consumer: raw chunk
// delivery to an inbox, flow control, idle heartbeats, by_start_sequence resume).
// Fault-injection hooks (drop/delay/disconnect) back the failure-detection tests.
#pragma once
#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "proto.h"
#include "util.h"

namespace natscore {

struct ServerOptions {
  std::string host = "127.0.0.1";
  int port = 0;                       // 0 = ephemeral
  size_t max_payload = 1 << 20;       // nats-server default 1 MiB
  bool jetstream = true;
  std::string store_dir;              // "" = memory only
  std::string server_name = "natscore";
  // authentication (any configured -> auth_required): a shared token, user/password pairs, and/or
  // user nkeys (public "U..." keys; the client signs the per-connection INFO nonce)
  std::string auth_token;
  std::vector<std::pair<std::string, std::string>> users;
  std::vector<std::string> nkeys;
  bool auth_required() const { return !auth_token.empty() || !users.empty() || !nkeys.empty(); }
};

class Server {
 public:
  explicit Server(ServerOptions o);
  ~Server();
  int start();
  void stop();
  int port() const { return port_; }
  bool running() const { return running_; }
  void set_fault(double drop_rate, int delay_ms);
  void disconnect_all();
  std::string stats_json();

 private:
  struct Conn;
  struct Sub;
  struct StoredMsg {
    uint64_t seq;
    std::string subject, hdr, data;
    int64_t time_ns;
  };
  struct Consumer {
    std::string stream, name, deliver, filter;
    uint64_t next_seq = 1;                 // next stream sequence to examine
    uint64_t delivered = 0;                // consumer sequence
    bool flow_control = false;
    int64_t heartbeat_ns = 0;
    int64_t created_ns = 0;
    std::atomic<bool> stop{false}, done{false};
    std::mutex m;
    std::condition_variable cv;
    std::string fc_wait;                   // reply subject of the outstanding flow-control request
    std::thread th;
  };
  struct Stream {
    std::string name;
    Json config;
    std::vector<std::string> subjects;
    std::map<uint64_t, StoredMsg> msgs;
    uint64_t last_seq = 0;
    uint64_t bytes = 0;
    int64_t created_ns = 0;
  };

  void accept_loop();
  void conn_loop(std::shared_ptr<Conn> c);
  void handle(const std::shared_ptr<Conn>& c, Op& op);
  bool authorize(const Conn& c, const Json& connect);
  void route(const std::string& subj, const std::string& reply, const std::string& hdr,
             const std::string& payload, Conn* from);
  bool js_handle(const std::string& subj, const std::string& reply, const std::string& hdr,
                 const std::string& payload);
  bool js_capture(const std::string& subj, const std::string& reply, const std::string& hdr,
                  const std::string& payload);
  void respond(const std::string& reply, const std::string& body);
  Json stream_info(const Stream& s);
  void persist(const Stream& s, char kind, const StoredMsg* m, const std::string& arg);
  void persist_config(const Stream& s);
  void load_store();
  void store_msg(Stream& s, const std::string& subj, const std::string& hdr, const std::string& data, bool log);
  void purge(Stream& s, const std::string& filter, uint64_t* n, bool log);
  std::string consumer_create(const std::string& stream, const std::string& name, const Json& req);
  Json consumer_info(const Consumer& c);
  void consumer_loop(std::shared_ptr<Consumer> c);
  bool has_interest(const std::string& subj);
  void stop_consumers(const std::string& stream);

  ServerOptions opt_;
  int lfd_ = -1;
  int port_ = 0;
  std::atomic<bool> running_{false};
  std::thread accept_th_;
  std::mutex mu_;                                 // conns + subs
  std::vector<std::shared_ptr<Conn>> conns_;
  std::vector<std::shared_ptr<Sub>> subs_;
  std::mutex js_mu_;
  std::map<std::string, std::unique_ptr<Stream>> streams_;
  std::map<std::string, std::shared_ptr<Consumer>> consumers_;   // "<stream>.<name>" -> consumer (js_mu_)
  std::vector<std::shared_ptr<Consumer>> consumer_threads_;       // every started consumer, joined (js_mu_)
  std::condition_variable js_cv_;                                 // new stream messages (js_mu_)
  std::mt19937 rng_{12345};
  std::atomic<uint64_t> next_cid_{1};
  std::atomic<double> drop_rate_{0.0};
  std::atomic<int> delay_ms_{0};
  std::atomic<uint64_t> in_msgs_{0}, out_msgs_{0}, in_bytes_{0}, out_bytes_{0};
  std::string server_id_;
};

}  // namespace natscore
