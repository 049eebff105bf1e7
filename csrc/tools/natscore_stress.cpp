// Concurrency stress of the natscore wire core, built with -fsanitize=thread or
// -fsanitize=address,undefined by tests/test_sanitizers.py (SURVEY.md §5 race detection):
// an embedded server, responders in a queue group, several client threads issuing
// request-reply concurrently over one shared connection (muxed inbox), publishers and
// wildcard subscribers, an auto-unsubscribe, a forced disconnect + reconnect, and an
// object-store round trip. Exit code 0 = every reply arrived with the right payload.
#include <atomic>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "client.h"
#include "objstore.h"
#include "server.h"

using namespace natscore;

int main() {
  ServerOptions so;
  Server srv(so);
  const int port = srv.start();
  const std::string url = "nats://127.0.0.1:" + std::to_string(port);
  std::atomic<bool> stop{false};
  std::atomic<long> served{0};

  // two responders in one queue group, each on its own connection and thread
  std::vector<std::thread> responders;
  for (int w = 0; w < 2; ++w) {
    responders.emplace_back([&, w] {
      Client c;
      c.connect(url);
      const int64_t sid = c.subscribe("svc.echo", "workers");
      c.flush(2000);
      while (!stop) {
        try {
          Msg m = c.next_msg(sid, 50);
          c.publish(m.reply, "echo:" + m.data);
          ++served;
        } catch (const TimeoutError&) {
        } catch (const std::exception&) {
        }
      }
      c.close();
    });
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(200));

  Client shared;
  shared.connect(url);
  std::atomic<int> bad{0};
  std::vector<std::thread> callers;
  for (int t = 0; t < 6; ++t) {
    callers.emplace_back([&, t] {
      for (int i = 0; i < 200; ++i) {
        const std::string p = std::to_string(t) + "-" + std::to_string(i);
        try {
          Msg m = shared.request("svc.echo", p, 5000);
          if (m.data != "echo:" + p) ++bad;
        } catch (const std::exception& e) {
          ++bad;
        }
      }
    });
  }
  // wildcard subscriber + publisher on a second connection, with an auto-unsubscribe
  std::thread pubsub([&] {
    Client c;
    c.connect(url);
    const int64_t all = c.subscribe("evt.>");
    const int64_t one = c.subscribe("evt.*.x");
    c.unsubscribe(one, 10);
    c.flush(2000);
    for (int i = 0; i < 300; ++i) c.publish("evt.a.x", std::to_string(i));
    c.flush(5000);
    int got = 0;
    try {
      while (got < 300) {
        c.next_msg(all, 2000);
        ++got;
      }
    } catch (const std::exception&) {
    }
    if (got != 300) ++bad;
    c.close();
  });
  for (auto& th : callers) th.join();
  pubsub.join();

  // disconnect everyone; the shared client reconnects and resubscribes its inbox
  srv.disconnect_all();
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  int ok_after = 0;
  for (int i = 0; i < 20; ++i) {
    try {
      Msg m = shared.request("svc.echo", "again", 2000);
      if (m.data == "echo:again") ++ok_after;
    } catch (const std::exception&) {
    }
  }
  if (ok_after == 0) ++bad;

  // object store round trip
  {
    Client c;
    c.connect(url);
    ObjectStore os(c, "stress", 5000);
    os.create("stress");
    std::string blob(300000, '\0');
    for (size_t i = 0; i < blob.size(); ++i) blob[i] = (char)(i * 131 + 7);
    os.put_bytes("a/b/c.gguf", blob, 64 * 1024);
    if (os.get_bytes("a/b/c.gguf") != blob) ++bad;
    c.close();
  }

  stop = true;
  for (auto& th : responders) th.join();
  shared.close();
  srv.stop();
  std::printf("served=%ld bad=%d ok_after_reconnect=%d\n", served.load(), bad.load(), ok_after);
  return bad.load() == 0 ? 0 : 1;
}
