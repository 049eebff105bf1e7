// nls-nats: native command-line front of natscore -- the `nats-server` / `nats` CLI workflow of
// the reference's README (`nats-server -js -c ...`, `nats req lmstudio.list_models '{}'`,
// `nats obj add llm-models`, `nats obj put llm-models model.gguf --name <publisher>/<model>/<file>`;
// README.md:87, :131, :183, :238, :269-276; scripts/setup_unix.sh:100-106), without Go tools.
//
//   nls-nats server [--host H] [--port 4222] [--store-dir DIR] [--max-payload BYTES]
//   nls-nats [--server URL] req <subject> <payload> [--timeout SEC]
//   nls-nats [--server URL] pub <subject> <payload>
//   nls-nats [--server URL] sub <subject> [--queue Q] [--count N]
//   nls-nats [--server URL] bench <subject> <payload> [--n N]        (request-reply RTT p50/p90/p99)
//   nls-nats [--server URL] obj add|ls <bucket>
//   nls-nats [--server URL] obj put <bucket> <file> [--name NAME] [--chunk BYTES]
//   nls-nats [--server URL] obj get <bucket> <name> [-O PATH]
//   nls-nats [--server URL] obj info|rm <bucket> <name>
#include <algorithm>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "client.h"
#include "objstore.h"
#include "server.h"

using namespace natscore;

namespace {

volatile std::sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

struct Args {
  std::vector<std::string> pos;
  std::string server, queue, name, out, host = "127.0.0.1", store_dir;
  int port = 4222, count = 0, n = 1000;
  double timeout = 120.0;
  size_t chunk = 128 * 1024, max_payload = 1 << 20;
};

int usage() {
  std::cerr << "usage: nls-nats [--server URL] {server|req|pub|sub|bench|obj} ...\n"
               "  server [--host H] [--port P] [--store-dir DIR] [--max-payload BYTES]\n"
               "  req <subject> <payload> [--timeout SEC]\n"
               "  pub <subject> <payload>\n"
               "  sub <subject> [--queue Q] [--count N]\n"
               "  bench <subject> <payload> [--n N]\n"
               "  obj add|ls <bucket> | obj put <bucket> <file> [--name NAME] [--chunk B]\n"
               "  obj get <bucket> <name> [-O PATH] | obj info|rm <bucket> <name>\n";
  return 2;
}

bool parse(int argc, char** argv, Args& a) {
  const char* env = std::getenv("NATS_URL");
  a.server = env ? env : "nats://127.0.0.1:4222";
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto val = [&](void) -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + s);
      return argv[++i];
    };
    if (s == "--server" || s == "-s") a.server = val();
    else if (s == "--queue") a.queue = val();
    else if (s == "--name") a.name = val();
    else if (s == "-O" || s == "--output") a.out = val();
    else if (s == "--host") a.host = val();
    else if (s == "--port" || s == "-p") a.port = std::stoi(val());
    else if (s == "--store-dir") a.store_dir = val();
    else if (s == "--count") a.count = std::stoi(val());
    else if (s == "--n") a.n = std::stoi(val());
    else if (s == "--timeout") a.timeout = std::stod(val());
    else if (s == "--chunk") a.chunk = std::stoul(val());
    else if (s == "--max-payload") a.max_payload = std::stoul(val());
    else a.pos.push_back(s);
  }
  return !a.pos.empty();
}

int run_server(const Args& a) {
  ServerOptions o;
  o.host = a.host;
  o.port = a.port;
  o.store_dir = a.store_dir;
  o.max_payload = a.max_payload;
  Server srv(o);
  const int port = srv.start();
  std::printf("nls-nats server listening on nats://%s:%d (jetstream%s)\n", a.host.c_str(), port,
              a.store_dir.empty() ? ", memory" : (", store " + a.store_dir).c_str());
  std::fflush(stdout);
  std::signal(SIGINT, on_signal);
  std::signal(SIGTERM, on_signal);
  while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  srv.stop();
  return 0;
}

int run_obj(Client& c, const Args& a) {
  if (a.pos.size() < 3) return usage();
  const std::string& op = a.pos[1];
  ObjectStore os(c, a.pos[2], (int)(a.timeout * 1000));
  if (op == "add") {
    std::cout << os.create("LLM model repository (.gguf)") << "\n";
  } else if (op == "ls") {
    std::cout << os.list() << "\n";
  } else if (op == "put") {
    if (a.pos.size() < 4) return usage();
    const std::string& file = a.pos[3];
    std::string name = a.name.empty() ? file.substr(file.find_last_of('/') + 1) : a.name;
    if (!os.exists()) os.create("LLM model repository (.gguf)");
    std::cout << os.put_file(name, file, a.chunk, "", [](uint64_t done, uint64_t total) {
      std::fprintf(stderr, "\r%llu / %llu bytes", (unsigned long long)done, (unsigned long long)total);
    }) << "\n";
    std::fprintf(stderr, "\n");
  } else if (op == "get") {
    if (a.pos.size() < 4) return usage();
    std::string out = a.out.empty() ? a.pos[3].substr(a.pos[3].find_last_of('/') + 1) : a.out;
    std::cout << os.get_file(a.pos[3], out, true, nullptr) << "\n";
  } else if (op == "info") {
    if (a.pos.size() < 4) return usage();
    std::cout << os.info(a.pos[3]) << "\n";
  } else if (op == "rm") {
    if (a.pos.size() < 4) return usage();
    os.remove(a.pos[3]);
    std::cout << "removed " << a.pos[3] << "\n";
  } else {
    return usage();
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  try {
    if (!parse(argc, argv, a)) return usage();
    const std::string& cmd = a.pos[0];
    if (cmd == "server") return run_server(a);
    Client c;
    ClientOptions co;
    co.name = "nls-nats";
    c.connect(a.server, co);
    const int to_ms = (int)(a.timeout * 1000);
    if (cmd == "req") {
      if (a.pos.size() < 3) return usage();
      Msg m = c.request(a.pos[1], a.pos[2], to_ms);
      std::cout << m.data << "\n";
    } else if (cmd == "pub") {
      if (a.pos.size() < 3) return usage();
      c.publish(a.pos[1], a.pos[2]);
      c.flush(to_ms);
    } else if (cmd == "sub") {
      if (a.pos.size() < 2) return usage();
      const int64_t sid = c.subscribe(a.pos[1], a.queue);
      std::signal(SIGINT, on_signal);
      int got = 0;
      while (!g_stop && (a.count <= 0 || got < a.count)) {
        try {
          Msg m = c.next_msg(sid, 200);
          std::cout << "[" << m.subject << "] " << m.data << std::endl;
          ++got;
        } catch (const TimeoutError&) {
        }
      }
    } else if (cmd == "bench") {
      if (a.pos.size() < 3) return usage();
      std::vector<double> us;
      us.reserve(a.n);
      for (int i = 0; i < a.n; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        c.request(a.pos[1], a.pos[2], to_ms);
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      }
      std::sort(us.begin(), us.end());
      auto pct = [&](double p) { return us[std::min(us.size() - 1, (size_t)(p / 100.0 * (us.size() - 1) + 0.5))]; };
      std::printf("{\"subject\":\"%s\",\"n\":%d,\"p50_ms\":%.4f,\"p90_ms\":%.4f,\"p99_ms\":%.4f}\n", a.pos[1].c_str(),
                  a.n, pct(50) / 1e3, pct(90) / 1e3, pct(99) / 1e3);
    } else if (cmd == "obj") {
      const int rc = run_obj(c, a);
      c.close();
      return rc;
    } else {
      return usage();
    }
    c.close();
  } catch (const std::exception& e) {
    std::cerr << "nls-nats: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
