// pybind11 bindings of the natscore wire core (module nats_llm_studio_amd.natsio._natscore).
// Every call that can block (socket I/O, waits) releases the GIL.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>

#include "client.h"
#include "objstore.h"
#include "server.h"

namespace py = pybind11;
using namespace natscore;

namespace {

py::bytes to_bytes(const std::string& s) { return py::bytes(s); }

struct PyMsg {
  std::string subject, reply;
  py::bytes data, hdr;
  int64_t sid;
  int status;
};

PyMsg wrap(Msg&& m) {
  return PyMsg{m.subject, m.reply, py::bytes(m.data), py::bytes(m.hdr), m.sid, m.status};
}

// bench helper: N sequential requests measured in C++ (microseconds per request)
std::vector<double> bench_requests(Client& c, const std::string& subj, const std::string& payload, int n,
                                   int timeout_ms) {
  std::vector<double> out;
  out.reserve(n);
  for (int k = 0; k < n; ++k) {
    auto t0 = std::chrono::steady_clock::now();
    c.request(subj, payload, timeout_ms);
    auto t1 = std::chrono::steady_clock::now();
    out.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_natscore, m) {
  m.doc() = "natscore: native NATS client, embedded server and JetStream object store";

  static py::exception<TimeoutError> exc_timeout(m, "TimeoutError", PyExc_TimeoutError);
  static py::exception<NoRespondersError> exc_nr(m, "NoRespondersError", PyExc_RuntimeError);
  static py::exception<ConnectionClosedError> exc_cc(m, "ConnectionClosedError", PyExc_ConnectionError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const TimeoutError& e) {
      py::set_error(exc_timeout, e.what());
    } catch (const NoRespondersError& e) {
      py::set_error(exc_nr, e.what());
    } catch (const ConnectionClosedError& e) {
      py::set_error(exc_cc, e.what());
    }
  });

  py::class_<PyMsg>(m, "Msg")
      .def_readonly("subject", &PyMsg::subject)
      .def_readonly("reply", &PyMsg::reply)
      .def_readonly("data", &PyMsg::data)
      .def_readonly("raw_headers", &PyMsg::hdr)
      .def_readonly("sid", &PyMsg::sid)
      .def_readonly("status", &PyMsg::status);

  py::class_<Server>(m, "Server")
      .def(py::init([](const std::string& host, int port, size_t max_payload, bool jetstream,
                       const std::string& store_dir, const std::string& auth_token,
                       const std::vector<std::pair<std::string, std::string>>& users,
                       const std::vector<std::string>& nkeys) {
             ServerOptions o;
             o.host = host;
             o.port = port;
             o.max_payload = max_payload;
             o.jetstream = jetstream;
             o.store_dir = store_dir;
             o.auth_token = auth_token;
             o.users = users;
             o.nkeys = nkeys;
             return new Server(o);
           }),
           py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("max_payload") = 1 << 20,
           py::arg("jetstream") = true, py::arg("store_dir") = "", py::arg("auth_token") = "",
           py::arg("users") = std::vector<std::pair<std::string, std::string>>(),
           py::arg("nkeys") = std::vector<std::string>())
      .def("start", &Server::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Server::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Server::port)
      .def_property_readonly("running", &Server::running)
      .def("set_fault", &Server::set_fault, py::arg("drop_rate") = 0.0, py::arg("delay_ms") = 0)
      .def("disconnect_all", &Server::disconnect_all, py::call_guard<py::gil_scoped_release>())
      .def("stats", &Server::stats_json);

  py::class_<Client>(m, "Client")
      .def(py::init<>())
      .def(
          "connect",
          [](Client& c, const std::string& url, const std::string& name, int timeout_ms, bool reconnect,
             int max_reconnect, int reconnect_wait_ms, const std::string& token, const std::string& user,
             const std::string& password, const std::string& nkey_seed, const std::string& jwt, bool tls,
             bool tls_first, bool tls_insecure, const std::string& tls_ca, const std::string& tls_cert,
             const std::string& tls_key) {
            ClientOptions o;
            o.tls.enable = tls;
            o.tls.first = tls_first;
            o.tls.insecure = tls_insecure;
            o.tls.ca = tls_ca;
            o.tls.cert = tls_cert;
            o.tls.key = tls_key;
            o.name = name;
            o.connect_timeout_ms = timeout_ms;
            o.allow_reconnect = reconnect;
            o.max_reconnect = max_reconnect;
            o.reconnect_wait_ms = reconnect_wait_ms;
            o.token = token;
            o.user = user;
            o.pass = password;
            o.nkey_seed = nkey_seed;
            o.jwt = jwt;
            py::gil_scoped_release r;
            c.connect(url, o);
          },
          py::arg("url"), py::arg("name") = "natscore", py::arg("timeout_ms") = 2000, py::arg("reconnect") = true,
          py::arg("max_reconnect") = 60, py::arg("reconnect_wait_ms") = 250, py::arg("token") = "",
          py::arg("user") = "", py::arg("password") = "", py::arg("nkey_seed") = "", py::arg("jwt") = "",
          py::arg("tls") = false, py::arg("tls_first") = false, py::arg("tls_insecure") = false,
          py::arg("tls_ca") = "", py::arg("tls_cert") = "", py::arg("tls_key") = "")
      .def("tls_cipher", &Client::tls_cipher)
      .def("close", &Client::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("connected", &Client::connected)
      .def(
          "publish",
          [](Client& c, const std::string& subj, py::bytes data, const std::string& reply, py::bytes hdr) {
            std::string d = data, h = hdr;
            py::gil_scoped_release r;
            c.publish(subj, d, reply, h);
          },
          py::arg("subject"), py::arg("data"), py::arg("reply") = "", py::arg("headers") = py::bytes(""))
      .def("subscribe", &Client::subscribe, py::arg("subject"), py::arg("queue") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("unsubscribe", &Client::unsubscribe, py::arg("sid"), py::arg("max_msgs") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def(
          "next_msg",
          [](Client& c, int64_t sid, int timeout_ms) {
            Msg m;
            {
              py::gil_scoped_release r;
              m = c.next_msg(sid, timeout_ms);
            }
            return wrap(std::move(m));
          },
          py::arg("sid"), py::arg("timeout_ms") = -1)
      .def("pending", &Client::pending)
      .def(
          "set_auto_reply",
          [](Client& c, int64_t sid, py::object body) {
            std::shared_ptr<const std::string> b;
            if (!body.is_none()) b = std::make_shared<const std::string>(std::string(body.cast<py::bytes>()));
            c.set_auto_reply(sid, std::move(b));
          },
          py::arg("sid"), py::arg("body"))
      .def("auto_replied", &Client::auto_replied)
      .def(
          "request",
          [](Client& c, const std::string& subj, py::bytes data, int timeout_ms, py::bytes hdr) {
            std::string d = data, h = hdr;
            Msg m;
            {
              py::gil_scoped_release r;
              m = c.request(subj, d, timeout_ms, h);
            }
            return wrap(std::move(m));
          },
          py::arg("subject"), py::arg("data"), py::arg("timeout_ms") = 5000, py::arg("headers") = py::bytes(""))
      .def("flush", &Client::flush, py::arg("timeout_ms") = 5000, py::call_guard<py::gil_scoped_release>())
      .def("new_inbox", &Client::new_inbox)
      .def("server_info", &Client::server_info)
      .def_property_readonly("max_payload", &Client::max_payload)
      .def("stats", &Client::stats_json)
      .def(
          "bench_requests",
          [](Client& c, const std::string& subj, py::bytes payload, int n, int timeout_ms) {
            std::string p = payload;
            py::gil_scoped_release r;
            return bench_requests(c, subj, p, n, timeout_ms);
          },
          py::arg("subject"), py::arg("payload"), py::arg("n"), py::arg("timeout_ms") = 5000);

  py::class_<ObjectStore>(m, "ObjectStore")
      .def(py::init<Client&, const std::string&, int>(), py::arg("client"), py::arg("bucket"),
           py::arg("timeout_ms") = 10000, py::keep_alive<1, 2>())
      .def("create", &ObjectStore::create, py::arg("description") = "", py::arg("file_storage") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("exists", &ObjectStore::exists, py::call_guard<py::gil_scoped_release>())
      .def("put_file", &ObjectStore::put_file, py::arg("name"), py::arg("path"), py::arg("chunk_size") = 128 * 1024,
           py::arg("description") = "", py::arg("progress") = nullptr, py::call_guard<py::gil_scoped_release>())
      .def(
          "put_bytes",
          [](ObjectStore& o, const std::string& name, py::bytes data, size_t chunk) {
            std::string d = data;
            py::gil_scoped_release r;
            return o.put_bytes(name, d, chunk);
          },
          py::arg("name"), py::arg("data"), py::arg("chunk_size") = 128 * 1024)
      .def("info", &ObjectStore::info, py::call_guard<py::gil_scoped_release>())
      .def("get_file", &ObjectStore::get_file, py::arg("name"), py::arg("path"), py::arg("resume") = true,
           py::arg("progress") = nullptr, py::arg("deadline_s") = 0.0, py::call_guard<py::gil_scoped_release>())
      .def(
          "get_bytes",
          [](ObjectStore& o, const std::string& name) {
            std::string d;
            {
              py::gil_scoped_release r;
              d = o.get_bytes(name);
            }
            return py::bytes(d);
          },
          py::arg("name"))
      .def("list", &ObjectStore::list, py::call_guard<py::gil_scoped_release>())
      .def("remove", &ObjectStore::remove, py::call_guard<py::gil_scoped_release>())
      .def("meta_subject", &ObjectStore::meta_subject)
      .def_property_readonly("stream", &ObjectStore::stream);

  m.def("sha256", [](py::bytes data) {
    std::string d = data;
    Sha256 s;
    s.update(d.data(), d.size());
    return py::bytes(s.digest());
  });
  m.def("b64encode", [](py::bytes d, bool url) { return b64encode(std::string(d), url); }, py::arg("data"),
        py::arg("url") = false);
  m.def("nuid", &nuid_next);
  m.def("nkey_public", [](const std::string& seed) {
    std::string raw;
    if (!nkey_seed_raw(seed, raw)) throw std::runtime_error("invalid nkey seed");
    return nkey_public(raw);
  });
  m.def("nkey_sign", [](const std::string& seed, py::bytes msg) {
    std::string raw;
    if (!nkey_seed_raw(seed, raw)) throw std::runtime_error("invalid nkey seed");
    return py::bytes(nkey_sign(raw, std::string(msg)));
  });
  m.def("nkey_verify", [](const std::string& pub, py::bytes msg, py::bytes sig) {
    return nkey_verify(pub, std::string(msg), std::string(sig));
  });
  m.def("nkey_user_seed_from_raw", [](py::bytes raw32) {
    // "SU..." text form of a raw 32-byte ed25519 seed (key generation / tests)
    std::string r = raw32;
    if (r.size() != 32) throw std::runtime_error("need 32 bytes");
    std::string body;
    body += (char)(NKEY_PREFIX_SEED | (NKEY_PREFIX_USER >> 5));
    body += (char)((NKEY_PREFIX_USER & 31) << 3);
    body += r;
    const uint16_t crc = crc16_xmodem(body);
    return base32_encode(body + std::string(1, (char)(crc & 0xFF)) + std::string(1, (char)(crc >> 8)));
  });
  m.def("parse_creds", [](const std::string& text) {
    std::string jwt, seed;
    if (!parse_creds(text, jwt, seed)) throw std::runtime_error("no user nkey seed in creds");
    return py::make_tuple(jwt, seed);
  });
  m.def("subject_matches", &subject_matches);
  m.def("parse_headers", [](py::bytes raw) {
    Headers h = parse_headers(std::string(raw));
    py::dict kv;
    for (auto& p : h.kv) kv[py::str(p.first)] = p.second;
    return py::make_tuple(h.status, h.description, kv);
  });
  m.def("build_headers", [](const std::vector<std::pair<std::string, std::string>>& kv, int status,
                            const std::string& desc) { return py::bytes(build_headers(kv, status, desc)); },
        py::arg("kv"), py::arg("status") = 0, py::arg("description") = "");
  m.def(
      "parse_stream",
      [](py::bytes data, size_t max_payload) {
        // protocol-parser test hook: feeds bytes, returns ops as tuples
        Parser p(max_payload);
        py::list out;
        std::string d = data;
        bool ok = p.feed(d.data(), d.size(), [&](Op& op) {
          out.append(py::make_tuple((int)op.kind, op.subject, op.reply, op.queue, op.sid, op.arg,
                                    py::bytes(op.hdr), py::bytes(op.payload), op.max_msgs));
        });
        if (!ok) throw std::runtime_error(p.error());
        return out;
      },
      py::arg("data"), py::arg("max_payload") = 1 << 20);
  m.def("parse_chunks", [](std::vector<py::bytes> chunks) {
    Parser p;
    py::list out;
    for (auto& c : chunks) {
      std::string d = c;
      if (!p.feed(d.data(), d.size(), [&](Op& op) {
            out.append(py::make_tuple((int)op.kind, op.subject, op.reply, op.queue, op.sid, op.arg,
                                      py::bytes(op.hdr), py::bytes(op.payload), op.max_msgs));
          }))
        throw std::runtime_error(p.error());
    }
    return out;
  });
}
