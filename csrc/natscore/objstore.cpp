#include "objstore.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <ctime>
#include <deque>

namespace natscore {

std::string rfc3339(int64_t ns) {
  time_t sec = (time_t)(ns / 1000000000);
  long frac = (long)(ns % 1000000000);
  struct tm tmv;
  gmtime_r(&sec, &tmv);
  char buf[64];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tmv);
  char out[80];
  snprintf(out, sizeof out, "%s.%09ldZ", buf, frac);
  return out;
}

static int64_t wall_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

Json ObjectStore::api(const std::string& subj, const std::string& body) {
  Msg m = c_.request(subj, body, to_);
  Json j = Json::parse(m.data);
  return j;
}

static std::string api_err(const Json& j) {
  if (auto* e = j.get("error")) return e->str("description", "jetstream error");
  return "";
}

std::string ObjectStore::create(const std::string& description, bool file_storage) {
  Json cfg = Json::O();
  cfg.set("name", Json::S(stream()));
  if (!description.empty()) cfg.set("description", Json::S(description));
  Json subj = Json::A();
  subj.a.push_back(Json::S("$O." + bucket_ + ".C.>"));
  subj.a.push_back(Json::S("$O." + bucket_ + ".M.>"));
  cfg.set("subjects", subj);
  cfg.set("retention", Json::S("limits"));
  cfg.set("max_consumers", Json::N(-1));
  cfg.set("max_msgs", Json::N(-1));
  cfg.set("max_bytes", Json::N(-1));
  cfg.set("discard", Json::S("new"));
  cfg.set("storage", Json::S(file_storage ? "file" : "memory"));
  cfg.set("num_replicas", Json::N(1));
  cfg.set("allow_rollup_hdrs", Json::B(true));
  cfg.set("allow_direct", Json::B(true));
  Json r = api("$JS.API.STREAM.CREATE." + stream(), cfg.dump());
  std::string e = api_err(r);
  if (!e.empty()) throw std::runtime_error("object store create: " + e);
  return r.dump();
}

bool ObjectStore::exists() {
  Json r = api("$JS.API.STREAM.INFO." + stream(), "");
  return api_err(r).empty();
}

Json ObjectStore::info_json(const std::string& name, bool allow_deleted) {
  Json req = Json::O();
  req.set("last_by_subj", Json::S(meta_subject(name)));
  Json r = api("$JS.API.STREAM.MSG.GET." + stream(), req.dump());
  if (auto* e = r.get("error")) {
    if ((int)e->num("code") == 404) throw std::runtime_error("object not found");
    throw std::runtime_error("object store: " + e->str("description"));
  }
  const Json* m = r.get("message");
  if (!m) throw std::runtime_error("object store: malformed response");
  Json info = Json::parse(b64decode(m->str("data")));
  if (!allow_deleted && info.boolean("deleted", false)) throw std::runtime_error("object not found");
  return info;
}

std::string ObjectStore::info(const std::string& name) { return info_json(name, false).dump(); }

std::string ObjectStore::put_stream(const std::string& name, const std::function<size_t(char*, size_t)>& reader,
                                    uint64_t total, size_t chunk_size, const std::string& description,
                                    const std::function<void(uint64_t, uint64_t)>& progress) {
  if (name.empty()) throw std::runtime_error("object name is required");
  if (chunk_size == 0 || chunk_size + 256 > c_.max_payload()) chunk_size = std::min<size_t>(128 * 1024, c_.max_payload() - 256);
  std::string old_nuid;
  try {
    old_nuid = info_json(name, true).str("nuid");
  } catch (...) {
  }
  const std::string nuid = nuid_next();
  const std::string csubj = chunk_subject(nuid);
  // windowed publish: up to W chunk publishes awaiting their PubAck
  const std::string inbox = c_.new_inbox();
  int64_t sid = c_.subscribe(inbox + ".*");
  const int W = 32;
  int outstanding = 0;
  Sha256 sha;
  uint64_t sent = 0, chunks = 0;
  std::string buf(chunk_size, '\0');
  auto wait_ack = [&]() {
    Msg a = c_.next_msg(sid, to_);
    Json j = Json::parse(a.data);
    std::string e = api_err(j);
    if (!e.empty()) throw std::runtime_error("object store put: " + e);
    --outstanding;
  };
  try {
    while (true) {
      size_t n = 0;
      while (n < chunk_size) {
        size_t r = reader(&buf[n], chunk_size - n);
        if (r == 0) break;
        n += r;
      }
      if (n == 0) break;
      sha.update(buf.data(), n);
      if (outstanding >= W) wait_ack();
      c_.publish(csubj, std::string(buf.data(), n), inbox + "." + std::to_string(chunks));
      ++outstanding;
      ++chunks;
      sent += n;
      if (progress) progress(sent, total);
      if (n < chunk_size) break;
    }
    while (outstanding > 0) wait_ack();
  } catch (...) {
    c_.unsubscribe(sid);
    // best effort: drop the partial chunks
    Json pr = Json::O();
    pr.set("filter", Json::S(csubj));
    try { api("$JS.API.STREAM.PURGE." + stream(), pr.dump()); } catch (...) {}
    throw;
  }
  c_.unsubscribe(sid);
  Json info = Json::O();
  info.set("name", Json::S(name));
  if (!description.empty()) info.set("description", Json::S(description));
  Json opts = Json::O();
  opts.set("max_chunk_size", Json::N((double)chunk_size));
  info.set("options", opts);
  info.set("bucket", Json::S(bucket_));
  info.set("nuid", Json::S(nuid));
  info.set("size", Json::N((double)sent));
  info.set("mtime", Json::S(rfc3339(wall_ns())));
  info.set("chunks", Json::N((double)chunks));
  info.set("digest", Json::S("SHA-256=" + b64encode(sha.digest(), true)));
  std::string hdr = build_headers({{"Nats-Rollup", "sub"}});
  Msg ack = c_.request(meta_subject(name), info.dump(), to_, hdr);
  std::string e = api_err(Json::parse(ack.data));
  if (!e.empty()) throw std::runtime_error("object store meta: " + e);
  if (!old_nuid.empty() && old_nuid != nuid) {
    Json pr = Json::O();
    pr.set("filter", Json::S(chunk_subject(old_nuid)));
    api("$JS.API.STREAM.PURGE." + stream(), pr.dump());
  }
  return info.dump();
}

std::string ObjectStore::put_file(const std::string& name, const std::string& path, size_t chunk_size,
                                  const std::string& description,
                                  const std::function<void(uint64_t, uint64_t)>& progress) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  struct stat st;
  fstat(fileno(f), &st);
  try {
    std::string r = put_stream(
        name, [&](char* p, size_t n) { return fread(p, 1, n, f); }, (uint64_t)st.st_size, chunk_size, description,
        progress);
    fclose(f);
    return r;
  } catch (...) {
    fclose(f);
    throw;
  }
}

std::string ObjectStore::put_bytes(const std::string& name, const std::string& data, size_t chunk_size) {
  size_t off = 0;
  return put_stream(
      name,
      [&](char* p, size_t n) {
        size_t k = std::min(n, data.size() - off);
        memcpy(p, data.data() + off, k);
        off += k;
        return k;
      },
      data.size(), chunk_size, "", nullptr);
}

std::string ObjectStore::get_file(const std::string& name, const std::string& path, bool resume,
                                  const std::function<void(uint64_t, uint64_t)>& progress, double deadline_s) {
  using clk = std::chrono::steady_clock;
  const bool has_dl = deadline_s > 0;
  const auto dl = clk::now() + std::chrono::microseconds((long long)(deadline_s * 1e6));
  // time left for one wait (capped by the per-operation timeout); throws once the deadline has passed
  auto wait_ms = [&]() -> int {
    if (!has_dl) return to_;
    const long long left = std::chrono::duration_cast<std::chrono::milliseconds>(dl - clk::now()).count();
    if (left <= 0) throw std::runtime_error("context deadline exceeded");
    return (int)std::min<long long>(to_, left);
  };
  Json info = info_json(name, false);
  const std::string nuid = info.str("nuid");
  const uint64_t size = (uint64_t)info.num("size"), nchunks = (uint64_t)info.num("chunks");
  const std::string digest = info.str("digest");
  const std::string part = path + ".part", idxp = path + ".part.idx";
  Sha256 sha;
  uint64_t got = 0, seq = 1, nread = 0;
  int fd = -1;
  if (resume) {   // continue an interrupted transfer of the same object version
    FILE* ix = fopen(idxp.c_str(), "rb");
    if (ix) {
      char b[512] = {0};
      size_t n = fread(b, 1, sizeof b - 1, ix);
      fclose(ix);
      try {
        Json j = Json::parse(std::string(b, n));
        if (j.str("nuid") == nuid) {
          uint64_t bytes = (uint64_t)j.num("bytes");
          fd = ::open(part.c_str(), O_RDWR);
          if (fd >= 0) {
            // re-hash the already-received prefix, then truncate to it
            std::string rb(1 << 20, '\0');
            uint64_t left = bytes;
            bool ok = true;
            while (left) {
              ssize_t r = ::read(fd, &rb[0], std::min<uint64_t>(left, rb.size()));
              if (r <= 0) { ok = false; break; }
              sha.update(rb.data(), (size_t)r);
              left -= (uint64_t)r;
            }
            if (ok && ftruncate(fd, (off_t)bytes) == 0 && lseek(fd, (off_t)bytes, SEEK_SET) == (off_t)bytes) {
              got = bytes;
              seq = (uint64_t)j.num("next_seq");
              nread = (uint64_t)j.num("chunks");
            } else {
              ::close(fd);
              fd = -1;
              sha = Sha256();
            }
          }
        }
      } catch (...) {
      }
    }
  }
  if (fd < 0) {
    fd = ::open(part.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw std::runtime_error("cannot create " + part);
    got = 0;
    seq = 1;
    nread = 0;
  }
  const std::string csubj = chunk_subject(nuid);
  auto save_idx = [&]() {
    FILE* ix = fopen(idxp.c_str(), "wb");
    if (!ix) return;
    Json j = Json::O();
    j.set("nuid", Json::S(nuid));
    j.set("bytes", Json::N((double)got));
    j.set("next_seq", Json::N((double)seq));
    j.set("chunks", Json::N((double)nread));
    std::string s = j.dump();
    fwrite(s.data(), 1, s.size(), ix);
    fclose(ix);
  };
  auto put_chunk = [&](const std::string& data, uint64_t sseq) {
    sha.update(data.data(), data.size());
    size_t off = 0;
    while (off < data.size()) {
      ssize_t w = ::write(fd, data.data() + off, data.size() - off);
      if (w <= 0) throw std::runtime_error("write failed: " + part);
      off += (size_t)w;
    }
    got += data.size();
    seq = sseq + 1;
    ++nread;
    if ((nread & 63) == 0) save_idx();
    if (progress) progress(got, size);
    if (has_dl) wait_ms();
  };
  try {
    // 1) ordered push consumer (what nats.go's ObjectStore.Get does): raw chunk payloads streamed to an
    //    inbox, no per-chunk request round trip and no base64; flow-control requests are answered as
    //    the chunks are consumed, so the server never runs more than a window ahead of the disk
    bool streamed = false;
    if (nread < nchunks) {
      const std::string inbox = c_.new_inbox();
      int64_t sid = c_.subscribe(inbox);
      const std::string cname = "get" + nuid_next();
      Json cfg = Json::O();
      cfg.set("name", Json::S(cname));
      cfg.set("deliver_subject", Json::S(inbox));
      cfg.set("filter_subject", Json::S(csubj));
      cfg.set("deliver_policy", Json::S("by_start_sequence"));
      cfg.set("opt_start_seq", Json::N((double)seq));
      cfg.set("ack_policy", Json::S("none"));
      cfg.set("max_deliver", Json::N(1));
      cfg.set("flow_control", Json::B(true));
      cfg.set("idle_heartbeat", Json::N(5e9));
      cfg.set("mem_storage", Json::B(true));
      Json creq = Json::O();
      creq.set("stream_name", Json::S(stream()));
      creq.set("config", cfg);
      std::string cerr;
      try {
        cerr = api_err(api("$JS.API.CONSUMER.CREATE." + stream() + "." + cname + "." + csubj, creq.dump()));
      } catch (const std::exception& ex) {
        cerr = ex.what();
      }
      if (cerr.empty()) {
        try {
          while (nread < nchunks) {
            Msg m = c_.next_msg(sid, wait_ms());
            if (m.status == 100) {                    // flow control request / idle heartbeat
              if (!m.reply.empty()) c_.publish(m.reply, "");
              continue;
            }
            // reply: $JS.ACK.<stream>.<consumer>.<delivered>.<stream seq>.<consumer seq>.<ts>.<pending>
            std::vector<std::string> tok;
            size_t a = 0;
            for (size_t b; (b = m.reply.find('.', a)) != std::string::npos; a = b + 1) tok.push_back(m.reply.substr(a, b - a));
            tok.push_back(m.reply.substr(a));
            if (tok.size() < 9 || tok[0] != "$JS" || tok[1] != "ACK") throw std::runtime_error("object store get: bad delivery");
            const uint64_t sseq = std::stoull(tok[5]);
            if (sseq < seq) continue;                 // duplicate (never expected)
            put_chunk(m.data, sseq);
          }
          streamed = true;
        } catch (...) {
          try { api("$JS.API.CONSUMER.DELETE." + stream() + "." + cname, ""); } catch (...) {}
          c_.unsubscribe(sid);
          throw;
        }
        try { api("$JS.API.CONSUMER.DELETE." + stream() + "." + cname, ""); } catch (...) {}
      }
      c_.unsubscribe(sid);
    }
    // 2) fallback (servers without push consumers): one direct get per chunk
    while (!streamed && nread < nchunks) {
      Json req = Json::O();
      req.set("seq", Json::N((double)seq));
      req.set("next_by_subj", Json::S(csubj));
      Json r = api("$JS.API.STREAM.MSG.GET." + stream(), req.dump());
      std::string e = api_err(r);
      if (!e.empty()) throw std::runtime_error("object store get: " + e);
      const Json* m = r.get("message");
      put_chunk(b64decode(m->str("data")), (uint64_t)m->num("seq"));
    }
  } catch (...) {
    save_idx();
    ::close(fd);
    if (has_dl && clk::now() >= dl) throw std::runtime_error("context deadline exceeded");
    throw;
  }
  ::fsync(fd);
  ::close(fd);
  if (got != size) throw std::runtime_error("object store get: size mismatch");
  std::string dg = "SHA-256=" + b64encode(sha.digest(), true);
  if (!digest.empty() && dg != digest) {
    ::unlink(part.c_str());
    ::unlink(idxp.c_str());
    throw std::runtime_error("object store get: digest mismatch (" + dg + " != " + digest + ")");
  }
  if (::rename(part.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed: " + path);
  ::unlink(idxp.c_str());
  return info.dump();
}

std::string ObjectStore::get_bytes(const std::string& name) {
  Json info = info_json(name, false);
  const std::string csubj = chunk_subject(info.str("nuid"));
  const uint64_t nchunks = (uint64_t)info.num("chunks");
  std::string out;
  uint64_t seq = 1;
  Sha256 sha;
  for (uint64_t k = 0; k < nchunks; ++k) {
    Json req = Json::O();
    req.set("seq", Json::N((double)seq));
    req.set("next_by_subj", Json::S(csubj));
    Json r = api("$JS.API.STREAM.MSG.GET." + stream(), req.dump());
    std::string e = api_err(r);
    if (!e.empty()) throw std::runtime_error("object store get: " + e);
    const Json* m = r.get("message");
    std::string d = b64decode(m->str("data"));
    sha.update(d.data(), d.size());
    out += d;
    seq = (uint64_t)m->num("seq") + 1;
  }
  std::string dg = "SHA-256=" + b64encode(sha.digest(), true);
  if (info.str("digest") != "" && dg != info.str("digest")) throw std::runtime_error("digest mismatch");
  return out;
}

std::string ObjectStore::list() {
  Json arr = Json::A();
  uint64_t seq = 1;
  const std::string filt = "$O." + bucket_ + ".M.>";
  std::map<std::string, Json> latest;
  while (true) {
    Json req = Json::O();
    req.set("seq", Json::N((double)seq));
    req.set("next_by_subj", Json::S(filt));
    Json r = api("$JS.API.STREAM.MSG.GET." + stream(), req.dump());
    if (r.get("error")) break;
    const Json* m = r.get("message");
    Json info = Json::parse(b64decode(m->str("data")));
    latest[m->str("subject")] = info;
    seq = (uint64_t)m->num("seq") + 1;
  }
  for (auto& kv : latest)
    if (!kv.second.boolean("deleted", false)) arr.a.push_back(kv.second);
  return arr.dump();
}

void ObjectStore::remove(const std::string& name) {
  Json info = info_json(name, false);
  Json del = info;
  del.set("deleted", Json::B(true));
  del.set("size", Json::N(0));
  del.set("chunks", Json::N(0));
  del.set("digest", Json::S(""));
  del.set("mtime", Json::S(rfc3339(wall_ns())));
  std::string hdr = build_headers({{"Nats-Rollup", "sub"}});
  c_.request(meta_subject(name), del.dump(), to_, hdr);
  Json pr = Json::O();
  pr.set("filter", Json::S(chunk_subject(info.str("nuid"))));
  api("$JS.API.STREAM.PURGE." + stream(), pr.dump());
}

}  // namespace natscore
