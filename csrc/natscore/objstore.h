// JetStream Object Store (nats.go v1.47 object.go / ADR-20 semantics) on top of Client:
// stream OBJ_<bucket> with subjects $O.<bucket>.C.> (chunks) and $O.<bucket>.M.> (meta,
// base64url(name) with rollup). Streaming put/get of files with SHA-256 digests,
// windowed chunk publishing, atomic .part -> final rename and resumable gets.
// This is the bucket the reference's README designs (`README.md:250-318`, `llm-models`).
#pragma once
#include <functional>
#include <string>

#include "client.h"

namespace natscore {

std::string rfc3339(int64_t ns);

class ObjectStore {
 public:
  ObjectStore(Client& c, const std::string& bucket, int timeout_ms = 10000) : c_(c), bucket_(bucket), to_(timeout_ms) {}
  // Creates the backing stream if missing (idempotent). Returns the stream info JSON.
  std::string create(const std::string& description = "", bool file_storage = true);
  bool exists();
  // Upload a local file as object `name` (replaces any previous version). Returns ObjectInfo JSON.
  std::string put_file(const std::string& name, const std::string& path, size_t chunk_size = 128 * 1024,
                       const std::string& description = "",
                       const std::function<void(uint64_t, uint64_t)>& progress = nullptr);
  std::string put_bytes(const std::string& name, const std::string& data, size_t chunk_size = 128 * 1024);
  // ObjectInfo JSON; throws std::runtime_error("object not found") when absent/deleted.
  std::string info(const std::string& name);
  // Streams the object into `path` (via `path`.part, digest-verified, fsync + rename).
  // With resume=true an interrupted `path`.part (+ `path`.part.idx) is continued.
  // deadline_s > 0: the whole transfer is bounded (the pull_model handler's 10-minute context); on expiry it
  // stops with "context deadline exceeded", leaving the .part file + index for a resumed pull
  std::string get_file(const std::string& name, const std::string& path, bool resume = true,
                       const std::function<void(uint64_t, uint64_t)>& progress = nullptr, double deadline_s = 0.0);
  std::string get_bytes(const std::string& name);
  std::string list();                      // JSON array of ObjectInfo (non-deleted)
  void remove(const std::string& name);    // marks deleted + purges chunks

  std::string stream() const { return "OBJ_" + bucket_; }
  std::string meta_subject(const std::string& name) const { return "$O." + bucket_ + ".M." + b64encode(name, true); }
  std::string chunk_subject(const std::string& nuid) const { return "$O." + bucket_ + ".C." + nuid; }

 private:
  Json api(const std::string& subj, const std::string& body);
  Json info_json(const std::string& name, bool allow_deleted);
  std::string put_stream(const std::string& name, const std::function<size_t(char*, size_t)>& reader, uint64_t total,
                         size_t chunk_size, const std::string& description,
                         const std::function<void(uint64_t, uint64_t)>& progress);
  Client& c_;
  std::string bucket_;
  int to_;
};

}  // namespace natscore
