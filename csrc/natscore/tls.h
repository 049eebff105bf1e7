// TLS transport of the NATS client (OpenSSL 3). nats.go's options: a `tls://` URL or `secure` forces TLS,
// a server INFO with `tls_required` upgrades the connection after the plaintext INFO line (the NATS
// protocol's upgrade), `handshake_first` runs the handshake before any byte of the protocol (nats-server
// 2.10 `handshake_first`). The server certificate is verified against a CA file (RootCAs) or the system
// store, with the URL host checked against its SAN / CN; an optional client certificate + key gives
// mutual TLS; `insecure` skips verification (InsecureSkipVerify).
//
// One SSL object serves the reader thread and the writers: the socket is non-blocking after the handshake
// and every SSL call runs under one mutex, the waiting (poll) outside it, so a reader parked on an empty
// socket never blocks a publish.
#pragma once
#include <atomic>
#include <mutex>
#include <string>

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace natscore {

struct TlsOptions {
  bool enable = false;       // TLS required by the client (tls:// URL, secure option)
  bool first = false;        // handshake before the server's INFO
  bool insecure = false;     // skip certificate verification
  std::string ca, cert, key; // PEM files: CA bundle (empty: system store), client certificate chain + key
};

class TlsConn {
 public:
  ~TlsConn();
  // TLS client handshake on a connected socket (blocking, bounded by timeout_ms). host: the name (or IP)
  // the certificate must carry. false + err on failure.
  bool handshake(int fd, const std::string& host, const TlsOptions& o, int timeout_ms, std::string& err);
  // > 0 bytes read, 0 peer closed, < 0 error / `stop` raised while waiting
  long read(char* buf, size_t n, const std::atomic<bool>& stop);
  bool write_all(const char* p, size_t n);
  std::string cipher() const;

 private:
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  int fd_ = -1;
  std::mutex mu_;
};

}  // namespace natscore
