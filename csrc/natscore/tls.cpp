#include "tls.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>

namespace natscore {

static std::string ssl_err(const char* what) {
  std::string s = what;
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    char b[256];
    ERR_error_string_n(e, b, sizeof b);
    s += ": ";
    s += b;
  }
  return s;
}

TlsConn::~TlsConn() {
  if (ssl_) SSL_free(ssl_);
  if (ctx_) SSL_CTX_free(ctx_);
}

bool TlsConn::handshake(int fd, const std::string& host, const TlsOptions& o, int timeout_ms, std::string& err) {
  fd_ = fd;
  ctx_ = SSL_CTX_new(TLS_client_method());
  if (!ctx_) { err = ssl_err("SSL_CTX_new"); return false; }
  SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
  if (o.insecure) {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
    const int ok = o.ca.empty() ? SSL_CTX_set_default_verify_paths(ctx_)
                                : SSL_CTX_load_verify_locations(ctx_, o.ca.c_str(), nullptr);
    if (ok != 1) { err = ssl_err("loading the CA certificates"); return false; }
  }
  if (!o.cert.empty()) {
    if (SSL_CTX_use_certificate_chain_file(ctx_, o.cert.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx_, (o.key.empty() ? o.cert : o.key).c_str(), SSL_FILETYPE_PEM) != 1 ||
        SSL_CTX_check_private_key(ctx_) != 1) {
      err = ssl_err("loading the client certificate");
      return false;
    }
  }
  ssl_ = SSL_new(ctx_);
  if (!ssl_ || SSL_set_fd(ssl_, fd) != 1) { err = ssl_err("SSL_new"); return false; }
  in6_addr a6;
  in_addr a4;
  const bool is_ip = inet_pton(AF_INET, host.c_str(), &a4) == 1 || inet_pton(AF_INET6, host.c_str(), &a6) == 1;
  if (!o.insecure) {
    X509_VERIFY_PARAM* vp = SSL_get0_param(ssl_);
    if (is_ip ? X509_VERIFY_PARAM_set1_ip_asc(vp, host.c_str()) != 1 : X509_VERIFY_PARAM_set1_host(vp, host.c_str(), 0) != 1) {
      err = ssl_err("setting the expected host");
      return false;
    }
  }
  if (!is_ip) SSL_set_tlsext_host_name(ssl_, host.c_str());
  // blocking handshake bounded by socket timeouts
  const int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  if (SSL_connect(ssl_) != 1) {
    const long vr = SSL_get_verify_result(ssl_);
    err = ssl_err("TLS handshake");
    if (vr != X509_V_OK) err += std::string(" (certificate: ") + X509_verify_cert_error_string(vr) + ")";
    return false;
  }
  timeval zero{0, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &zero, sizeof zero);
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &zero, sizeof zero);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  return true;
}

long TlsConn::read(char* buf, size_t n, const std::atomic<bool>& stop) {
  while (!stop) {
    int r, e;
    {
      std::lock_guard<std::mutex> g(mu_);
      r = SSL_read(ssl_, buf, (int)n);
      e = r > 0 ? SSL_ERROR_NONE : SSL_get_error(ssl_, r);
    }
    if (r > 0) return r;
    if (e == SSL_ERROR_ZERO_RETURN) return 0;
    if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) return -1;
    pollfd p{fd_, (short)(e == SSL_ERROR_WANT_READ ? POLLIN : POLLOUT), 0};
    if (poll(&p, 1, 100) < 0) return -1;
    if (p.revents & (POLLERR | POLLNVAL)) return -1;
  }
  return -1;
}

// Callers serialise writers (Client::write_raw holds the connection's write mutex); mu_ guards the SSL
// object against the reader thread and is held only around SSL_write itself -- the wait for socket space
// runs unlocked, so a slow link never stops incoming messages. A retried SSL_write gets the same buffer
// and length, as OpenSSL requires after WANT_WRITE / WANT_READ.
bool TlsConn::write_all(const char* p, size_t n) {
  int waits = 0;
  while (n) {
    const int len = (int)std::min<size_t>(n, 1 << 30);
    int r, e;
    {
      std::lock_guard<std::mutex> g(mu_);
      r = SSL_write(ssl_, p, len);
      e = r > 0 ? SSL_ERROR_NONE : SSL_get_error(ssl_, r);
    }
    if (r > 0) {
      p += r;
      n -= (size_t)r;
      waits = 0;
      continue;
    }
    if ((e != SSL_ERROR_WANT_WRITE && e != SSL_ERROR_WANT_READ) || ++waits > 600) return false;   // ~60 s stalled
    pollfd q{fd_, (short)(e == SSL_ERROR_WANT_WRITE ? POLLOUT : POLLIN), 0};
    if (poll(&q, 1, 100) < 0) return false;
  }
  return true;
}

std::string TlsConn::cipher() const {
  if (!ssl_) return "";
  return std::string(SSL_get_version(ssl_)) + " " + SSL_get_cipher(ssl_);
}

}  // namespace natscore
