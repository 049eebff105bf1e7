"""NATS over TLS (csrc/natscore/tls.cpp), CPU. The embedded server speaks plain NATS, so a TLS front
(Python `ssl`, certificates made with the openssl CLI) stands in for a TLS nats-server: it forwards the
server's INFO line with `tls_required` set (the NATS upgrade) -- or, in handshake-first mode, completes
the TLS handshake before forwarding anything -- then relays the streams. Checked: the upgrade and
handshake-first paths, `tls://` URLs, CA verification (a certificate from another CA and a wrong host are
refused), `tls_insecure`, mutual TLS, and request-reply / large payloads across the TLS link."""
import json
import os
import select
import shutil
import socket
import ssl
import subprocess
import threading

import pytest

from nats_llm_studio_amd.natsio import Client, ConnectionClosedError, EmbeddedServer

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI needed for test certificates")


def _cert(d, name, cn, san, ca=None):
    key, crt = os.path.join(d, name + ".key"), os.path.join(d, name + ".pem")
    if ca is None:
        subprocess.check_call(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt,
                               "-days", "2", "-subj", f"/CN={cn}", "-addext", "basicConstraints=critical,CA:TRUE"],
                              stderr=subprocess.DEVNULL)
        return crt, key
    csr = os.path.join(d, name + ".csr")
    ext = os.path.join(d, name + ".ext")
    with open(ext, "w") as f:
        f.write(f"subjectAltName={san}\n" if san else "basicConstraints=CA:FALSE\n")
    subprocess.check_call(["openssl", "req", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", csr,
                           "-subj", f"/CN={cn}"], stderr=subprocess.DEVNULL)
    subprocess.check_call(["openssl", "x509", "-req", "-in", csr, "-CA", ca[0], "-CAkey", ca[1], "-CAcreateserial",
                           "-out", crt, "-days", "2", "-extfile", ext], stderr=subprocess.DEVNULL)
    return crt, key


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pki"))
    ca = _cert(d, "ca", "nls test CA", None)
    other = _cert(d, "other", "other CA", None)
    srv = _cert(d, "server", "localhost", "IP:127.0.0.1,DNS:localhost", ca)
    wrong = _cert(d, "wrong", "elsewhere", "DNS:elsewhere.example", ca)
    cli = _cert(d, "client", "worker", "DNS:worker", ca)
    return dict(ca=ca, other=other, srv=srv, wrong=wrong, cli=cli)


class TlsFront:
    """TLS listener in front of a plain NATS server (one relay thread per connection)."""

    def __init__(self, upstream_port, cert, first=False, client_ca=None):
        self.ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        self.ctx.load_cert_chain(*cert)
        if client_ca:
            self.ctx.verify_mode = ssl.CERT_REQUIRED
            self.ctx.load_verify_locations(client_ca)
        self.up, self.first = upstream_port, first
        self.ls = socket.socket()
        self.ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.ls.bind(("127.0.0.1", 0))
        self.ls.listen(8)
        self.port = self.ls.getsockname()[1]
        self.stop = False
        self.handshakes = 0
        threading.Thread(target=self._accept, daemon=True).start()

    def close(self):
        self.stop = True
        self.ls.close()

    def _accept(self):
        while not self.stop:
            try:
                c, _ = self.ls.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        up = socket.create_connection(("127.0.0.1", self.up))
        try:
            if self.first:
                c = self.ctx.wrap_socket(c, server_side=True)
            line = b""
            while not line.endswith(b"\r\n"):           # the server's INFO (it sends nothing more until CONNECT)
                ch = up.recv(1)
                if not ch:
                    return
                line += ch
            info = json.loads(line[5:].decode())
            info["tls_required"] = True
            c.sendall(b"INFO " + json.dumps(info).encode() + b"\r\n")
            if not self.first:
                c = self.ctx.wrap_socket(c, server_side=True)
            self.handshakes += 1
            self._relay(c, up)
        except (OSError, ssl.SSLError, ValueError):
            pass
        finally:
            for s in (c, up):
                try:
                    s.close()
                except OSError:
                    pass

    def _relay(self, c, up):
        c.setblocking(False)
        up.setblocking(False)
        while not self.stop:
            r, _, _ = select.select([c, up], [], [], 0.2)
            if c in r or c.pending():
                try:
                    data = c.recv(1 << 16)
                except ssl.SSLWantReadError:
                    data = None
                if data == b"":
                    return
                if data:
                    up.setblocking(True)
                    up.sendall(data)
                    up.setblocking(False)
            if up in r:
                data = up.recv(1 << 16)
                if not data:
                    return
                c.setblocking(True)
                c.sendall(data)
                c.setblocking(False)


@pytest.fixture()
def server():
    s = EmbeddedServer().start()
    yield s
    s.stop()


def _roundtrip(c: Client, n=5, size=4096):
    sub = c.subscribe("tls.echo")
    srv = c

    def echo():
        for _ in range(n):
            m = sub.next_msg(5.0)
            srv.publish(m.reply, m.data[::-1])

    t = threading.Thread(target=echo)
    t.start()
    for i in range(n):
        payload = os.urandom(size + i)
        assert c.request("tls.echo", payload, timeout=5.0).data == payload[::-1]
    t.join()


@pytest.mark.parametrize("first", [False, True])
def test_tls_upgrade_and_first(server, pki, first):
    front = TlsFront(server.port, pki["srv"], first=first)
    try:
        c = Client().connect(f"nats://127.0.0.1:{front.port}", tls_ca=pki["ca"][0], tls_first=first)
        assert "TLS" in c._c.tls_cipher()
        _roundtrip(c, size=300_000)
        c.close()
        assert front.handshakes >= 1
    finally:
        front.close()


def test_tls_url_scheme_and_verification(server, pki):
    front = TlsFront(server.port, pki["srv"])
    bad = TlsFront(server.port, pki["wrong"])          # valid chain, wrong host name
    try:
        c = Client().connect(f"tls://127.0.0.1:{front.port}", tls_ca=pki["ca"][0])
        _roundtrip(c)
        c.close()
        with pytest.raises(ConnectionClosedError, match="certificate"):
            Client().connect(f"tls://127.0.0.1:{front.port}", tls_ca=pki["other"][0], reconnect=False)
        with pytest.raises(ConnectionClosedError):
            Client().connect(f"tls://127.0.0.1:{bad.port}", tls_ca=pki["ca"][0], reconnect=False)
        c = Client().connect(f"tls://127.0.0.1:{bad.port}", tls_insecure=True)     # InsecureSkipVerify
        _roundtrip(c, n=2)
        c.close()
    finally:
        front.close()
        bad.close()


def test_tls_mutual(server, pki):
    front = TlsFront(server.port, pki["srv"], client_ca=pki["ca"][0])
    try:
        with pytest.raises(ConnectionClosedError):
            Client().connect(f"tls://127.0.0.1:{front.port}", tls_ca=pki["ca"][0], reconnect=False).flush(2.0)
        c = Client().connect(f"tls://127.0.0.1:{front.port}", tls_ca=pki["ca"][0], tls_cert=pki["cli"][0],
                             tls_key=pki["cli"][1])
        _roundtrip(c, n=3)
        c.close()
    finally:
        front.close()


def test_plain_server_with_tls_required_by_client(server, pki):
    """A client that requires TLS against a plain server fails instead of falling back to plaintext."""
    with pytest.raises(ConnectionClosedError):
        Client().connect(f"tls://127.0.0.1:{server.port}", tls_ca=pki["ca"][0], reconnect=False, timeout=1.0)


def test_worker_config_tls_env():
    from nats_llm_studio_amd.service.config import WorkerConfig
    c = WorkerConfig.from_env({"NATS_TLS": "1", "NATS_TLS_CA": "/x/ca.pem", "NATS_TLS_CERT": "/x/c.pem",
                               "NATS_TLS_KEY": "/x/k.pem", "NATS_TLS_FIRST": "true"})
    kw = c.nats_auth()
    assert kw["tls"] and kw["tls_first"] and not kw["tls_insecure"]
    assert (kw["tls_ca"], kw["tls_cert"], kw["tls_key"]) == ("/x/ca.pem", "/x/c.pem", "/x/k.pem")


def test_configured_ca_requires_tls(server, pki):
    """A CA bundle (or client certificate) makes TLS required: against a plaintext server whose INFO does not
    ask for TLS (e.g. a man in the middle stripped tls_required) the client must refuse rather than send its
    credentials in the clear (nats.go: RootCAs / ClientCert imply Secure)."""
    with pytest.raises(ConnectionClosedError):
        Client().connect(f"nats://127.0.0.1:{server.port}", tls_ca=pki["ca"][0], reconnect=False, timeout=2.0)
    c = Client().connect(f"nats://127.0.0.1:{server.port}", reconnect=False)     # no TLS options: plaintext ok
    c.flush(2.0)
    c.close()
