"""Python face of the native NATS core (`_natscore`, C++ in csrc/natscore).

* `Client`  -- connect / publish / subscribe (queue groups, callback dispatcher threads) /
  request (muxed inbox) / flush / close, with automatic reconnect + resubscribe.
* `EmbeddedServer` -- in-process nats-server subset (core + JetStream object-store subset).
* `ObjectStore` -- JetStream object store (bucket `llm-models` in the reference README).

nats-py is not installed and there is no nats-server binary in this image, so both
sides of the wire are implemented natively here.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Callable, Dict, Optional

from ..build import natscore_path

try:
    from . import _natscore as _nc
except ImportError as e:  # pragma: no cover - build missing
    raise ImportError(f"natscore extension not built ({natscore_path()}); run "
                      "`python -m nats_llm_studio_amd.build`") from e

TimeoutError = _nc.TimeoutError
NoRespondersError = _nc.NoRespondersError
ConnectionClosedError = _nc.ConnectionClosedError
Msg = _nc.Msg


def headers(msg) -> Dict[str, str]:
    if not msg.raw_headers:
        return {}
    return dict(_nc.parse_headers(msg.raw_headers)[2])


class Subscription:
    def __init__(self, client: "Client", sid: int, subject: str, queue: str, cb, workers: int):
        self.client = client
        self.sid = sid
        self.subject = subject
        self.queue = queue
        self._cb = cb
        self._stop = False
        self._threads = []
        if cb is not None:
            for i in range(max(1, workers)):
                t = threading.Thread(target=self._run, name=f"nats-sub-{subject}-{i}", daemon=True)
                t.start()
                self._threads.append(t)

    def _run(self):
        nc = self.client._c
        while not self._stop:
            try:
                m = nc.next_msg(self.sid, 500)
            except TimeoutError:
                continue
            except (ConnectionClosedError, RuntimeError):
                return
            try:
                self._cb(m)
            except Exception:  # a handler bug must not kill the dispatcher
                import traceback
                traceback.print_exc()

    def next_msg(self, timeout: float = 1.0):
        return self.client._c.next_msg(self.sid, int(timeout * 1000))

    def set_auto_reply(self, body: Optional[bytes]):
        """Answer this subscription's requests with `body` from the native reader thread (None: hand them to
        the callback again). For cached read-only replies; the owner keeps `body` current."""
        self.client._c.set_auto_reply(self.sid, body)

    @property
    def auto_replied(self) -> int:
        return self.client._c.auto_replied(self.sid)

    def unsubscribe(self):
        self._stop = True
        try:
            self.client._c.unsubscribe(self.sid)
        except Exception:
            pass


class Client:
    def __init__(self):
        self._c = _nc.Client()
        self.subs = []

    def connect(self, url: str = "nats://127.0.0.1:4222", name: str = "nats-llm-studio-amd", timeout: float = 2.0,
                reconnect: bool = True, max_reconnect: int = 60, reconnect_wait: float = 0.25, token: str = "",
                user: str = "", password: str = "", nkey_seed: str = "", creds: str = "", tls: bool = False,
                tls_first: bool = False, tls_insecure: bool = False, tls_ca: str = "", tls_cert: str = "",
                tls_key: str = "") -> "Client":
        """Authentication as nats.go: `token`, `user`/`password` (or in the URL), `nkey_seed` ("SU..."),
        or a `.creds` file (user JWT + seed); nkey-based methods sign the server's INFO nonce.
        TLS (OpenSSL, csrc/natscore/tls.cpp): a `tls://` URL or `tls=True` requires it, a server INFO with
        `tls_required` upgrades to it; `tls_ca` (CA bundle, else the system store), `tls_cert` / `tls_key`
        (mutual TLS), `tls_insecure` (no verification), `tls_first` (handshake before the server's INFO)."""
        jwt = ""
        if creds:
            with open(os.path.expanduser(creds)) as f:
                jwt, nkey_seed = _nc.parse_creds(f.read())
        self._c.connect(url, name, int(timeout * 1000), reconnect, max_reconnect, int(reconnect_wait * 1000), token,
                        user, password, nkey_seed, jwt, tls, tls_first, tls_insecure,
                        os.path.expanduser(tls_ca) if tls_ca else "", os.path.expanduser(tls_cert) if tls_cert else "",
                        os.path.expanduser(tls_key) if tls_key else "")
        return self

    @property
    def connected(self) -> bool:
        return self._c.connected

    @property
    def max_payload(self) -> int:
        return self._c.max_payload

    def publish(self, subject: str, data: bytes = b"", reply: str = "", headers: Optional[Dict[str, str]] = None):
        hdr = _nc.build_headers(list(headers.items())) if headers else b""
        self._c.publish(subject, data, reply, hdr)

    def subscribe(self, subject: str, queue: str = "", cb: Callable = None, workers: int = 1) -> Subscription:
        sid = self._c.subscribe(subject, queue)
        s = Subscription(self, sid, subject, queue, cb, workers)
        self.subs.append(s)
        return s

    def request(self, subject: str, data: bytes = b"", timeout: float = 5.0, headers: Optional[Dict[str, str]] = None):
        hdr = _nc.build_headers(list(headers.items())) if headers else b""
        return self._c.request(subject, data, int(timeout * 1000), hdr)

    def request_json(self, subject: str, obj, timeout: float = 5.0):
        m = self.request(subject, json.dumps(obj).encode(), timeout)
        return json.loads(m.data)

    def flush(self, timeout: float = 5.0):
        self._c.flush(int(timeout * 1000))

    def new_inbox(self) -> str:
        return self._c.new_inbox()

    def stats(self) -> dict:
        return json.loads(self._c.stats())

    def close(self):
        for s in self.subs:
            s._stop = True
        self._c.close()
        for s in self.subs:
            for t in s._threads:
                t.join(timeout=2)


class EmbeddedServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, max_payload: int = 1 << 20, jetstream: bool = True,
                 store_dir: str = "", auth_token: str = "", users=(), nkeys=()):
        """`auth_token` / `users` [(user, password)] / `nkeys` ["U..." public keys]: any of them makes
        the server require authentication (INFO auth_required + a per-connection nonce)."""
        self._s = _nc.Server(host, port, max_payload, jetstream, store_dir, auth_token, list(users), list(nkeys))
        self.host = host

    def start(self) -> "EmbeddedServer":
        self._s.start()
        return self

    @property
    def port(self) -> int:
        return self._s.port

    @property
    def url(self) -> str:
        return f"nats://{self.host}:{self.port}"

    def stop(self):
        self._s.stop()

    def set_fault(self, drop_rate: float = 0.0, delay_ms: int = 0):
        self._s.set_fault(drop_rate, delay_ms)

    def disconnect_all(self):
        self._s.disconnect_all()

    def stats(self) -> dict:
        return json.loads(self._s.stats())

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()


def nkey_keypair(raw32: bytes = None):
    """(seed "SU...", public "U...") of a new (or given 32-byte) user nkey."""
    raw32 = raw32 if raw32 is not None else os.urandom(32)
    seed = _nc.nkey_user_seed_from_raw(raw32)
    return seed, _nc.nkey_public(seed)


class ObjectStore:
    def __init__(self, client: Client, bucket: str, timeout: float = 10.0):
        self.client = client
        self.bucket = bucket
        self._o = _nc.ObjectStore(client._c, bucket, int(timeout * 1000))

    def create(self, description: str = "", file_storage: bool = True) -> dict:
        return json.loads(self._o.create(description, file_storage))

    def exists(self) -> bool:
        return self._o.exists()

    def put_file(self, name: str, path: str, chunk_size: int = 128 * 1024, description: str = "",
                 progress: Callable[[int, int], None] = None) -> dict:
        return json.loads(self._o.put_file(name, path, chunk_size, description, progress))

    def put_bytes(self, name: str, data: bytes, chunk_size: int = 128 * 1024) -> dict:
        return json.loads(self._o.put_bytes(name, data, chunk_size))

    def info(self, name: str) -> dict:
        return json.loads(self._o.info(name))

    def get_file(self, name: str, path: str, resume: bool = True, progress: Callable[[int, int], None] = None,
                 deadline_s: float = 0.0) -> dict:
        """Stream an object to `path` (.part + resume index, SHA-256 verified); deadline_s > 0 bounds the
        whole transfer (RuntimeError "context deadline exceeded", resumable)."""
        return json.loads(self._o.get_file(name, path, resume, progress, float(deadline_s)))

    def get_bytes(self, name: str) -> bytes:
        return self._o.get_bytes(name)

    def list(self):
        return json.loads(self._o.list())

    def remove(self, name: str):
        self._o.remove(name)


def sha256_digest(data: bytes) -> str:
    """ObjectInfo digest string: 'SHA-256=' + base64url(sha256) (nats.go format)."""
    return "SHA-256=" + _nc.b64encode(_nc.sha256(data), True)
