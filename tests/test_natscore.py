"""Native NATS core: protocol parser, embedded server, client, object store (CPU)."""
import os
import threading
import time

import pytest
from hypothesis import given, settings, strategies as st

from nats_llm_studio_amd.natsio import (Client, ConnectionClosedError, EmbeddedServer, NoRespondersError,
                                        ObjectStore, TimeoutError, _nc, headers, sha256_digest)

PING, PONG, PUB, HPUB, MSG, HMSG = 8, 9, 2, 3, 6, 7


@pytest.fixture()
def server():
    s = EmbeddedServer().start()
    yield s
    s.stop()


def client(server, **kw):
    return Client().connect(server.url, **kw)


# ---------------------------------------------------------------- parser
def test_parser_ops():
    raw = (b"PING\r\nPONG\r\nPUB a.b 5\r\nhello\r\nPUB a.b _INBOX.x 0\r\n\r\n"
           b"HPUB h.s rep 24 29\r\nNATS/1.0\r\nK: V\r\nX: Y\r\n\r\nworld\r\n"
           b"SUB foo.* q1 7\r\nUNSUB 7 3\r\nMSG s 1 r 3\r\nabc\r\n+OK\r\n-ERR 'x'\r\n")
    ops = _nc.parse_stream(raw)
    kinds = [o[0] for o in ops]
    assert kinds == [8, 9, 2, 2, 3, 4, 5, 6, 10, 11]
    assert ops[2][1] == "a.b" and ops[2][7] == b"hello"
    assert ops[3][2] == "_INBOX.x" and ops[3][7] == b""
    assert ops[4][6] == b"NATS/1.0\r\nK: V\r\nX: Y\r\n\r\n" and ops[4][7] == b"world"
    assert ops[5][1:5] == ("foo.*", "", "q1", "7")
    assert ops[6][4] == "7" and ops[6][8] == 3
    assert ops[7][1:5] == ("s", "r", "", "1") and ops[7][7] == b"abc"


@settings(max_examples=60, deadline=None)
@given(st.lists(st.binary(min_size=0, max_size=300), min_size=1, max_size=6), st.data())
def test_parser_split_invariance(payloads, data):
    """Any split of the byte stream yields the same ops (partial control lines / payloads)."""
    stream = b"".join(b"PUB s.%d %d\r\n" % (i, len(p)) + p + b"\r\n" for i, p in enumerate(payloads))
    cuts = sorted(data.draw(st.lists(st.integers(0, len(stream)), max_size=8)))
    chunks, prev = [], 0
    for c in cuts:
        chunks.append(stream[prev:c])
        prev = c
    chunks.append(stream[prev:])
    whole = _nc.parse_stream(stream, 1 << 20)
    split = _nc.parse_chunks(chunks)
    assert whole == split
    assert [o[7] for o in whole] == payloads


def test_parser_errors():
    with pytest.raises(RuntimeError, match="Maximum Payload"):
        _nc.parse_stream(b"PUB a 100\r\n" + b"x" * 100 + b"\r\n", 10)
    with pytest.raises(RuntimeError, match="Unknown Protocol"):
        _nc.parse_stream(b"BOGUS x\r\n")


def test_headers_codec():
    h = _nc.build_headers([("A", "1"), ("B", "two")], 503, "No Responders")
    st_, desc, kv = _nc.parse_headers(h)
    assert st_ == 503 and desc == "No Responders" and kv == {"A": "1", "B": "two"}


def test_subject_matching():
    m = _nc.subject_matches
    assert m("a.*.c", "a.b.c") and not m("a.*.c", "a.b.d") and m("a.>", "a.b.c") and not m("a.>", "a")
    assert m("lmstudio.*", "lmstudio.chat_model") and not m("*", "a.b") and m(">", "a.b")


def test_sha256_and_digest():
    import hashlib, base64
    for d in (b"", b"abc", os.urandom(1000)):
        assert _nc.sha256(d) == hashlib.sha256(d).digest()
    d = os.urandom(333)
    assert sha256_digest(d) == "SHA-256=" + base64.urlsafe_b64encode(hashlib.sha256(d).digest()).decode()


# ---------------------------------------------------------------- server + client
def test_pubsub_wildcards_headers(server):
    a, b = client(server), client(server)
    s1 = b.subscribe("x.*")
    s2 = b.subscribe("x.>")
    b.flush()
    a.publish("x.y", b"1")
    a.publish("x.y.z", b"2", headers={"Trace": "t1"})
    a.flush()
    m = s1.next_msg(2)
    assert m.subject == "x.y" and m.data == b"1"
    got = sorted([s2.next_msg(2).data, s2.next_msg(2).data])
    assert got == [b"1", b"2"]
    with pytest.raises(TimeoutError):
        s1.next_msg(0.2)
    a.close(); b.close()


def test_request_reply_and_no_responders(server):
    srv, cli = client(server), client(server)
    srv.subscribe("svc.echo", "g", cb=lambda m: srv.publish(m.reply, b"re:" + m.data, headers={"X": "1"}))
    srv.flush()
    r = cli.request("svc.echo", b"ping", 2)
    assert r.data == b"re:ping" and headers(r) == {"X": "1"}
    with pytest.raises(NoRespondersError):
        cli.request("nobody.home", b"", 1)
    with pytest.raises(RuntimeError, match="maximum payload"):
        cli.publish("big", b"x" * (cli.max_payload + 1))
    srv.close(); cli.close()


def test_auto_reply_static_responder(server):
    """set_auto_reply: requests on the subscription are answered by the reader thread with the stored body (the
    callback never runs); None hands them back to the callback; plain publishes still reach it."""
    srv, cli = client(server), client(server)
    seen = []
    sub = srv.subscribe("svc.static", "g", cb=lambda m: (seen.append(m.data),
                                                          m.reply and srv.publish(m.reply, b"cb")))
    srv.flush()
    sub.set_auto_reply(b"cached")
    assert [cli.request("svc.static", b"q", 2).data for _ in range(3)] == [b"cached"] * 3
    assert sub.auto_replied == 3 and seen == []
    sub.set_auto_reply(b"v2")
    assert cli.request("svc.static", b"q", 2).data == b"v2"
    cli.publish("svc.static", b"no-reply")
    cli.flush()
    for _ in range(100):
        if seen:
            break
        time.sleep(0.01)
    assert seen == [b"no-reply"]
    sub.set_auto_reply(None)
    assert cli.request("svc.static", b"q", 2).data == b"cb" and sub.auto_replied == 4
    srv.close(); cli.close()


def test_concurrent_requests(server):
    srv, cli = client(server), client(server)
    srv.subscribe("add", "", cb=lambda m: srv.publish(m.reply, str(int(m.data) + 1).encode()), workers=4)
    srv.flush()
    out, errs = {}, []

    def go(i):
        try:
            out[i] = int(cli.request("add", str(i).encode(), 5).data)
        except Exception as e:
            errs.append(e)
    ts = [threading.Thread(target=go, args=(i,)) for i in range(64)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs and all(out[i] == i + 1 for i in range(64))
    srv.close(); cli.close()


def test_queue_group_balancing(server):
    cli = client(server)
    counts = [0, 0, 0]
    workers = []
    for k in range(3):
        w = client(server)

        def cb(m, k=k, w=w):
            counts[k] += 1
            w.publish(m.reply, b"ok")
        w.subscribe("work", "pool", cb=cb)
        w.flush()
        workers.append(w)
    for i in range(300):
        cli.request("work", b"x", 2)
    assert sum(counts) == 300 and min(counts) > 40, counts     # each member gets a share, exactly once
    for w in workers:
        w.close()
    cli.close()


def test_unsub_max_and_reconnect(server):
    a, b = client(server), client(server, reconnect_wait=0.05)
    s = b.subscribe("r")
    b._c.unsubscribe(s.sid, 2)
    b.flush()
    for i in range(5):
        a.publish("r", b"%d" % i)
    a.flush()
    assert s.next_msg(1).data == b"0" and s.next_msg(1).data == b"1"
    s3 = b.subscribe("after")
    b.flush()
    server.disconnect_all()        # fault injection: drop every connection
    time.sleep(0.5)
    a2 = client(server)
    deadline = time.time() + 5
    while not b.connected and time.time() < deadline:
        time.sleep(0.05)
    assert b.connected and b.stats()["reconnects"] >= 1
    b.flush()
    a2.publish("after", b"again")
    a2.flush()
    assert s3.next_msg(2).data == b"again"        # subscription re-established after reconnect
    a.close(); a2.close(); b.close()


def test_fault_injection_drop(server):
    srv, cli = client(server), client(server)
    srv.subscribe("svc", "", cb=lambda m: srv.publish(m.reply, b"ok"))
    srv.flush()
    server.set_fault(drop_rate=1.0)
    with pytest.raises(TimeoutError):
        cli.request("svc", b"", 0.3)
    server.set_fault(0.0, delay_ms=50)
    t0 = time.time()
    assert cli.request("svc", b"", 2).data == b"ok"
    assert time.time() - t0 >= 0.05
    server.set_fault(0.0, 0)
    srv.close(); cli.close()


def test_connect_refused():
    with pytest.raises(ConnectionClosedError):
        Client().connect("nats://127.0.0.1:1", timeout=0.5)


# ---------------------------------------------------------------- object store
def test_object_store_roundtrip(server, tmp_path):
    c = client(server)
    os_ = ObjectStore(c, "llm-models")
    os_.create()
    assert os_.exists()
    data = os.urandom(700_000)
    p = tmp_path / "m.gguf"
    p.write_bytes(data)
    info = os_.put_file("pub/model-GGUF/m.gguf", str(p), chunk_size=64 * 1024)
    assert info["size"] == len(data) and info["chunks"] == 11 and info["digest"] == sha256_digest(data)
    assert os_.info("pub/model-GGUF/m.gguf")["nuid"] == info["nuid"]
    out = tmp_path / "o.gguf"
    os_.get_file("pub/model-GGUF/m.gguf", str(out))
    assert out.read_bytes() == data and not (tmp_path / "o.gguf.part").exists()
    assert os_.get_bytes("pub/model-GGUF/m.gguf") == data
    # replace -> old chunks purged, new version served
    info2 = os_.put_bytes("pub/model-GGUF/m.gguf", b"v2" * 1000)
    assert os_.get_bytes("pub/model-GGUF/m.gguf") == b"v2" * 1000 and info2["nuid"] != info["nuid"]
    os_.put_bytes("other/x/y.gguf", b"zz")
    names = sorted(o["name"] for o in os_.list())
    assert names == ["other/x/y.gguf", "pub/model-GGUF/m.gguf"]
    os_.remove("other/x/y.gguf")
    assert [o["name"] for o in os_.list()] == ["pub/model-GGUF/m.gguf"]
    with pytest.raises(RuntimeError, match="not found"):
        os_.info("other/x/y.gguf")
    c.close()


def test_object_store_resume(server, tmp_path):
    c = client(server)
    os_ = ObjectStore(c, "b2")
    os_.create()
    data = os.urandom(300_000)
    info = os_.put_bytes("a/b/c.gguf", data, chunk_size=32 * 1024)
    dest = tmp_path / "c.gguf"
    # simulate an interrupted pull: first 3 chunks already on disk + index
    import json
    part = tmp_path / "c.gguf.part"
    part.write_bytes(data[:3 * 32 * 1024])
    (tmp_path / "c.gguf.part.idx").write_text(json.dumps({"nuid": info["nuid"], "bytes": 3 * 32 * 1024,
                                                          "next_seq": 4, "chunks": 3}))
    os_.get_file("a/b/c.gguf", str(dest), resume=True)
    assert dest.read_bytes() == data
    c.close()


def test_jetstream_persistence(tmp_path):
    store = str(tmp_path / "js")
    s = EmbeddedServer(store_dir=store).start()
    c = Client().connect(s.url)
    o = ObjectStore(c, "persist")
    o.create()
    o.put_bytes("p/m/f.gguf", b"hello world" * 100)
    c.close()
    s.stop()
    s2 = EmbeddedServer(store_dir=store).start()       # restart: bucket content survives
    c2 = Client().connect(s2.url)
    assert ObjectStore(c2, "persist").get_bytes("p/m/f.gguf") == b"hello world" * 100
    c2.close()
    s2.stop()


def test_object_store_get_streams_over_push_consumer(server, tmp_path):
    """get_file streams raw chunks over an ordered push consumer: > 2 flow-control windows (32 MiB
    each) of data, interrupted half way then resumed from the .part checkpoint, digest verified, and
    the ephemeral consumer is gone afterwards (stream consumer_count back to 0)."""
    import hashlib
    import json
    c = client(server)
    os_ = ObjectStore(c, "big")
    os_.create()
    data = os.urandom(80 << 20)
    os_.put_bytes("p/m/big.gguf", data, chunk_size=512 * 1024)
    dest = tmp_path / "big.gguf"

    class Cut(Exception):
        pass

    def cut(got, total):
        if got > total // 2:
            raise Cut()
    with pytest.raises(Exception):
        os_.get_file("p/m/big.gguf", str(dest), True, cut)
    part = (tmp_path / "big.gguf.part").stat().st_size
    assert 0 < part < len(data)
    info = os_.get_file("p/m/big.gguf", str(dest), True)
    assert dest.stat().st_size == len(data) and hashlib.sha256(dest.read_bytes()).digest() == hashlib.sha256(data).digest()
    assert info["digest"] == sha256_digest(data)
    import time
    for _ in range(100):          # the interrupted consumer ends once its inbox has no subscriber
        st = json.loads(c.request("$JS.API.STREAM.INFO.OBJ_big", b"", 5).data)
        if st["state"]["consumer_count"] == 0:
            break
        time.sleep(0.1)
    assert st["state"]["consumer_count"] == 0
    c.close()


def test_sha256_matches_hashlib():
    import hashlib
    from nats_llm_studio_amd.natsio import _natscore as n
    for L in (0, 1, 55, 56, 63, 64, 65, 127, 128, 129, 1000, 65536 + 7):
        b = os.urandom(L)
        assert n.sha256(b) == hashlib.sha256(b).digest(), L


# ---------------------------------------------------------------- authentication
def test_nkeys_sign_verify_roundtrip():
    from nats_llm_studio_amd.natsio import _natscore as n, nkey_keypair
    seed, pub = nkey_keypair(bytes(range(32)))
    assert seed.startswith("SU") and pub.startswith("U") and len(pub) == 56 and len(seed) == 58
    assert nkey_keypair(bytes(range(32))) == (seed, pub)            # deterministic from the raw seed
    sig = n.nkey_sign(seed, b"nonce-123")
    assert len(sig) == 64 and n.nkey_verify(pub, b"nonce-123", sig)
    assert not n.nkey_verify(pub, b"nonce-124", sig)
    bad = bytes([sig[0] ^ 1]) + sig[1:]
    assert not n.nkey_verify(pub, b"nonce-123", bad)
    with pytest.raises(Exception):
        n.nkey_public(seed[:-1] + ("A" if seed[-1] != "A" else "B"))   # checksum mismatch


def test_server_auth_token_user_nkey(tmp_path):
    from nats_llm_studio_amd.natsio import _natscore as n, nkey_keypair
    seed, pub = nkey_keypair()
    other_seed, _ = nkey_keypair()
    s = EmbeddedServer(auth_token="s3cret", users=[("alice", "pw")], nkeys=[pub]).start()
    try:
        url = s.url
        ok = [Client().connect(url, token="s3cret", reconnect=False),
              Client().connect(url.replace("nats://", "nats://alice:pw@"), reconnect=False),
              Client().connect(url, nkey_seed=seed, reconnect=False)]
        creds = tmp_path / "u.creds"
        creds.write_text("-----BEGIN NATS USER JWT-----\neyJhbGciOi.fake.jwt\n------END NATS USER JWT------\n\n"
                         "************************* IMPORTANT *************************\n"
                         f"-----BEGIN USER NKEY SEED-----\n{seed}\n------END USER NKEY SEED------\n")
        assert n.parse_creds(creds.read_text()) == ("eyJhbGciOi.fake.jwt", seed)
        for c in ok:
            sub = c.subscribe("auth.echo", cb=lambda m, c=c: c.publish(m.reply, m.data))
            c.flush()
            assert c.request("auth.echo", b"hi", 2).data == b"hi"
            sub.unsubscribe()
            c.close()
        for kw in (dict(token="wrong"), dict(user="alice", password="nope"), dict(nkey_seed=other_seed), {}):
            with pytest.raises(Exception, match="Authorization|cannot connect|timeout|closed"):
                Client().connect(url, reconnect=False, timeout=1.0, **kw)
    finally:
        s.stop()


def test_flush_waits_for_server_after_connect():
    """flush() must not return on the PONG of the CONNECT handshake PING (which once ran the
    PONG count one ahead): a SUB followed by flush() is registered before the peer publishes."""
    lost = 0
    for _ in range(40):
        s = EmbeddedServer().start()
        a, b = client(s), client(s)
        sub = b.subscribe("x.*")
        b.flush()
        a.publish("x.y", b"1")
        a.flush()
        try:
            sub.next_msg(2)
        except TimeoutError:
            lost += 1
        a.close(); b.close(); s.stop()
    assert lost == 0
