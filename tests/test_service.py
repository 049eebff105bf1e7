"""End-to-end service tests over the embedded NATS server (BASELINE config 1 + the model
lifecycle). Error strings are the reference's (nats_llm_studio.go:256-344)."""
import json
import os
import shutil
import threading
import time

import pytest

from nats_llm_studio_amd.natsio import Client, EmbeddedServer, NoRespondersError, ObjectStore
from nats_llm_studio_amd.service.config import WorkerConfig
from nats_llm_studio_amd.service.service import Service


@pytest.fixture()
def env(tmp_path):
    srv = EmbeddedServer().start()
    cfg = WorkerConfig(nats_url=srv.url, models_dir=str(tmp_path / "models"), backend="stub")
    os.makedirs(cfg.models_dir)
    svc = Service(cfg).start()
    cli = Client().connect(srv.url)
    yield srv, cfg, svc, cli
    cli.close()
    svc.stop()
    svc.client.close()
    srv.stop()


def req(cli, name, payload, timeout=10):
    data = payload if isinstance(payload, bytes) else json.dumps(payload).encode()
    return json.loads(cli.request(f"lmstudio.{name}", data, timeout).data)


def test_list_models_empty(env):
    _, _, _, cli = env
    r = req(cli, "list_models", {})
    assert r == {"ok": True, "data": {"http_status": 200, "models": {"object": "list", "data": []}}}


@pytest.mark.parametrize("subject,payload,err", [
    ("pull_model", b"{bad", "invalid JSON in PullModel: invalid character 'b' looking for beginning of object key string"),
    ("pull_model", b"{}", "'identifier' is required"),
    ("pull_model", b'{"identifier": 5}',
     "invalid JSON in PullModel: json: cannot unmarshal number into Go struct field PullModelRequest.identifier of type string"),
    ("delete_model", b"nope", "invalid JSON in DeleteModel: invalid character 'o' in literal null (expecting 'u')"),
    ("delete_model", b'{"model_id": ""}', "'model_id' is required"),
    ("chat_model", b"", "payload vazio em ChatModel"),
    ("chat_model", b"[", "invalid JSON in ChatModel: unexpected end of JSON input"),
    ("chat_model", b'{"messages": []}', "'model' is required in ChatModel"),
])
def test_validation_errors(env, subject, payload, err):
    _, _, _, cli = env
    r = req(cli, subject, payload)
    if subject == "delete_model" and payload == b"nope":
        assert r["ok"] is False and r["error"].startswith("invalid JSON in DeleteModel: invalid character")
    else:
        assert r == {"ok": False, "error": err, "data": None}


def test_chat_stub_echo(env):
    _, _, _, cli = env
    r = req(cli, "chat_model", {"model": "granite-3.0-2b-instruct",
                                "messages": [{"role": "system", "content": "x"},
                                             {"role": "user", "content": "hello over nats"}]})
    assert r["ok"] is True and r["data"]["http_status"] == 200
    resp = r["data"]["response"]
    assert resp["object"] == "chat.completion" and resp["choices"][0]["message"]["content"] == "hello over nats"
    assert resp["usage"]["completion_tokens"] == 3 and "stats" in resp and "model_info" in resp
    bad = req(cli, "chat_model", {"model": "m", "messages": "notalist"})
    assert bad["ok"] is True and bad["data"]["http_status"] == 400     # backend status, not bridge status


def test_metrics_health(env):
    _, _, svc, cli = env
    req(cli, "list_models", {})                      # native responder
    svc.native_list(False)
    req(cli, "list_models", {})                      # the Python handler
    for _ in range(50):   # the handler records its latency just after it has replied
        m = req(cli, "metrics", {})
        if "list_models" in m["data"]["latency_ms"]:
            break
        time.sleep(0.01)
    r = m["data"]["requests"]
    assert m["ok"] and r["list_models"] == 2 and r["list_models_native"] == 1, r
    assert "p50" in m["data"]["latency_ms"]["list_models"]
    h = req(cli, "health", {})
    assert h["data"]["status"] == "ok" and h["data"]["backend"] == "stub"


def test_list_models_native_matches_handler(env, tiny_models):
    """The native list_models reply (client reader thread, cached registry body) is byte-identical to the
    handler's, and a listing requested right after a pull / delete reply already shows the change (the body is
    refreshed before the service sends any reply)."""
    srv, cfg, svc, cli = env
    raw = lambda: cli.request("lmstudio.list_models", b"{}", 10).data
    empty = raw()
    svc.native_list(False)
    assert raw() == empty
    svc.native_list(True)
    _push_tiny(srv.url, tiny_models["tiny-llama"], "synthetic/tiny-llama-GGUF/tiny-llama-Q4_K_M.gguf")
    assert req(cli, "pull_model", {"identifier": "synthetic/tiny-llama"}, timeout=60)["ok"]
    one = raw()
    assert [m["id"] for m in json.loads(one)["data"]["models"]["data"]] == ["tiny-llama"]
    svc.native_list(False)
    assert raw() == one
    svc.native_list(True)
    n0 = svc._list_sub.auto_replied
    assert req(cli, "delete_model", {"model_id": "tiny-llama"})["ok"]
    assert raw() == empty and svc._list_sub.auto_replied == n0 + 1


def _push_tiny(srv_url, tiny_path, name):
    c = Client().connect(srv_url)
    o = ObjectStore(c, "llm-models")
    o.create()
    info = o.put_file(name, tiny_path)
    c.close()
    return info


def test_pull_list_delete_lifecycle(env, tiny_models):
    srv, cfg, svc, cli = env
    name = "synthetic/tiny-llama-GGUF/tiny-llama-Q4_K_M.gguf"
    info = _push_tiny(srv.url, tiny_models["tiny-llama"], name)
    r = req(cli, "pull_model", {"identifier": "synthetic/tiny-llama"}, timeout=60)
    assert r["ok"] is True and r["data"]["model"] == "synthetic/tiny-llama", r
    local = os.path.join(cfg.models_dir, "synthetic", "tiny-llama-GGUF", "tiny-llama-Q4_K_M.gguf")
    assert os.path.getsize(local) == info["size"]
    lst = req(cli, "list_models", {})["data"]["models"]["data"]
    assert [m["id"] for m in lst] == ["tiny-llama"]
    m = lst[0]
    assert m["publisher"] == "synthetic" and m["arch"] == "llama" and m["quantization"] == "Q4_K_M"
    assert m["state"] == "not-loaded" and m["max_context_length"] == 512
    # unknown model
    r = req(cli, "pull_model", {"identifier": "nobody/nothing"})
    assert r["ok"] is False and r["data"]["model"] == "nobody/nothing" and "not found" in r["error"]
    # delete
    r = req(cli, "delete_model", {"model_id": "tiny-llama"})
    assert r["ok"] is True and r["data"] == {"model_id": "tiny-llama",
                                            "deleted_dir": os.path.join(cfg.models_dir, "synthetic", "tiny-llama-GGUF")}
    assert not os.path.exists(local)
    r = req(cli, "delete_model", {"model_id": "tiny-llama"})
    assert r["ok"] is False and r["data"] == {"model_id": "tiny-llama", "dir": ""}


def test_sync_model_from_bucket(env, tiny_models):
    srv, cfg, svc, cli = env
    _push_tiny(srv.url, tiny_models["tiny-granite"], "ibm/granite/granite.gguf")
    r = req(cli, "sync_model_from_bucket", {"bucket": "llm-models", "object_name": "ibm/granite/granite.gguf",
                                            "publisher": "ibm", "model_dir": "granite-3.0-2b"}, timeout=60)
    assert r["ok"] and r["data"]["local_path"].endswith("ibm/granite-3.0-2b/model.gguf")
    ids = [m["id"] for m in req(cli, "list_models", {})["data"]["models"]["data"]]
    assert ids == ["granite-3.0-2b"]
    r = req(cli, "sync_model_from_bucket", {"object_name": "x"})
    assert r == {"ok": False, "error": "'publisher' is required", "data": None}


def test_delete_refuses_escape(env):
    _, cfg, svc, cli = env
    assert not svc.registry.safe_dir(cfg.models_dir)
    assert not svc.registry.safe_dir("/etc")
    assert svc.registry.safe_dir(os.path.join(cfg.models_dir, "a", "b"))


def test_queue_group_scale_out(env):
    srv, cfg, svc, cli = env
    svc2 = Service(cfg).start()          # second worker, same queue group
    try:
        for _ in range(200):
            assert req(cli, "list_models", {})["ok"]
        n1, n2 = svc._request_counts()["list_models"], svc2._request_counts()["list_models"]
        assert n1 > 20 and n2 > 20 and n1 + n2 == 200, (n1, n2)
    finally:
        svc2.stop()
        svc2.client.close()


def test_no_responders_when_down(tmp_path):
    srv = EmbeddedServer().start()
    cli = Client().connect(srv.url)
    with pytest.raises(NoRespondersError):
        cli.request("lmstudio.list_models", b"{}", 1)
    cli.close()
    srv.stop()


def test_engine_backend_chat_cpu(tmp_path, tiny_models):
    srv = EmbeddedServer().start()
    md = tmp_path / "models" / "synthetic" / "tiny-llama-GGUF"
    md.mkdir(parents=True)
    shutil.copy(tiny_models["tiny-llama"], md / "tiny-llama-Q4_K_M.gguf")
    cfg = WorkerConfig(nats_url=srv.url, models_dir=str(tmp_path / "models"), backend="engine", device="cpu",
                       max_batch=8, max_ctx=256)
    svc = Service(cfg).start()
    cli = Client().connect(srv.url)
    try:
        body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "Hello!"}], "max_tokens": 5,
                "temperature": 0}
        out = {}

        def go(i):
            out[i] = req(cli, "chat_model", dict(body, seed=i), timeout=120)
        ts = [threading.Thread(target=go, args=(i,)) for i in range(4)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        for i in range(4):
            r = out[i]
            assert r["ok"] and r["data"]["http_status"] == 200, r
            resp = r["data"]["response"]
            assert resp["usage"]["completion_tokens"] <= 5 and resp["model_info"]["quant"] == "Q4_K_M"
        texts = {out[i]["data"]["response"]["choices"][0]["message"]["content"] for i in range(4)}
        assert len(texts) == 1                         # greedy: identical answers for identical prompts
        lst = req(cli, "list_models", {})["data"]["models"]["data"]
        assert lst[0]["state"] == "loaded"
        tr = req(cli, "metrics", {})["data"]["trace"]      # recv->validate->queue->prefill->decode->respond
        assert {"validate", "queue", "prefill", "decode", "respond", "total"} <= set(tr["phases_ms"])
        assert tr["phases_ms"]["total"]["count"] == 4 and tr["recent"][-1]["request_id"].startswith("req-")
        r = req(cli, "chat_model", {"model": "missing-model", "messages": [{"role": "user", "content": "x"}]})
        assert r["ok"] and r["data"]["http_status"] == 404
        r = req(cli, "delete_model", {"model_id": "tiny-llama"})       # unloads then deletes
        assert r["ok"] and svc.backend.loaded_ids() == []
    finally:
        cli.close()
        svc.stop()
        svc.client.close()
        srv.stop()


class _FakeLMStudio:
    """Minimal LM Studio REST v0 stand-in for the `http` backend (the reference's own mode)."""

    def __init__(self):
        import http.server

        outer = self
        self.bodies = []

        class H(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body: bytes):
                self.send_response(code)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path == "/api/v0/models":
                    self._send(200, b'{"object":"list","data":[{"id":"m1","object":"model","state":"loaded"}]}')
                else:
                    self._send(404, b'{"error":"nope"}')

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                body = self.rfile.read(n)
                outer.bodies.append((self.headers.get("Content-Type"), body))
                req = json.loads(body)
                if req.get("model") == "missing":
                    self._send(404, b'{"error":"Model not found"}')
                elif req.get("model") == "garbage":
                    self._send(200, b"data: not json")
                else:
                    self._send(200, json.dumps({"object": "chat.completion", "model": req["model"],
                                                "choices": [{"message": {"role": "assistant", "content": "hi"}}]}).encode())

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


def test_http_backend_total_deadline_against_a_dripping_server():
    """The reference's context bounds the WHOLE request (`nats_llm_studio.go:36`, `:229`): a server that drips
    one byte every 50 ms (each socket read well inside urllib's per-operation timeout) is cut at the deadline."""
    import http.server
    import time as _t
    from nats_llm_studio_amd.service.backends import HttpBackend

    class Drip(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            self.send_response(200)
            self.send_header("Content-Length", "1000")
            self.end_headers()
            try:
                for _ in range(1000):
                    self.wfile.write(b" ")
                    self.wfile.flush()
                    _t.sleep(0.05)
            except OSError:
                pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Drip)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        be = HttpBackend(f"http://127.0.0.1:{srv.server_address[1]}", timeout=120)
        t0 = _t.monotonic()
        with pytest.raises(TimeoutError):
            be.list_models_raw(timeout=0.6)
        assert _t.monotonic() - t0 < 2.0
    finally:
        srv.shutdown()


def test_http_backend_proxy_semantics(tmp_path):
    """backend=http reproduces nats_llm_studio.go:136-179/228-364: raw bodies embedded, status
    NOT checked (404 -> ok:true + http_status 404), payload forwarded verbatim as JSON, a
    non-JSON body -> the literal marshal-failure fallback, transport failure -> http_status 0."""
    lm = _FakeLMStudio()
    srv = EmbeddedServer().start()
    cfg = WorkerConfig(nats_url=srv.url, models_dir=str(tmp_path), backend="http", lmstudio_base_url=lm.url)
    svc = Service(cfg).start()
    cli = Client().connect(srv.url)
    try:
        r = req(cli, "list_models", {})
        assert r == {"ok": True, "data": {"http_status": 200, "models": {
            "object": "list", "data": [{"id": "m1", "object": "model", "state": "loaded"}]}}}
        raw = b'{"model": "m1",   "messages": [{"role": "user", "content": "x"}], "extra": 1}'
        r = req(cli, "chat_model", raw)
        assert r["ok"] is True and r["data"]["http_status"] == 200
        assert r["data"]["response"]["choices"][0]["message"]["content"] == "hi"
        assert lm.bodies[-1] == ("application/json", raw)
        r = req(cli, "chat_model", {"model": "missing"})
        assert r == {"ok": True, "data": {"http_status": 404, "response": {"error": "Model not found"}}}
        r = cli.request("lmstudio.chat_model", b'{"model": "garbage"}', 10).data
        assert bytes(r) == b'{"ok":false,"error":"internal error serializing response"}'
        lm.close()
        svc.backend.base = "http://127.0.0.1:1"           # nothing listens: transport error
        r = req(cli, "chat_model", {"model": "m1"})
        assert r["ok"] is False and r["error"].startswith("error calling LM Studio:")
        assert r["data"] == {"http_status": 0}
    finally:
        cli.close()
        svc.stop()
        svc.client.close()
        srv.stop()


def test_engine_chat_rtt_helper(tiny_models):
    """bench.py's chat_model RTT against a real engine (CPU here, the 8B GPU engine in the bench)."""
    from nats_llm_studio_amd.engine.engine import Engine
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.llama import LlamaModel
    from nats_llm_studio_amd.service.bench_rtt import measure_engine_chat_rtt
    r = GGUFReader(tiny_models["tiny-llama"])
    eng = Engine(LlamaModel(r, "cpu"), None, max_batch=4, ctx=256, num_blocks=64, use_graphs=False)
    out = measure_engine_chat_rtt(eng, r.metadata, model_id="tiny-llama", n=3, warmup=1)
    assert out["n"] == 3 and 0 < out["p50_ms"] <= out["p99_ms"] and out["prompt_tokens"] > 0
    assert eng.thread is None


def test_pull_deadline_stalled_bucket_then_resume(env, tiny_models):
    """pull_model runs under its handler context (reference: 10 min, nats_llm_studio.go:251): a stalled bucket
    (every client publish delayed by the embedded server's fault injection) answers ok:false with the deadline
    error instead of hanging, and the next pull completes."""
    srv, cfg, svc, cli = env
    name = "synthetic/tiny-llama-GGUF/tiny-llama-Q4_K_M.gguf"
    _push_tiny(srv.url, tiny_models["tiny-llama"], name)
    cfg.timeout_pull = 1.0
    srv.set_fault(0.0, delay_ms=400)
    try:
        t0 = time.time()
        r = req(cli, "pull_model", {"identifier": "synthetic/tiny-llama"}, timeout=30)
        took = time.time() - t0
    finally:
        srv.set_fault(0.0, 0)
    assert r["ok"] is False and "context deadline exceeded" in r["error"], r
    assert r["data"]["model"] == "synthetic/tiny-llama"
    assert took < 10, took
    cfg.timeout_pull = 600.0
    r = req(cli, "pull_model", {"identifier": "synthetic/tiny-llama"}, timeout=60)
    assert r["ok"] is True, r
    local = os.path.join(cfg.models_dir, "synthetic", "tiny-llama-GGUF", "tiny-llama-Q4_K_M.gguf")
    assert os.path.getsize(local) == os.path.getsize(tiny_models["tiny-llama"])


def test_list_and_delete_deadlines(env):
    """list_models (30 s) and delete_model (2 min) contexts: a stuck registry read / engine unload answers
    with the deadline error at the configured bound."""
    srv, cfg, svc, cli = env
    d = os.path.join(cfg.models_dir, "synthetic", "slow-GGUF")
    os.makedirs(d)
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    write_synthetic_gguf(os.path.join(d, "slow-Q4_K_M.gguf"), "tiny-llama", "Q4_K_M")
    real_list = svc.registry.list_api
    svc.native_list(False)                # the handler path holds the 30 s context (the native reply never waits)
    cfg.timeout_list = 0.3
    svc.registry.list_api = lambda *a, **k: (time.sleep(2.0), real_list(*a, **k))[1]
    svc._list_cache = {}                  # a registry snapshot not encoded yet (the slow read runs)
    r = req(cli, "list_models", {})
    assert r == {"ok": False, "error": "error reading model registry: context deadline exceeded",
                 "data": {"http_status": 0}}
    svc.registry.list_api = real_list
    cfg.timeout_delete = 0.3
    real_unload = svc.backend.unload
    svc.backend.unload = lambda mid: time.sleep(2.0)
    r = req(cli, "delete_model", {"model_id": "slow"})
    assert r["ok"] is False and r["error"] == "context deadline exceeded", r
    assert os.path.isdir(d)               # the reply says what happened: a timed-out delete removes nothing
    svc.backend.unload = real_unload
    cfg.timeout_delete = 120.0
    time.sleep(2.2)                       # the timed-out unload finished in the background
    assert os.path.isdir(d)
    r = req(cli, "delete_model", {"model_id": "slow"})
    assert r["ok"] is True and r["data"]["deleted_dir"] == d, r
    assert not os.path.exists(d)
