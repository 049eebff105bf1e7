"""EngineBackend model lifecycle under concurrency (CPU engine over the embedded NATS server):
a JIT load never blocks list_models / health, an evicted or deleted model keeps serving the
chats already running on it, and a stopped engine refuses new work instead of parking it.

The reference's list_models handler has a 30 s context (`/root/reference/nats_llm_studio.go:229`)
and its chat handler 2 min (`:328`); neither may be starved by a model load."""
import json
import shutil
import statistics
import threading
import time

import pytest

from nats_llm_studio_amd.natsio import Client, EmbeddedServer
from nats_llm_studio_amd.service.config import WorkerConfig
from nats_llm_studio_amd.service.service import Service


def req(cli, name, payload, timeout=60):
    return json.loads(cli.request(f"lmstudio.{name}", json.dumps(payload).encode(), timeout).data)


def _tree(tmp_path, tiny_models, names):
    for n in names:
        d = tmp_path / "models" / "synthetic" / f"{n}-GGUF"
        d.mkdir(parents=True)
        shutil.copy(tiny_models[n], d / f"{n}-Q4_K_M.gguf")
    return str(tmp_path / "models")


@pytest.fixture()
def svc_env(tmp_path, tiny_models):
    srv = EmbeddedServer().start()
    cfg = WorkerConfig(nats_url=srv.url, models_dir=_tree(tmp_path, tiny_models, ["tiny-llama", "tiny-qwen2"]),
                       backend="engine", device="cpu", max_batch=8, max_ctx=256, max_loaded_models=1)
    svc = Service(cfg).start()
    cli = Client().connect(srv.url)
    yield svc, cli
    cli.close()
    svc.stop()
    svc.client.close()
    srv.stop()


def test_list_models_not_blocked_by_load(svc_env):
    svc, cli = svc_env
    be = svc.backend
    orig = be.build_state

    def slow_build(*a, **k):               # a 70B-sized load, simulated
        time.sleep(3.0)
        return orig(*a, **k)
    be.build_state = slow_build
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("r", req(cli, "chat_model", {
        "model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 2})))
    t.start()
    t_end = time.time() + 10
    while not be.stats()["loading"] and time.time() < t_end:   # handler dispatch + first imports
        time.sleep(0.02)
    assert be.stats()["loading"] == ["tiny-llama"]
    lat = []
    for _ in range(50):
        t0 = time.perf_counter()
        r = req(cli, "list_models", {}, timeout=5)
        lat.append((time.perf_counter() - t0) * 1e3)
        assert r["ok"]
    assert be.stats()["loading"] == ["tiny-llama"], "the load finished before the measurement ended"
    p50 = statistics.median(lat)
    assert p50 < 5.0, f"list_models p50 {p50:.3f} ms during a model load"
    t.join(60)
    assert out["r"]["data"]["http_status"] == 200


def test_eviction_keeps_inflight_chats(svc_env):
    """max_loaded_models=1, chats running on two models at once: every chat gets a 200 with its
    full token budget; the evicted model is unloaded only after its chats finished."""
    svc, cli = svc_env
    res = {}

    def chat(i, model):
        res[i] = req(cli, "chat_model", {"model": model, "messages": [{"role": "user", "content": f"q{i}"}],
                                         "max_tokens": 48, "ignore_eos": True, "temperature": 0}, timeout=120)
    ts = [threading.Thread(target=chat, args=(i, "tiny-llama")) for i in range(3)]
    [t.start() for t in ts]
    time.sleep(0.5)
    ts2 = [threading.Thread(target=chat, args=(10 + i, "tiny-qwen2")) for i in range(2)]
    [t.start() for t in ts2]
    [t.join(120) for t in ts + ts2]
    assert sorted(res) == [0, 1, 2, 10, 11]
    for r in res.values():
        assert r["ok"] and r["data"]["http_status"] == 200, r
        assert r["data"]["response"]["usage"]["completion_tokens"] == 48
    assert svc.backend.loaded_ids() == ["tiny-qwen2"]


def test_stopped_engine_refuses_requests(tiny_models):
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.llama import LlamaModel
    eng = Engine(LlamaModel(GGUFReader(tiny_models["tiny-llama"]), "cpu"), None, max_batch=2, use_graphs=False,
                 ctx=128, num_blocks=32)
    eng.start()
    eng.unload()
    fut = eng.submit(GenRequest([1, 2, 3]))
    with pytest.raises(RuntimeError, match="not running"):
        fut.result(timeout=5)


def test_concurrent_first_loads_of_two_models_are_serialised(svc_env):
    """max_loaded_models=1 and the first chats for TWO different models arrive together: the two
    builds must not overlap (each sizes device memory at build time), the second build evicts the
    first model only after it is done, and both chats are answered."""
    svc, cli = svc_env
    be = svc.backend
    orig = be.build_state
    active, peak = [0], [0]
    lk = threading.Lock()

    def slow_build(*a, **k):
        with lk:
            active[0] += 1
            peak[0] = max(peak[0], active[0])
        try:
            time.sleep(1.0)
            return orig(*a, **k)
        finally:
            with lk:
                active[0] -= 1
    be.build_state = slow_build
    res = {}

    def chat(model):
        res[model] = req(cli, "chat_model", {"model": model, "messages": [{"role": "user", "content": "hi"}],
                                             "max_tokens": 4, "ignore_eos": True, "temperature": 0}, timeout=120)
    ts = [threading.Thread(target=chat, args=(m,)) for m in ("tiny-llama", "tiny-qwen2")]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    assert peak[0] == 1, "two model builds overlapped"
    for r in res.values():
        assert r["ok"] and r["data"]["http_status"] == 200, r
        assert r["data"]["response"]["usage"]["completion_tokens"] == 4
    assert len(be.loaded_ids()) == 1


def test_chat_deadline_covers_jit_load(svc_env):
    """The chat context starts at receipt and includes the JIT load (reference: 2 min, nats_llm_studio.go:328):
    a load slower than the context answers with the deadline envelope; the build completes in the background,
    releases the abandoned request's pin, and serves the next chat."""
    svc, cli = svc_env
    be = svc.backend
    orig = be.build_state

    def slow_build(*a, **k):
        time.sleep(2.0)
        return orig(*a, **k)
    be.build_state = slow_build
    svc.cfg.timeout_chat = 0.5
    body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 2}
    t0 = time.time()
    r = req(cli, "chat_model", body)
    assert time.time() - t0 < 1.8
    assert r == {"ok": False, "error": "context deadline exceeded", "data": {"http_status": 0}}, r
    t_end = time.time() + 20
    while be.loaded_ids() != ["tiny-llama"] and time.time() < t_end:
        time.sleep(0.05)
    assert be.loaded_ids() == ["tiny-llama"]
    svc.cfg.timeout_chat = 120.0
    r = req(cli, "chat_model", body)
    assert r["ok"] is True and r["data"]["http_status"] == 200, r
    time.sleep(0.2)
    assert be.stats()["models"]["tiny-llama"]["inflight"] == 0      # the abandoned pin was released
