"""bench.py contract on CPU (gloo): `--gpus N` starts N ranks itself when no launcher set
WORLD_SIZE, TP/EP replicas replay the leader's steps, and rank 0 prints ONE JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, *args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "3", "--warmup", "1",
           "--concurrency", "4", "--prompt-len", "16", "--no-rtt", "--model-dir", str(tmp_path), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("extra,par,scaling", [
    (["--gpus", "2", "--tp", "2", "--model", "tiny-llama-tp"], "tp2", "strong"),
    (["--gpus", "2", "--model", "tiny-llama-tp", "--tp-leg", "0"], "dp2", "weak"),
    (["--gpus", "2", "--tp", "2", "--ep", "--model", "tiny-mixtral-tp"], "tp2+ep", "strong"),
])
def test_bench_spawns_ranks(tmp_path, extra, par, scaling):
    out = _bench(tmp_path, *extra)
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == par
    assert out["scaling"] == scaling
    assert out["steps"] == 3 and out["value"] > 0
    if "tp" in par:
        assert out["comm"]["all_reduce_per_step"] > 0
    assert out["config"]["global_batch"] == (4 if "tp" in par else 8)


def test_bench_dp_run_adds_tp_leg(tmp_path):
    """--gpus N (dp, the driver's scaling run) also reports a tensor-parallel leg over all N ranks on the
    70B per-layer shapes (CPU: one layer) with its all-reduce accounting: 2 row-parallel sums of 8192
    fp32 per layer and token, plus the vocab-parallel argmax."""
    out = _bench(tmp_path, "--gpus", "4", "--model", "tiny-llama-tp", "--tp-leg-concurrency", "2")
    assert out["config"]["parallelism"] == "dp4" and out["value"] > 0
    tl = out["tp_leg"]
    assert tl["parallelism"] == "tp4" and tl["model"].startswith("llama-3-70b-1layer") and tl["value"] > 0
    c = tl["comm"]
    assert c["all_reduce_per_step"] >= 3 and c["all_reduce_bytes_per_step"] >= 2 * 2 * 8192 * 4
    assert c["oneshot"] is False and c["ctrl_transport"] == "shm-ring"


def test_bench_tp_leg_time_limit(tmp_path):
    """A TP leg that overruns its limit costs the leg only: its whole process group (launcher + ranks) is killed
    and the headline line still comes out."""
    out = _bench(tmp_path, "--gpus", "2", "--model", "tiny-llama-tp", "--tp-leg-timeout", "1")
    assert out["config"]["parallelism"] == "dp2" and out["value"] > 0
    assert "process group killed" in out["tp_leg"]["error"], out["tp_leg"]


def test_bench_rejects_mismatched_world(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_service_load_generator_cpu(tiny_models):
    """The bench's service-path burst: concurrent chat_model requests (half sampled) all answered 200
    through natscore by the real engine, tokens counted from the replies' usage."""
    from nats_llm_studio_amd.engine.engine import Engine
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.llama import LlamaModel
    from nats_llm_studio_amd.service.bench_rtt import measure_engine_chat_load
    r = GGUFReader(tiny_models["tiny-llama"])
    eng = Engine(LlamaModel(r, "cpu"), None, max_batch=8, use_graphs=False, ctx=512)
    out = measure_engine_chat_load(eng, r.metadata, n=8, max_tokens=3, prompt_tokens=32)
    assert out["complete"] and out["ok"] == 8 and out["completion_tokens"] == 24 == out["completion_tokens_requested"]
    assert out["tok_s"] > 0 and out["rtt_p99_ms"] >= out["rtt_p50_ms"]
    assert 16 <= out["prompt_tokens_mean"] <= 64
    ph = out["phases_ms"]
    for k in ("validate", "tokenize", "queue", "prefill", "decode", "respond", "total"):
        assert ph[k]["count"] == 8, (k, ph)
    assert out["engine"]["prefill_tokens"] >= 8 * 16


def test_gpu_telemetry_summary_without_periodic_samples():
    """A timed region shorter than the sampling period still reports its clocks (from the begin / end snapshots) and
    the power-limit residency from the accumulated counters."""
    from nats_llm_studio_amd.utils.telemetry import GpuTelemetry
    t = GpuTelemetry.__new__(GpuTelemetry)
    t.h, t.err, t.samples = object(), None, []
    t.begin = dict(gfx_mhz=2200, mem_mhz=2000, power_w=600, hotspot_c=50, accumulation_counter=100,
                   ppt_residency_acc=10, socket_thm_residency_acc=0)
    t.end = dict(gfx_mhz=2000, mem_mhz=2000, power_w=1200, hotspot_c=52, accumulation_counter=300,
                 ppt_residency_acc=110, socket_thm_residency_acc=0)
    s = t.summary()
    assert s["gfx_mhz"] == {"min": 2000, "mean": 2100.0, "max": 2200}
    assert s["ppt_limited_frac"] == 0.5 and s["thermal_limited_frac"] == 0.0
    assert "accumulation_counter" not in s["begin"]
