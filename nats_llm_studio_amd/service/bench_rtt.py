"""p50/p99 NATS request-reply RTT (BASELINE metric, config 1): embedded server + worker with the
CPU stub backend, measured from a native client (C++ timing loop, no Python in the timed path
on the requesting side; the worker's handlers run in Python)."""
from __future__ import annotations

import json
import statistics
import tempfile


def _pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(p / 100.0 * (len(xs) - 1))))]


def measure_rtt(n: int = 1000, warmup: int = 100) -> dict:
    from ..natsio import Client, EmbeddedServer
    from .config import WorkerConfig
    from .service import Service
    out = {}
    with tempfile.TemporaryDirectory() as d:
        srv = EmbeddedServer().start()
        cfg = WorkerConfig(nats_url=srv.url, models_dir=d, backend="stub")
        svc = Service(cfg).start()
        cli = Client().connect(srv.url)
        try:
            for subj, payload in (("lmstudio.list_models", b"{}"),
                                  ("lmstudio.chat_model", json.dumps({"model": "granite-3.0-2b-instruct", "messages": [
                                      {"role": "user", "content": "ping"}]}).encode())):
                cli._c.bench_requests(subj, payload, warmup, 5000)
                us = cli._c.bench_requests(subj, payload, n, 5000)
                out[subj.split(".")[1]] = {"p50_ms": round(_pct(us, 50) / 1e3, 4), "p99_ms": round(_pct(us, 99) / 1e3, 4),
                                           "mean_ms": round(statistics.mean(us) / 1e3, 4), "n": n}
            # raw wire RTT (echo responder in C++ client threads, no service logic)
            echo = Client().connect(srv.url)
            echo.subscribe("rtt.echo", "", cb=lambda m: echo.publish(m.reply, m.data))
            echo.flush()
            us = cli._c.bench_requests("rtt.echo", b"{}", n, 5000)
            out["wire_echo"] = {"p50_ms": round(_pct(us, 50) / 1e3, 4), "p99_ms": round(_pct(us, 99) / 1e3, 4), "n": n}
            echo.close()
        finally:
            cli.close()
            svc.stop()
            svc.client.close()
            srv.stop()
    out["p50_ms"] = out["list_models"]["p50_ms"]
    return out


def measure_engine_chat_rtt(engine, metadata: dict, model_id: str = "llama-3-8b", n: int = 50, warmup: int = 5,
                            max_tokens: int = 1) -> dict:
    """p50/p99 of `lmstudio.chat_model` request-reply against the REAL engine (GPU model in
    `engine`): NATS -> validation -> chat template -> tokenize -> continuous-batching engine
    (prefill + `max_tokens` decode) -> LM-Studio-shaped reply, timed by the native client."""
    from ..natsio import Client, EmbeddedServer
    from ..tokenizer.bpe import tokenizer_from_metadata
    from ..tokenizer.chat_template import ChatTemplate, default_template
    from .backends import EngineBackend
    from .config import WorkerConfig
    from .registry import ModelEntry
    from .service import Service
    tok = tokenizer_from_metadata(metadata)
    tmpl = metadata.get("tokenizer.chat_template") or default_template(engine.cfg.arch,
                                                                       metadata.get("tokenizer.ggml.model", "gpt2"))
    bos = tok.tokens[tok.bos_id] if tok.bos_id is not None else ""
    eos = tok.tokens[tok.eos_id] if tok.eos_id is not None else ""
    engine.tok = tok
    started = engine.thread is None
    engine.start()
    with tempfile.TemporaryDirectory() as d:
        srv = EmbeddedServer().start()
        cfg = WorkerConfig(nats_url=srv.url, models_dir=d, backend="engine")
        backend = EngineBackend(cfg)
        entry = ModelEntry(id=model_id, publisher="synthetic", model_dir=model_id, path="", dir=d,
                           arch=engine.cfg.arch, quantization="Q4_K_M", max_context_length=engine.ctx)
        backend.adopt({"engine": engine, "tok": tok, "tmpl": ChatTemplate(tmpl, bos, eos), "entry": entry,
                       "load_s": 0.0})
        svc = Service(cfg, backend=backend)
        svc.start()
        svc.registry.add(entry)
        cli = Client().connect(srv.url)
        try:
            body = json.dumps({"model": model_id, "messages": [{"role": "user", "content": "ping"}],
                               "max_tokens": max_tokens, "temperature": 0}).encode()
            r = json.loads(cli.request("lmstudio.chat_model", body, 60).data)
            if not r.get("ok") or r["data"].get("http_status") != 200:
                raise RuntimeError(f"chat_model failed: {str(r)[:300]}")
            cli._c.bench_requests("lmstudio.chat_model", body, warmup, 60000)
            us = cli._c.bench_requests("lmstudio.chat_model", body, n, 60000)
        finally:
            cli.close()
            for sub in svc.subs:
                sub.unsubscribe()
            svc.client.close()
            srv.stop()
            if started:
                engine.shutdown()
    return {"p50_ms": round(_pct(us, 50) / 1e3, 4), "p99_ms": round(_pct(us, 99) / 1e3, 4),
            "mean_ms": round(statistics.mean(us) / 1e3, 4), "n": n, "max_tokens": max_tokens,
            "prompt_tokens": r["data"]["response"]["usage"]["prompt_tokens"]}


if __name__ == "__main__":
    print(json.dumps(measure_rtt()))
