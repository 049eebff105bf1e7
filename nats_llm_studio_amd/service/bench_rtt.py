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
            # where one request's time goes (service tracer, p50 per phase over the timed requests)
            phases = {k: v.get("p50") for k, v in svc.tracer.summary(last=0)["phases_ms"].items()}
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
            "prompt_tokens": r["data"]["response"]["usage"]["prompt_tokens"], "phases_p50_ms": phases}


def measure_engine_chat_load(engine, metadata: dict, model_id: str = "llama-3-8b", n: int = 512,
                             max_tokens: int = 64, sampled_frac: float = 0.5, timeout_s: float = 600.0,
                             seed: int = 0, prompt_tokens: int = 128) -> dict:
    """Service-path throughput: `n` concurrent `lmstudio.chat_model` requests published at once through
    the embedded NATS server (natscore) -> Python handlers -> chat template / tokenizer -> the REAL
    continuous-batching engine -> JSON replies to per-request inboxes. A fraction `sampled_frac` of the
    requests carries the reference README's sampling payload (`temperature: 0.7`,
    /root/reference/README.md:200-203); the rest are greedy. Reports output tok/s over the whole
    burst (first publish -> last reply, from the replies' usage.completion_tokens) and per-request
    RTT p50/p99. Prompts are random word sequences cut to a rendered length drawn uniformly from
    [prompt_tokens/2, 3*prompt_tokens/2] tokens (mean = the headline config's seq_len). The result
    carries the per-phase breakdown of the service tracer (recv -> validate -> tokenize -> queue ->
    prefill -> decode -> respond, p50/p99 over all requests), the client-side dispatch share (RTT minus
    the traced span) and the engine's counters over the burst."""
    import random
    import threading
    import time
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
    rnd = random.Random(seed)
    words = ("the model of a system that runs on eight GPUs with fast links between them and a large cache "
             "tell me about history science music art code data network latency token batch kernel memory").split()
    done = threading.Event()
    t_send, t_recv, bodies = {}, {}, {}
    lock = threading.Lock()
    with tempfile.TemporaryDirectory() as d:
        srv = EmbeddedServer(max_payload=8 << 20).start()
        cfg = WorkerConfig(nats_url=srv.url, models_dir=d, backend="engine")
        cfg.handler_workers = max(cfg.handler_workers, 8)
        backend = EngineBackend(cfg)
        entry = ModelEntry(id=model_id, publisher="synthetic", model_dir=model_id, path="", dir=d,
                           arch=engine.cfg.arch, quantization="Q4_K_M", max_context_length=engine.ctx)
        backend.adopt({"engine": engine, "tok": tok, "tmpl": ChatTemplate(tmpl, bos, eos), "entry": entry,
                       "load_s": 0.0})
        svc = Service(cfg, backend=backend)
        svc.start()
        svc.registry.add(entry)
        cli = Client().connect(srv.url)

        def on_reply(m):
            now = time.monotonic()
            i = int(m.subject.rsplit(".", 1)[1])
            with lock:
                t_recv[i] = now
                bodies[i] = m.data
                if len(t_recv) == n:
                    done.set()

        sub = cli.subscribe("_INBOX.load.>", "", on_reply, 4)
        cli.flush()
        payloads = []
        plens = []
        tmpl_o = ChatTemplate(tmpl, bos, eos)
        for i in range(n):
            target = rnd.randint(max(8, prompt_tokens // 2), max(9, 3 * prompt_tokens // 2))
            ws = []
            while True:
                ws.append(rnd.choice(words))
                msgs = [{"role": "system", "content": "You are a helpful assistant."},
                        {"role": "user", "content": " ".join(ws)}]
                nt = len(tok.encode(tmpl_o.render(msgs, add_generation_prompt=True), add_bos=False))
                if nt >= target:
                    break
            plens.append(nt)
            req = {"model": model_id, "messages": msgs, "max_tokens": max_tokens, "ignore_eos": True}
            if i < int(round(sampled_frac * n)):
                req.update(temperature=0.7, top_p=0.95, seed=i)
            else:
                req["temperature"] = 0
            payloads.append(json.dumps(req).encode())
        order = list(range(n))
        rnd.shuffle(order)                  # sampled and greedy requests interleave in the batch
        c0 = dict(engine.counters)
        h0 = dict(engine.host_ms) if hasattr(engine, "host_ms") else {}
        try:
            t0 = time.monotonic()
            for i in order:
                t_send[i] = time.monotonic()
                cli.publish("lmstudio.chat_model", payloads[i], reply=f"_INBOX.load.{i}")
            cli.flush()
            ok = done.wait(timeout_s)
            t1 = max(t_recv.values()) if t_recv else time.monotonic()
            phases = svc.tracer.summary(last=0)["phases_ms"]
            eng_d = {k: engine.counters[k] - c0.get(k, 0) for k in engine.counters}
            if h0 or hasattr(engine, "host_ms"):
                eng_d["host_ms"] = {k: round(v - h0.get(k, 0.0), 1) for k, v in engine.host_ms.items()}
        finally:
            sub.unsubscribe()
            cli.close()
            for s2 in svc.subs:
                s2.unsubscribe()
            svc.client.close()
            srv.stop()
            if started:
                engine.shutdown()
    comp, good, rtts, ttft, gen, errors = 0, 0, [], [], [], []
    for i, b in bodies.items():
        r = json.loads(b)
        if not (r.get("ok") and r["data"].get("http_status") == 200) and len(errors) < 3:
            errors.append(b[:300].decode("utf-8", "replace"))
        if r.get("ok") and r["data"].get("http_status") == 200:
            good += 1
            resp = r["data"]["response"]
            comp += resp["usage"]["completion_tokens"]
            st = resp.get("stats", {})
            if "time_to_first_token" in st:
                ttft.append(st["time_to_first_token"] * 1e3)
                gen.append(st["generation_time"] * 1e3)
        rtts.append((t_recv[i] - t_send[i]) * 1e3)
    wall = t1 - t0
    totals = [ph for ph in (phases.get("total") or {},)]
    return {"requests": n, "ok": good, "complete": bool(ok), "sampled_frac": sampled_frac, "max_tokens": max_tokens,
            "prompt_tokens_mean": round(sum(plens) / len(plens), 1), "prompt_tokens_max": max(plens),
            "completion_tokens": comp, "completion_tokens_requested": n * max_tokens,
            "wall_s": round(wall, 3), "tok_s": round(comp / wall, 1) if wall > 0 else None,
            "rtt_p50_ms": round(_pct(rtts, 50), 1) if rtts else None,
            "rtt_p99_ms": round(_pct(rtts, 99), 1) if rtts else None,
            "ttft_p50_ms": round(_pct(ttft, 50), 1) if ttft else None,
            "generation_p50_ms": round(_pct(gen, 50), 1) if gen else None,
            "phases_ms": phases, "engine": {k: v for k, v in eng_d.items() if v},
            "client_dispatch_p50_ms": (round(_pct(rtts, 50) - totals[0]["p50"], 2)
                                       if rtts and totals and "p50" in totals[0] else None),
            "errors": errors}


if __name__ == "__main__":
    print(json.dumps(measure_rtt()))
