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


if __name__ == "__main__":
    print(json.dumps(measure_rtt()))
