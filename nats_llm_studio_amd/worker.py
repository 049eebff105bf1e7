"""Runnable worker (the reference is a library with no `main`, `nats_llm_studio.go:1`;
its README's `go run .` cannot work -- this entry point is the real one).

    python -m nats_llm_studio_amd.worker [--nats-url nats://127.0.0.1:4222] [--models-dir DIR]
        [--queue-group lmstudio-workers] [--backend engine|stub] [--embedded-server]

Run N copies (one per GPU, HIP_VISIBLE_DEVICES / --device cuda:i) in the same queue group
to scale out (README.md:484).
"""
from __future__ import annotations

import signal
import sys
import threading

from .service.config import WorkerConfig
from .service.service import Service
from .utils.metrics import log


def main(argv=None):
    cfg = WorkerConfig.from_args(argv)
    server = None
    if cfg.embedded_server:
        from .natsio import EmbeddedServer
        port = int(cfg.nats_url.rsplit(":", 1)[-1]) if ":" in cfg.nats_url.split("//")[-1] else 4222
        server = EmbeddedServer(port=port, store_dir=cfg.store_dir).start()
        log("embedded_server", url=server.url)
    svc = Service(cfg).start()
    log("worker_started", nats_url=cfg.nats_url, queue_group=cfg.queue_group, models_dir=cfg.models_dir,
        backend=cfg.backend, subjects=[s.subject for s in svc.subs])
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    stop.wait()
    svc.stop()
    svc.client.close()
    if server:
        server.stop()
    log("worker_stopped")
    return 0


if __name__ == "__main__":
    sys.exit(main())
