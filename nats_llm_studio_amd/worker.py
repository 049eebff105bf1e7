"""Runnable worker (the reference is a library with no `main`, `nats_llm_studio.go:1`;
its README's `go run .` cannot work -- this entry point is the real one).

    python -m nats_llm_studio_amd.worker [--nats-url nats://127.0.0.1:4222] [--models-dir DIR]
        [--queue-group lmstudio-workers] [--backend engine|stub] [--embedded-server]

Run N copies (one per GPU, HIP_VISIBLE_DEVICES / --device cuda:i) in the same queue group
to scale out (README.md:484).

Tensor parallel (one model over several GPUs, e.g. Llama-3-70B at TP=8):

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m nats_llm_studio_amd.worker \
        --tp 8 --model meta/llama-3-70b [--ep]

Every rank loads its shard; rank 0 joins NATS and schedules, ranks 1..N-1 follow its steps.
"""
from __future__ import annotations

import signal
import sys
import threading

from .service.config import WorkerConfig
from .service.service import Service
from .utils.metrics import log


def _resolve_model(cfg):
    import os
    from .service.registry import ModelEntry, Registry
    reg = Registry(cfg.models_dir)
    reg.scan()
    ent = reg.resolve(cfg.model) if cfg.model else None
    if ent is None and cfg.model and os.path.isfile(cfg.model):
        d = os.path.dirname(os.path.abspath(cfg.model))
        ent = ModelEntry(id=os.path.splitext(os.path.basename(cfg.model))[0].lower(), publisher="local",
                         model_dir=os.path.basename(d), path=os.path.abspath(cfg.model), dir=d)
    if ent is None:
        raise SystemExit(f"--model {cfg.model!r} not found under {cfg.models_dir}")
    return ent


def main_tp(cfg) -> int:
    """One rank of a tensor-parallel worker (launched by torchrun)."""
    from .models.llama import ShardSpec
    from .parallel.comm import init_distributed
    from .service.backends import EngineBackend
    comm = init_distributed()
    entry = _resolve_model(cfg)
    backend = EngineBackend(cfg)
    if comm.device is not None:
        backend._device = comm.device
    st = backend.build_state(entry, ShardSpec(comm.rank, comm.size, cfg.ep), comm, start=comm.rank == 0)
    log("tp_rank_ready", rank=comm.rank, world=comm.size, model=entry.id, load_s=round(st["load_s"], 2))
    if comm.rank != 0:
        st["engine"].follow()
        return 0
    backend.adopt(st)
    code = serve(cfg, backend)
    st["engine"].shutdown()          # releases the followers (STOP)
    return code


def main(argv=None):
    cfg = WorkerConfig.from_args(argv)
    import os
    if cfg.tp > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return main_tp(cfg)
    return serve(cfg)


def serve(cfg, backend=None):
    server = None
    if cfg.embedded_server:
        from .natsio import EmbeddedServer
        port = int(cfg.nats_url.rsplit(":", 1)[-1]) if ":" in cfg.nats_url.split("//")[-1] else 4222
        server = EmbeddedServer(port=port, store_dir=cfg.store_dir).start()
        log("embedded_server", url=server.url)
    svc = Service(cfg, backend=backend).start()
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
