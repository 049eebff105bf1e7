#!/usr/bin/env python3
"""BASELINE config 4: JetStream Object-Store bucket -> `lmstudio.pull_model` -> .gguf on disk -> model
loaded on one MI355X. Measures the real service path end to end:

  1. writes a random-init GGUF of the named model (once; e.g. Llama-3-8B Q4_K_M, 4.9 GB),
  2. `put`s it into bucket `llm-models` of an embedded NATS server as
     `<publisher>/<model>-GGUF/<file>.gguf` (README.md:278-282 naming) with the C++ object-store client,
  3. sends `lmstudio.pull_model {"identifier": ..., "load": <--load>}` to a worker and times the reply:
     chunks stream to the worker over an ordered push consumer (flow-controlled), are SHA-256
     verified, renamed into MODELS_DIR, and (--load) the model is loaded onto the GPU,
  4. optionally (--resume-test) kills a pull half way and checks the second pull resumes.

    python tools/pull_bench.py [--model llama-3-8b] [--load] [--device cuda] [--out gpurun_out/pull.json]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--work", default=os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench"))
    ap.add_argument("--load", action="store_true", help="pull_model with load=true (GPU)")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--resume-test", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    from nats_llm_studio_amd.natsio import Client, EmbeddedServer, ObjectStore
    from nats_llm_studio_amd.service.config import WorkerConfig
    from nats_llm_studio_amd.service.service import Service

    os.makedirs(a.work, exist_ok=True)
    src = os.path.join(a.work, f"{a.model}-{a.ftype}.gguf")
    if not os.path.exists(src):
        write_synthetic_gguf(src, a.model, a.ftype, seed=0)
    size = os.path.getsize(src)
    name = f"synthetic/{a.model}-GGUF/{a.model}-{a.ftype}.gguf"
    res = {"model": a.model, "ftype": a.ftype, "bytes": size}
    models = tempfile.mkdtemp(prefix="nls_models_", dir=a.work)
    srv = EmbeddedServer(max_payload=8 << 20).start()
    try:
        cli = Client().connect(srv.url)
        st = ObjectStore(cli, "llm-models", timeout=60.0)
        st.create("LLM model repository (.gguf)")
        t0 = time.time()
        st.put_file(name, src)
        res["put_s"] = round(time.time() - t0, 2)
        res["put_MBps"] = round(size / (time.time() - t0) / 1e6, 1)
        if a.resume_test:   # interrupted pull, then resume from the .part / .part.idx checkpoint
            dest = os.path.join(a.work, "resume_test.gguf")
            for f in (dest, dest + ".part", dest + ".part.idx"):
                if os.path.exists(f):
                    os.unlink(f)

            class Stop(Exception):
                pass

            def cut(got, total):
                if got > total // 2:
                    raise Stop()
            try:
                st.get_file(name, dest, True, cut)
            except Exception:
                pass
            part = os.path.getsize(dest + ".part") if os.path.exists(dest + ".part") else 0
            t1 = time.time()
            st.get_file(name, dest, True, None)
            res["resume"] = {"bytes_before_cut": part, "resumed_s": round(time.time() - t1, 2),
                             "ok": os.path.getsize(dest) == size}
            os.unlink(dest)
        cfg = WorkerConfig(nats_url=srv.url, models_dir=models, backend="engine", device=a.device)
        svc = Service(cfg).start()
        try:
            t0 = time.time()
            r = json.loads(cli.request("lmstudio.pull_model", json.dumps(
                {"identifier": f"synthetic/{a.model}", "load": bool(a.load)}).encode(), 900).data)
            dt = time.time() - t0
            res["pull_ok"] = bool(r.get("ok"))
            res["pull_s"] = round(dt, 2)
            res["pull_MBps"] = round(size / dt / 1e6, 1)
            res["pull_reply"] = {k: v for k, v in (r.get("data") or {}).items() if k != "output"}
            if not r.get("ok"):
                res["error"] = r.get("error")
        finally:
            svc.stop()
            svc.client.close()
        cli.close()
    finally:
        srv.stop()
        shutil.rmtree(models, ignore_errors=True)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
