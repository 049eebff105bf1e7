#!/bin/bash
# round 4, call Z: the default bench (B=512 + service load) with first tokens read back once per step, prefill
# chunks per step 4 (default) and 8; the sync per-chunk picks (NLS_ASYNC_FIRST=0) as the baseline
source tools/gpu_steps.sh
step bench_async4 400 python3 -u bench.py
step bench_sync4 400 env NLS_ASYNC_FIRST=0 python3 -u bench.py --tp-leg 0
step bench_async8 400 env NLS_PREFILL_CHUNKS=8 python3 -u bench.py --tp-leg 0
for f in bench_async4 bench_sync4 bench_async8; do
  python3 - "$f" <<'PY'
import json, sys
n = sys.argv[1]
line = [l for l in open(f"gpurun_out/{n}.log") if l.startswith("{")][-1]
d = json.loads(line)
s = d.get("service_load") or {}
print(n, d["value"], d["ms_per_step"], s.get("tok_s"), s.get("ttft_p50_ms"), (s.get("engine") or {}).get("host_ms"))
PY
done
exit $STEPS_RC
