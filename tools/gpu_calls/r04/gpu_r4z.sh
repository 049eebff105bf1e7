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
step pf_prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_prof_z -o run -- python3 tools/prefill_probe.py --lens 32768 --reps 1
python3 tools/prefill_probe.py --analyze "$(find gpurun_out/pf_prof_z -name '*kernel_trace.csv' | head -1)" --lens 32768 > gpurun_out/pf_breakdown_z.txt 2>&1; head -12 gpurun_out/pf_breakdown_z.txt; tail -2 gpurun_out/pf_breakdown_z.txt
rm -rf gpurun_out/pf_prof_z
exit $STEPS_RC
