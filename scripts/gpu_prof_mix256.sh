#!/bin/bash
# rocprofv3 kernel breakdown of Mixtral-8x7B B=256 decode; TAG names the run (env knobs pass through)
set -u
TAG=${TAG:-mix256}
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3 --no-rtt --serve-load 0 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python tools/analyze_trace.py gpurun_out/prof_$TAG/run_results.db > gpurun_out/${TAG}_breakdown.txt 2>&1; head -16 gpurun_out/${TAG}_breakdown.txt
TAG=$TAG python - <<'PY'
import sqlite3
from collections import defaultdict
import os
c=sqlite3.connect('gpurun_out/prof_%s/run_results.db' % os.environ['TAG'])
rows=list(c.execute("select name, start, end, grid_size from kernels order by start")) if False else list(c.execute("select name, start, end from kernels order by start"))
d=defaultdict(list)
for n,s,e in rows[-393*10:]:
    if 'qmm_lds' in n or 'hgemm' in n: d[n[:40]].append((e-s)/1e3)
for n,v in d.items():
    v=sorted(v); print(n, len(v), 'p10 %.1f med %.1f p90 %.1f max %.1f' % (v[len(v)//10], v[len(v)//2], v[9*len(v)//10], v[-1]))
PY
rm -f /tmp/nls_bench/*.gguf
