#!/bin/bash
# Long-context decode sweep (prompt length x concurrency), one bench process per point
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
: > gpurun_out/ctx_sweep.jsonl
for pt in "1 4096" "16 4096" "64 1024" "256 1024" "1 128" "512 128"; do
  set -- $pt
  timeout -k 10 300 python -u bench.py --concurrency $1 --prompt-len $2 --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/ctx_$1_$2.log 2>&1 || { echo "B=$1 P=$2 failed"; tail -5 gpurun_out/ctx_$1_$2.log; exit 1; }
  tail -1 gpurun_out/ctx_$1_$2.log >> gpurun_out/ctx_sweep.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/ctx_$1_$2.log').read().strip().splitlines()[-1]); print('B=$1 prompt=$2', d['value'], 'tok/s', d['ms_per_step'], 'ms/step', 'prefill', d['timings_s']['prefill_all'], 's')"
done
