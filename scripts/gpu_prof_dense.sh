#!/bin/bash
# rocprofv3 kernel stats of the B=512 decode bench: dense f16 GEMMs (mode 4) vs quantised GEMMs
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for arm in dense quant; do
  if [ $arm = quant ]; then export NLS_DENSE_WEIGHTS=0; else export NLS_DENSE_WEIGHTS=1; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-rtt --serve-load 0 > gpurun_out/bench_$arm.log 2>&1 || { tail -20 gpurun_out/bench_$arm.log; exit 1; }
  echo "$arm $(tail -1 gpurun_out/bench_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$arm -o run -- python -u bench.py --steps 20 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/prof_$arm.log 2>&1 || { tail -20 gpurun_out/prof_$arm.log; exit 1; }
done
