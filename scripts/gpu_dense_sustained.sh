#!/bin/bash
# sustained (200-step, the driver's default) B=512 decode: dense f16 GEMMs on vs off, interleaved
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in 1 0; do
    NLS_DENSE_WEIGHTS=$arm timeout -k 10 400 python -u bench.py --no-rtt --serve-load 0 > gpurun_out/sus_$arm.log 2>&1 || { tail -20 gpurun_out/sus_$arm.log; exit 1; }
    echo "dense=$arm rep=$rep $(tail -1 gpurun_out/sus_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["steps"])')"
  done
done
