#!/bin/bash
# B=1 A/B of the decode-time norm fusions (one process per arm, interleaved twice)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for arm in "base" "NLS_FUSE_NORM=1" "NLS_ADDNORM=8"; do
  env $([ $arm = base ] || echo $arm) timeout -k 10 300 python -u bench.py --concurrency 1 --steps 200 --warmup 10 --no-rtt > gpurun_out/b1_$arm.log 2>&1 || exit $?
  echo "$arm $(tail -1 gpurun_out/b1_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
done
