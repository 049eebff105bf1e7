#!/bin/bash
# dense GEMM: mid-step-barrier pipelined loop vs the end-of-step barrier (one process, interleaved)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
K=$PWD/nats_llm_studio_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hgemm" > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -1 gpurun_out/pipe_tests.log
for M in 256 512 1024; do
  timeout -k 10 300 python -u tools/gemm_ab.py --dense --libs $K/_kernels_base.so,$K/_kernels.so --M $M --shapes qkv,o,gateup,down,lm_head || exit 1
done
for arm in base pipe; do
  lib=$K/_kernels.so; [ $arm = base ] && lib=$K/_kernels_base.so
  NLS_KERNELS_SO=$lib timeout -k 10 400 python -u bench.py --no-rtt --serve-load 0 --steps 100 > gpurun_out/pipe_$arm.log 2>&1 || { tail -20 gpurun_out/pipe_$arm.log; exit 1; }
  echo "$arm $(tail -1 gpurun_out/pipe_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
