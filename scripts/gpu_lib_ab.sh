#!/usr/bin/env bash
# Mode 7 (hipBLASLt on the f16 copies + epilogue pass) on a GPU box: its tests, the per-shape A/B and the
# headline bench with it on / off. Every GPU step has its own time limit; a failure ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "lib_gemm or hgemm_dense_swiglu" tests/test_production_gpu.py -k "lib_gemm" \
    > gpurun_out/lib_tests.log 2>&1 || { tail -20 gpurun_out/lib_tests.log; exit 1; }
tail -2 gpurun_out/lib_tests.log
timeout -k 10 300 python -u tools/blaslt_ab.py --M 256,512,1024 --shapes qkv,gateup,lm_head \
    > gpurun_out/blaslt_ab_mode7.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/blaslt_ab_mode7.txt
for v in 1 0 1 0; do
  NLS_LIB_GEMM=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-rtt --serve-load 0 \
      > gpurun_out/bench_lib$v.log 2>&1 || { tail -5 gpurun_out/bench_lib$v.log; exit 1; }
  echo "NLS_LIB_GEMM=$v $(tail -1 gpurun_out/bench_lib$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
