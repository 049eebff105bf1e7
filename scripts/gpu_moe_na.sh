#!/bin/bash
# LDS-dequant GEMM with per-block active tile count: tests, Mixtral decode sweeps, Llama B=512 check
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/na_tests.log 2>&1 || { tail -30 gpurun_out/na_tests.log; exit 1; }
tail -1 gpurun_out/na_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/na_$label.log 2>&1 || { tail -20 gpurun_out/na_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/na_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
BARGS="--concurrency 256"
run gu4dn2
run gu4dn4 NLS_MOE_RT_DN=4
run gu2dn2 NLS_MOE_RT_GU=2
run gu1dn1 NLS_MOE_RT_GU=1 NLS_MOE_RT_DN=1
run dn4ks1 NLS_MOE_RT_DN=4 NLS_MOE_KS_DN=1
run dn4ks2 NLS_MOE_RT_DN=4 NLS_MOE_KS_DN=2
BARGS="--concurrency 128"
run b128
BARGS="--concurrency 64"
run b64
rm -f /tmp/nls_bench/*.gguf
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > gpurun_out/na_llama.log 2>&1 || { tail -20 gpurun_out/na_llama.log; exit 1; }
echo "llama $(tail -1 gpurun_out/na_llama.log | cut -c1-300)"
