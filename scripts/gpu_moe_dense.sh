#!/bin/bash
# MoE experts on f16 copies (dense DMA GEMM, mapped rows): tests, then Mixtral B=256 decode over the
# gate/up (NLS_MOE_DENSE_GU) and down (NLS_MOE_DENSE_DN) configs; "quant" = experts not expanded
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mapped or moe" > gpurun_out/moed_tests.log 2>&1 || { tail -30 gpurun_out/moed_tests.log; exit 1; }
tail -1 gpurun_out/moed_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/moed_$label.log 2>&1 || { tail -20 gpurun_out/moed_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/moed_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
BARGS="--concurrency 256"
run d582_d5824
run g584 NLS_MOE_DENSE_GU=5,8,4
run g482 NLS_MOE_DENSE_GU=4,8,2
run g5162 NLS_MOE_DENSE_GU=5,16,2
run dn5821 NLS_MOE_DENSE_DN=5,8,2,1
run dn5822 NLS_MOE_DENSE_DN=5,8,2,2
run dn4824 NLS_MOE_DENSE_DN=4,8,2,4
BARGS="--concurrency 128"
run b128 
BARGS="--concurrency 64"
run b64
rm -f /tmp/nls_bench/*.gguf
