#!/bin/bash
# Split RMSNorm + short-split attention: tests, then B=1 decode A/B, kernel breakdown of the best arm
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "split_rmsnorm or fused or addnorm or qkv_rope or attention" > gpurun_out/splitnorm_tests.log 2>&1 || { tail -30 gpurun_out/splitnorm_tests.log; exit 1; }
tail -2 gpurun_out/splitnorm_tests.log
run() {  # label env... -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --no-rtt --serve-load 0 $BARGS > gpurun_out/ab_$label.log 2>&1 || { tail -20 gpurun_out/ab_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/ab_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for rep in 1 2; do
  BARGS="--concurrency 1"
  run fn0_c64 NLS_FUSE_NORM=0 NLS_ATTN_MIN_CHUNK=64
  run fn1_c64 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=64
  run fn1_c32 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=32
  run fn1_c16 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=16
  BARGS="--concurrency 1 --prompt-len 1024"
  run p1k_c64 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=64
  run p1k_c16 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=16
  BARGS="--concurrency 16 --prompt-len 1024"
  run b16_c64 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=64
  run b16_c16 NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=16
done
NLS_FUSE_NORM=1 NLS_ATTN_MIN_CHUNK=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1fn -o run -- python3 -u bench.py --concurrency 1 --steps 40 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/prof_b1fn.log 2>&1 || { tail -5 gpurun_out/prof_b1fn.log; exit 1; }
python tools/analyze_trace.py gpurun_out/prof_b1fn/run_results.db > gpurun_out/b1fn_breakdown.txt 2>&1; head -14 gpurun_out/b1fn_breakdown.txt
