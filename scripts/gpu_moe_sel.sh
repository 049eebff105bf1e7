#!/bin/bash
# MoE: selected-expert launches + fused combine/norm (tests + Mixtral batch 1/16/256)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "moe or mapped or mixtral or reference or graph" > gpurun_out/moe_tests.log 2>&1 || { tail -30 gpurun_out/moe_tests.log; exit 1; }
tail -1 gpurun_out/moe_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 100 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/moe_$label.log 2>&1 || { tail -20 gpurun_out/moe_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/moe_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for B in 1 16 256; do BARGS="--concurrency $B"; run b$B; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix1 -o run -- python3 -u bench.py --model mixtral-8x7b --ftype Q5_K_M --concurrency 1 --steps 30 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/prof_mix1.log 2>&1 || { tail -5 gpurun_out/prof_mix1.log; exit 1; }
python tools/analyze_trace.py gpurun_out/prof_mix1/run_results.db > gpurun_out/mix1_breakdown.txt 2>&1; head -16 gpurun_out/mix1_breakdown.txt
rm -f /tmp/nls_bench/*.gguf
