#!/bin/bash
# kernel tests, the Llama B=512 bench config whose service-load phase faulted (30 steps: KV pool
# smaller than the service burst), Mixtral decode at the new MoE defaults
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/fix_tests.log 2>&1 || { tail -30 gpurun_out/fix_tests.log; exit 1; }
tail -1 gpurun_out/fix_tests.log
timeout -k 10 500 python -u bench.py --steps 30 --warmup 5 > gpurun_out/fix_llama.log 2>&1 || { tail -30 gpurun_out/fix_llama.log; exit 1; }
tail -1 gpurun_out/fix_llama.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("llama", d["ms_per_step"], d["value"], d["service_load"])'
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/fix_$label.log 2>&1 || { tail -20 gpurun_out/fix_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/fix_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
BARGS="--concurrency 256"; run b256
BARGS="--concurrency 128"; run b128
BARGS="--concurrency 128"; run b128dn2ks4 NLS_MOE_RT_DN=2 NLS_MOE_KS_DN=4
BARGS="--concurrency 512"; run b512
rm -f /tmp/nls_bench/*.gguf
