#!/bin/bash
# LDS-dequant GEMM with the 4-stage activation register ring: tests, MoE probe, Mixtral decode
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_gpu.py > gpurun_out/xr_tests.log 2>&1 || { tail -30 gpurun_out/xr_tests.log; exit 1; }
tail -1 gpurun_out/xr_tests.log
P="python3 -u tools/moe_probe.py"
for a in "--proj gateup --T 256 --rt 4" "--proj gateup --T 64 --rt 2" "--proj gateup --T 64 --rt 4" \
         "--proj down --T 256 --rt 4 --type Q6_K" "--proj gateup --T 512 --rt 4" "--proj gateup --T 1 --k 8 --rt 4"; do
  timeout -k 10 120 $P $a >> gpurun_out/xr_probe.log 2>&1 || { tail -5 gpurun_out/xr_probe.log; exit 1; }
done
grep "^moe" gpurun_out/xr_probe.log | sed 's/counts=\[[^]]*\] //'
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/xr_$label.log 2>&1 || { tail -20 gpurun_out/xr_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/xr_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
for B in 32 64 128 256 512; do BARGS="--concurrency $B"; run b$B; done
rm -f /tmp/nls_bench/*.gguf
