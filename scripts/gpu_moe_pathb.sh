#!/bin/bash
# MoE grouped GEMM on path B (mode 1, register dequant, active tiles): tests, probe, Mixtral decode
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_gpu.py > gpurun_out/pb_tests.log 2>&1 || { tail -30 gpurun_out/pb_tests.log; exit 1; }
tail -1 gpurun_out/pb_tests.log
P="python3 -u tools/moe_probe.py"
for a in "--proj gateup --T 256 --mode 1 --rt 2" "--proj gateup --T 256 --mode 1 --rt 1" "--proj gateup --T 256 --mode 1 --rt 2 --waves 4" \
         "--proj gateup --T 64 --mode 1 --rt 2" "--proj gateup --T 512 --mode 1 --rt 2" "--proj gateup --T 1 --k 8 --mode 1 --rt 2" \
         "--proj down --T 256 --mode 1 --rt 2 --type Q6_K" "--proj down --T 256 --mode 1 --rt 2 --type Q6_K --ks 2" "--proj down --T 256 --mode 1 --rt 2 --type Q4_K"; do
  timeout -k 10 120 $P $a >> gpurun_out/pb_probe.log 2>&1 || { tail -5 gpurun_out/pb_probe.log; exit 1; }
done
grep "^moe" gpurun_out/pb_probe.log | sed 's/counts=\[[^]]*\] //'
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/pb_$label.log 2>&1 || { tail -20 gpurun_out/pb_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/pb_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
for B in 64 256; do
  BARGS="--concurrency $B"
  run b${B}m1 NLS_MOE_QCFG_GU=1,8,2 NLS_MOE_QCFG_DN=1,8,2
done
BARGS="--concurrency 512"; run b512m1 NLS_MOE_QCFG_GU=1,8,2 NLS_MOE_QCFG_DN=1,8,2
BARGS="--concurrency 256"; run b256m1ks2 NLS_MOE_QCFG_GU=1,8,2 NLS_MOE_QCFG_DN=1,8,2 NLS_MOE_KS_DN=2
rm -f /tmp/nls_bench/*.gguf
