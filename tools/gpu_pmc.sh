#!/usr/bin/env bash
# PMC passes over one large-M GEMM shape (tools/gemm_probe.py), one counter group per run, + a summary.
#   tools/gpu_pmc.sh [shape] [M]      (CFG=mode,waves,rt,ks / DENSE=1 select the kernel)
set -u
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SHAPE=${1:-gateup}
M=${2:-256}
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 120 python -u tools/gemm_probe.py --shape $SHAPE --M $M ${CFG:+--cfg $CFG} ${DENSE:+--dense} > gpurun_out/pmc/time.log 2>&1 || exit $?
cat gpurun_out/pmc/time.log
i=0
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
          "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CT -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 tools/gemm_probe.py --shape $SHAPE --M $M ${CFG:+--cfg $CFG} ${DENSE:+--dense} --iters 5 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; cat gpurun_out/pmc/summary.txt
