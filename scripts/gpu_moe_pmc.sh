#!/bin/bash
# MoE grouped GEMM in isolation (tools/moe_probe.py): timing sweep, then PMC passes on gate/up B=256
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/moepmc
P="python3 -u tools/moe_probe.py"
for a in "--proj gateup --T 256 --rt 4" "--proj gateup --T 256 --rt 2" "--proj gateup --T 64 --rt 2" "--proj gateup --T 64 --rt 4" \
         "--proj down --T 256 --rt 4 --type Q6_K" "--proj down --T 256 --rt 4 --type Q4_K" "--proj gateup --T 1 --k 8 --rt 4"; do
  timeout -k 10 120 $P $a >> gpurun_out/moepmc/time.log 2>&1 || { tail -5 gpurun_out/moepmc/time.log; exit 1; }
done
grep "^moe" gpurun_out/moepmc/time.log
i=0
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
          "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CT -d gpurun_out/moepmc/p$i -o run --output-format csv -- python3 tools/moe_probe.py --proj gateup --T 256 --rt 4 --iters 5 > gpurun_out/moepmc/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/moepmc/p$i.log; exit 1; }
done
echo pmc-done
