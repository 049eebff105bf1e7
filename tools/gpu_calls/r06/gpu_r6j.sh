#!/bin/bash
# round 6, call J: PMC passes over the Mixtral B=256 gate|up launch on the mapped LDS-DMA GEMM (mode 3, 96-row
# blocks), for what bounds it (MFMA / VALU / LDS / waits / fetched bytes).
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_m3
i=0
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
          "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  step r6j_pmc$i 90 rocprofv3 --pmc $CT -d gpurun_out/pmc_m3/p$i -o run --output-format csv -- python3 tools/diag/moe_probe.py --proj gateup --cfg 3,4,6,1 --iters 3
done
python3 tools/pmc_summary.py gpurun_out/pmc_m3 > gpurun_out/pmc_m3/summary.txt 2>&1; cat gpurun_out/pmc_m3/summary.txt
exit $STEPS_RC
