#!/bin/bash
# round 5, call J: Mixtral-8x7B B=256 grouped expert GEMMs: timing of mode 2 (default) vs mode 12 per projection, then
# PMC passes over the default gate|up launch (VALU / MFMA / LDS / waits) to see what bounds it.
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 -u tools/diag/moe_probe.py"
step r5j_gu_m2 120 $P --proj gateup --cfg 2,8,4,1
step r5j_gu_m2r2 120 $P --proj gateup --cfg 2,8,2,1
step r5j_gu_m12 120 $P --proj gateup --cfg 12,4,2,1
step r5j_gu_m12r4 120 $P --proj gateup --cfg 12,4,4,1
step r5j_dn_m2 120 $P --proj down --cfg 2,8,4,1
step r5j_dn_m2q6 120 $P --proj down --cfg 2,8,4,1 --type Q6_K
step r5j_dn_m12 120 $P --proj down --cfg 12,4,2,1
mkdir -p gpurun_out/pmcj
i=0
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
          "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  step r5j_pmc$i 90 rocprofv3 --pmc $CT -d gpurun_out/pmcj/p$i -o run --output-format csv -- python3 tools/diag/moe_probe.py --proj gateup --cfg 2,8,4,1 --iters 3
done
python3 tools/pmc_summary.py gpurun_out/pmcj > gpurun_out/pmcj/summary.txt 2>&1; cat gpurun_out/pmcj/summary.txt
exit $STEPS_RC
