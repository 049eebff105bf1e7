#!/bin/bash
# PMC of the batch-1 GEMVs (gate|up path B XL, Q|K|V path A): issue / wait / VALU mix
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmc_b1
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
C2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_SALU"
for s in gateup qkv; do
  timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/pmc_b1/$s/p1 -o p1 --output-format csv -- python3 tools/l3_warm_probe.py --shape $s > gpurun_out/pmc_b1/$s.p1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/pmc_b1/$s/p2 -o p2 --output-format csv -- python3 tools/l3_warm_probe.py --shape $s > gpurun_out/pmc_b1/$s.p2.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_b1/$s > gpurun_out/pmc_b1/$s.summary.txt 2>&1 || exit 1
done
