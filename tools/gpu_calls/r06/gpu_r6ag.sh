#!/bin/bash
# round 6, call AG: PMC of the quantised mode-9 GEMM (qgemm9.hip) on the 8B gate|up at M = 512 (9,8,2,1) next to the
# dense mode 10 (10,8,1,1): is mode 9 fetch-bound (as the dense GEMMs are, profiles/pmc_dense_mem_r06.txt) or
# dequant / issue bound?
set -u
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmc_ag
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P4="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
run() {   # name shape cfg [--dense]
  local n=$1 sh=$2 cfg=$3 d=${4:-}
  timeout -k 10 120 python3 -u tools/gemm_probe.py --shape $sh --M 512 --cfg $cfg $d > gpurun_out/pmc_ag/$n.time 2>&1 || { echo "$n time rc=$?"; tail -5 gpurun_out/pmc_ag/$n.time; exit 1; }
  cat gpurun_out/pmc_ag/$n.time
  local i=0
  for CT in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $CT -d gpurun_out/pmc_ag/${n}_p$i -o run --output-format csv -- python3 tools/gemm_probe.py --shape $sh --M 512 --cfg $cfg $d --iters 5 > gpurun_out/pmc_ag/${n}_p$i.log 2>&1 || { echo "$n pass $i rc=$?"; tail -5 gpurun_out/pmc_ag/${n}_p$i.log; exit 1; }
  done
  echo "$n done"
}
run gateup_m9 gateup 9,8,2,1
run gateup_m10 gateup 10,8,1,1 --dense
