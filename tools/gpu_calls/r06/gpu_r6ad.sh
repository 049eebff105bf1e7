#!/bin/bash
# round 6, call AD: memory-side PMC of the dense GEMMs at the 8B decode shapes (M = 512): Q|K|V on mode 4 (16 waves,
# 128 x 128 tiles) and mode 7 (4 waves, 128 x 96), gate|up on mode 10 (256 x 256) -- L2 hit rate, L2->L1 request
# latency, TLB, TA/TD stalls -- to find what holds the narrow shapes at ~40 GB/s of fetch per CU.
set -u
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmc_ad
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
run() {   # name shape cfg
  local n=$1 sh=$2 cfg=$3
  timeout -k 10 120 python3 -u tools/gemm_probe.py --shape $sh --M 512 --cfg $cfg --dense > gpurun_out/pmc_ad/$n.time 2>&1 || { echo "$n time rc=$?"; tail -5 gpurun_out/pmc_ad/$n.time; exit 1; }
  cat gpurun_out/pmc_ad/$n.time
  local i=0
  for CT in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $CT -d gpurun_out/pmc_ad/${n}_p$i -o run --output-format csv -- python3 tools/gemm_probe.py --shape $sh --M 512 --cfg $cfg --dense --iters 5 > gpurun_out/pmc_ad/${n}_p$i.log 2>&1 || { echo "$n pass $i rc=$?"; tail -5 gpurun_out/pmc_ad/${n}_p$i.log; exit 1; }
  done
  echo "$n done"
}
run qkv_m4 qkv 4,16,2,1
run qkv_m7 qkv 7,4,3,1
run gateup_m10 gateup 10,8,1,1
