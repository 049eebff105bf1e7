#!/bin/bash
# round 6, call G: re-tag OFF by default (one-shot kernel tests, TP / EP rehearsals with zero PyTorch kernels in the
# decode graphs and EP payload checksums), the fence-free chain probe with the fixed reference, then the Mixtral
# grouped-expert GEMM sweep (mode 2 vs the mapped LDS-DMA GEMM at 64 / 96-row blocks, split-K on down).
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6g_oneshot 300 $T tests/test_kernels_gpu.py -k "oneshot or mapped_moe or moe"
step r6g_tp 900 $T tests/test_tp_rehearsal_gpu.py
step r6g_chain 180 python3 -u tools/diag/fencefree_chain.py 64 20
P="python3 -u tools/diag/moe_probe.py --T 256 --iters 20"
for c in 2,8,4,1 2,8,1,1 3,4,6,1 3,4,4,1 3,4,8,1; do step r6g_moe_gu_${c//,/_} 120 $P --proj gateup --cfg $c; done
for c in 2,8,4,1 2,8,4,2 2,8,4,4 3,4,6,1 3,4,6,2 3,4,6,4 3,4,4,2 3,4,4,4; do
  step r6g_moe_dn_${c//,/_} 120 $P --proj down --cfg $c; done
exit $STEPS_RC
