#!/bin/bash
# round 6, call F: Mixtral grouped expert GEMM sweep -- mode 2 vs the mapped LDS-DMA GEMM (mode 3 at 64 / 96-row
# blocks, two workgroups per CU), split-K on down (tools/diag/moe_probe.py, B=256), then the Mixtral
# B=256 step with them.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
# the mapped mode-3 kernels against the fp32 reference before any timing run uses them
step r6f_mapped_tests 300 $T tests/test_kernels_gpu.py -k "mapped_moe"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
P="python3 -u tools/diag/moe_probe.py --T 256 --iters 20"
for c in 2,8,4,1 2,8,1,1 3,4,6,1 3,4,4,1 3,4,8,1; do step r6f_moe_gu_${c//,/_} 120 $P --proj gateup --cfg $c; done
for c in 2,8,4,1 2,8,4,2 2,8,4,4 2,8,1,2 3,4,6,1 3,4,6,2 3,4,6,4 3,4,4,2 3,4,4,4; do
  step r6f_moe_dn_${c//,/_} 120 $P --proj down --cfg $c; done
# Mixtral-8x7B B=256 step: the default configs vs the mapped DMA GEMM at 96-row blocks (down split 2 / 4)
B="python3 -u bench.py --model mixtral-8x7b --concurrency 256 --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6f_mx_default 600 $B
NLS_MOE_QCFG_GU=3,4,6 NLS_MOE_QCFG_DN=3,4,6 NLS_MOE_KS_DN=2 step r6f_mx_dma6_ks2 600 $B
NLS_MOE_QCFG_GU=3,4,6 NLS_MOE_QCFG_DN=3,4,6 NLS_MOE_KS_DN=4 step r6f_mx_dma6_ks4 600 $B
NLS_MOE_QCFG_GU=3,4,4 NLS_MOE_QCFG_DN=3,4,4 NLS_MOE_KS_DN=2 step r6f_mx_dma4_ks2 600 $B
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
