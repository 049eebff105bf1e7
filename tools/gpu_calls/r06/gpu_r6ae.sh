#!/bin/bash
# round 6, call AE: L2-channel spread for the dense GEMMs -- per-weight-tile K rotation (NLS_HG_KROT) and padded
# activation rows (gemm_probe --ldx-pad): kernel tests with the rotation on, probe timings, B=512 benches.
source tools/gpu_steps.sh
T="python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k"
NLS_HG_KROT=7 step r6ae_tests 600 $T "test_hgemm_dense or test_hgemm10 or test_qkv_rope_kv_dense"
P="python3 -u tools/gemm_probe.py --M 512 --dense --iters 50"
for kr in 0 1 7 13 29; do
  NLS_HG_KROT=$kr step r6ae_qkv_k$kr 120 $P --shape qkv --cfg 4,16,2,1
  NLS_HG_KROT=$kr step r6ae_gu_k$kr 120 $P --shape gateup --cfg 10,8,1,1
  NLS_HG_KROT=$kr step r6ae_dn_k$kr 120 $P --shape down --cfg 10,8,2,4
  NLS_HG_KROT=$kr step r6ae_o_k$kr 120 $P --shape o --cfg 4,16,2,2
done
step r6ae_qkv_pad 120 $P --shape qkv --cfg 4,16,2,1 --ldx-pad 64
step r6ae_gu_pad 120 $P --shape gateup --cfg 10,8,1,1 --ldx-pad 64
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6ae_b512_k0 300 $B
NLS_HG_KROT=7 step r6ae_b512_k7 300 $B
NLS_HG_KROT=13 step r6ae_b512_k13 300 $B
step r6ae_b512_k0b 300 $B
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
