#!/bin/bash
# round 6, call A: mode-14 GEMM + split-RMSNorm (EPI_ADDX / rin) numerics, whole-model xnorm path, first timings.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6a_kern 600 $T tests/test_kernels_gpu.py -k "hgemm14 or split_rmsnorm_chain or rope_kv_dense or hgemm_dense or hgemm10"
step r6a_model 600 $T tests/test_model_gpu.py -k "xnorm or prefill_logits or greedy_matches"
step r6a_tune 600 python3 -u tools/dense_tune.py --xnorm --M 256,512 --roles qkv,o,gateup,down,lm_head --rounds 3 --emit
step r6a_bench 400 python3 -u bench.py --steps 20 --warmup 5 --no-rtt --serve-load 0
exit $STEPS_RC
