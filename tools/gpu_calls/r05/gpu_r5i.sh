#!/bin/bash
# round 5, call I: stream-K dense GEMM (mode 13): numerics (owner sums / fallback / graph replays, RoPE epilogue),
# then the 8B dense shapes at M = 256 / 512 against modes 4 / 10.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step r5i_kern 300 $T tests/test_kernels_gpu.py -k "streamk or qkv_rope_kv_dense or hgemm_dense"
step r5i_tune 600 python3 -u tools/dense_tune.py --model llama-3-8b --M 256,512 --roles qkv,o,down,gateup --modes 4,5,10,13
exit $STEPS_RC
