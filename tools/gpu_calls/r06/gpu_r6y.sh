#!/bin/bash
# round 6, call Y: Qwen2 with its Q / K rows permuted to adjacent RoPE pairs at load (RoPE fused into the Q|K|V epilogue,
# no separate rope_kv launch): the model tests against the fp32 oracle, then Qwen2.5-7B B=1 / B=512 with and without
# (NLS_NEOX_PERMUTE=0), back to back.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step r6y_model_tests 600 $T tests/test_model_gpu.py tests/test_production_gpu.py -k "qwen"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
B="python3 -u bench.py --model qwen2.5-7b --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6y_b1_perm 300 $B --concurrency 1
NLS_NEOX_PERMUTE=0 step r6y_b1_neox 300 $B --concurrency 1
step r6y_b512_perm 300 $B
NLS_NEOX_PERMUTE=0 step r6y_b512_neox 300 $B
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
