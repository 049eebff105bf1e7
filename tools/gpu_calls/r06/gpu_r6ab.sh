#!/bin/bash
# round 6, call AB: mode 7 (4-wave narrow dense tiles, 128 x 64/96/128) -- kernel tests, dense tuning of the 8B
# Q|K|V / o / down at M = 256 / 512 restricted to mode 7 (+ the current entry), then the B=512 / B=256 benches with
# and without the fresh entries (NLS_TUNING_EXTRA_FILE).
source tools/gpu_steps.sh
step r6ab_tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_hgemm_dense or test_qkv_rope_kv_dense"
step r6ab_tune 900 python3 -u tools/tune_gemv.py --model llama-3-8b --dense --ms 256,512 --modes 7 --only qkv,o,down --out gpurun_out/tune_r6ab.json --log gpurun_out/tune_r6ab.log
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6ab_b512_cur 300 $B
NLS_TUNING_EXTRA_FILE=gpurun_out/tune_r6ab.json step r6ab_b512_m7 300 $B
step r6ab_b256_cur 300 $B --concurrency 256
NLS_TUNING_EXTRA_FILE=gpurun_out/tune_r6ab.json step r6ab_b256_m7 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
