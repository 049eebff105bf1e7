#!/bin/bash
# round 6, call AC: deeper LDS rings for the one-workgroup-per-CU dense GEMMs -- mode 7 at 5 stages (default now)
# and mode 4 (128-row blocks) at 5 stages (NLS_M4_NST=5) vs 3: kernel tests under both, dense tuning of the 8B
# Q|K|V / o / down, and the B=512 / B=256 benches.
source tools/gpu_steps.sh
T="python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k"
step r6ac_tests 600 $T "test_hgemm_dense or test_qkv_rope_kv_dense"
NLS_M4_NST=5 step r6ac_tests_m4 600 $T "test_hgemm_dense or test_qkv_rope_kv_dense"
step r6ac_tune7 900 python3 -u tools/tune_gemv.py --model llama-3-8b --dense --ms 256,512 --modes 7 --only qkv,o,down --out gpurun_out/tune_r6ac7.json --log gpurun_out/tune_r6ac7.log
NLS_M4_NST=5 step r6ac_tune4 900 python3 -u tools/tune_gemv.py --model llama-3-8b --dense --ms 256,512 --modes 4 --only qkv,o,down --out gpurun_out/tune_r6ac4.json --log gpurun_out/tune_r6ac4.log
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6ac_b512_cur 300 $B
NLS_M4_NST=5 step r6ac_b512_m4n5 300 $B
NLS_TUNING_EXTRA_FILE=gpurun_out/tune_r6ac7.json step r6ac_b512_m7 300 $B
NLS_M4_NST=5 NLS_TUNING_EXTRA_FILE=gpurun_out/tune_r6ac4.json step r6ac_b512_m4t 300 $B
step r6ac_b256_cur 300 $B --concurrency 256
NLS_M4_NST=5 step r6ac_b256_m4n5 300 $B --concurrency 256
NLS_TUNING_EXTRA_FILE=gpurun_out/tune_r6ac7.json step r6ac_b256_m7 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
