#!/bin/bash
# round 5, call AO: Llama-3-70B one GPU B=512 under auto (quantised GEMMs) with the 70B-tuned mode-9 winners; the tuning
# entry tests (every table entry at its real shape vs the fp32 reference).
source tools/gpu_steps.sh
#step r5ao_auto 900 python3 -u bench.py --model llama-3-70b --concurrency 512 --steps 10 --warmup 3 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
step r5ao_tests 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_gpu.py -k "tuning_table_entries"
exit $STEPS_RC
