#!/bin/bash
# round 5, call AQ: tuning-table entry tests at real shapes (70B entries, re-tuned 8B entries); the 8B headline bench on
# the quantised GEMMs (no f16 copies) and with the default copies.
source tools/gpu_steps.sh
step r5aq_tests 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_gpu.py -k "tuning_table_entries"
export NLS_DENSE_WEIGHTS=0; step r5aq_nocopies 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-rtt --serve-load 0
unset NLS_DENSE_WEIGHTS; step r5aq_default 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
