#!/bin/bash
# round 5, call AL: single-prompt prefill graphs: equality tests, the short-prefill probe, bench chat RTT.
source tools/gpu_steps.sh
step r5al_test 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "prefill_graphs or graph_equals or greedy_matches or async_first"
step r5al_pf 300 python3 -u tools/diag/prefill_small.py --tokens 21 --reps 8
step r5al_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
