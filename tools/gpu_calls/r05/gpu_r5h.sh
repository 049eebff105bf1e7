#!/bin/bash
# round 5, call H: full GPU suite + smoke with eager one-shot calls on by default (bounded add+norm grid);
# kernel-node lists of every captured TP / EP decode graph; the MALL-prefetch experiment for batch-1 decode;
# the default bench with the host/device step breakdown.
source tools/gpu_steps.sh
step r5h_gpu 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r5h_smoke 120 python3 -u __graft_entry__.py smoke
rm -rf gpurun_out/graphs_tp gpurun_out/graphs_ep
step r5h_dump_tp 200 env NLS_GRAPH_DUMP=gpurun_out/graphs_tp python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref
step r5h_dump_ep 200 env NLS_GRAPH_DUMP=gpurun_out/graphs_ep python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --model mixtral-8x7b-1layer --ep
step r5h_prefetch 200 python3 -u tools/diag/prefetch_b1.py
step r5h_bench 300 python3 -u bench.py --step-breakdown
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
