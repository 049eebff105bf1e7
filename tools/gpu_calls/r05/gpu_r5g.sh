#!/bin/bash
# round 5, call G: (1) simulated-rank add+norm without re-tag (which rows of h go wrong, and how); (2) the TP
# rehearsal with eager one-shot calls and a DOT dump of every captured decode graph (kernel-node list, RCCL nodes).
source tools/gpu_steps.sh
step r5g_sim_noretag 120 env NLS_AR_RETAG=0 python3 -u tools/diag/addnorm_sim.py 2 16 4096 8
step r5g_sim_retag 120 env NLS_AR_RETAG=1 python3 -u tools/diag/addnorm_sim.py 2 16 4096 8
step r5g_sim_noretag_w8 120 env NLS_AR_RETAG=0 python3 -u tools/diag/addnorm_sim.py 8 16 8192 8
rm -rf gpurun_out/graphs
step r5g_dump 300 env NLS_ONESHOT_EAGER=1 NLS_GRAPH_DUMP=gpurun_out/graphs python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
