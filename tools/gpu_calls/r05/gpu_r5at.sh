#!/bin/bash
# round 5, call AT: full GPU suite + smoke at the head (TP4/TP8/EP4/EP8 rehearsals, EP prefill row exchange, polling
# grids per co-resident rank), then the driver's bench command.
source tools/gpu_steps.sh
step r5at_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step r5at_smoke 120 python3 -u __graft_entry__.py smoke
step r5at_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
