#!/bin/bash
# round 5, call M: full GPU suite + smoke at the current head (one-shot cap 2M floats, EP exchange, stream-K, native
# pre-tokeniser), graph node lists of the EP2 decode graphs (epx_kernel, no RCCL), then the driver's bench command.
source tools/gpu_steps.sh
step r5m_gpu 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step r5m_smoke 120 python3 -u __graft_entry__.py smoke
rm -rf gpurun_out/graphs_ep5
step r5m_dump_ep 200 env NLS_GRAPH_DUMP=gpurun_out/graphs_ep5 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --model mixtral-8x7b-1layer --ep
step r5m_bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
