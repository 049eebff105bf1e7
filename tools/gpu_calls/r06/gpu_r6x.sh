#!/bin/bash
# round 6, call X: Qwen2.5-7B batch 1 takes 2.05 ms/token for fewer bytes and layers than Llama-3-8B (1.83): its kernel
# breakdown.
source tools/gpu_steps.sh
BS=1 MODEL=qwen2.5-7b step r6x_prof 500 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
