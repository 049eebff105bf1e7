#!/bin/bash
# round 4: B=512 decode, HEAD python vs the validated head's python (9578039: engine / sampling / llama / comm),
# same kernels (.so), same box, interleaved
source tools/gpu_steps.sh
rm -rf /tmp/oldrepo && mkdir -p /tmp/oldrepo && cp -r nats_llm_studio_amd bench.py /tmp/oldrepo/ && tar -xf tools/ab/old_py_9578039.tar -C /tmp/oldrepo
for i in 1 2; do
  step head_$i 300 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
  step old_$i 300 bash -c "cd /tmp/oldrepo && PYTHONPATH=/tmp/oldrepo python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0"
done
grep -h '^{' gpurun_out/head_1.log gpurun_out/old_1.log gpurun_out/head_2.log gpurun_out/old_2.log | cut -c150-260
exit $STEPS_RC
