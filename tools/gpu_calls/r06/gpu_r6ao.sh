#!/bin/bash
# round 6, call AO: soak at the final head -- the driver-form bench (engine + NATS RTT + service burst) three times back to
# back, a half-sampled B=512 decode (device sampler at full batch), and Mixtral / Qwen service bursts.
source tools/gpu_steps.sh
step r6ao_soak1 600 python3 -u bench.py --steps 20 --warmup 5
step r6ao_soak2 600 python3 -u bench.py --steps 20 --warmup 5
step r6ao_soak3 600 python3 -u bench.py --steps 20 --warmup 5
step r6ao_sampled 600 python3 -u bench.py --steps 20 --warmup 5 --sample-frac 0.5 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
step r6ao_qwen_svc 600 python3 -u bench.py --steps 20 --warmup 5 --model qwen2.5-7b
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
