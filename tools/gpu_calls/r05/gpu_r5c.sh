#!/bin/bash
# round 5, call C: (1) the eager one-shot timeout with every push read back by an atomic RMW right after it
# completed (NLS_AR_PROBE=1), consumer re-tag on / off; (2) mode 11 with the dequantisation spread over three
# phases (raw -> registers at Q0, row-tile 0 at Q1, row-tile 1 at Q2) vs mode 9 on the Llama-3-8B shapes.
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5c_probe 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 $R
step r5c_probe_noretag 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 NLS_AR_RETAG=0 $R
for f in probe probe_noretag; do
  echo "== $f"; grep -h -o "'addnorm_timeout_detail': {[^}]*}[^}]*}\|'push_readback_mismatch': {[^}]*}\|'pusher_view_of_rank0': {[^}]*}[^}]*}" gpurun_out/r5c_$f.log | head -6 || true
done
step r5c_m11 300 python3 -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "qgemm11 or quant11"
step r5c_tune 500 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --modes 9,11 --out gpurun_out/tune11c.json --log gpurun_out/tune11c.log
exit $STEPS_RC
