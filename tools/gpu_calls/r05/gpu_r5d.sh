#!/bin/bash
# round 5, call D: (1) eager one-shot: every push read back by an atomic RMW right after it completed
# (NLS_AR_PROBE=1), re-tag on / off; (2) mode 11 (dequant spread over three phases) vs mode 9 on the 8B shapes;
# (3) mode 12 (mode 9 over 64-row blocks of each expert's routed rows) numerics, then Mixtral-8x7B B=256 with
# the expert GEMMs on mode 2 (default) / mode 12.
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5d_probe 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 $R
step r5d_probe_noretag 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 NLS_AR_RETAG=0 $R
for f in probe probe_noretag; do
  echo "== $f"; grep -h -o "'addnorm_timeout_detail': {[^}]*}[^}]*}\|'push_readback_mismatch': {[^}]*}\|'pusher_view_of_rank0': {[^}]*}[^}]*}" gpurun_out/r5d_$f.log | head -6 || true
done
step r5d_kern 300 python3 -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "qgemm11 or quant11 or mapped_moe"
step r5d_tune 500 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --modes 9,11 --out gpurun_out/tune11d.json --log gpurun_out/tune11d.log
M="python3 -u bench.py --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0"
step r5d_mx_m2 400 $M
step r5d_mx_m12 300 env NLS_MOE_QCFG_GU=12,4,2 NLS_MOE_QCFG_DN=12,4,2 $M
step r5d_mx_m12r4 300 env NLS_MOE_QCFG_GU=12,4,4 NLS_MOE_QCFG_DN=12,4,4 $M
grep -h '^{' gpurun_out/r5d_mx_*.log | cut -c1-260
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
