#!/bin/bash
# round 5, call E: eager one-shot timeout -- timing history of every add+norm workgroup slot (NLS_AR_PROBE=1:
# start / pushed / polled on the device-wide clock, per epoch) on both ranks, re-tag on / off: was the peer's
# push of the timed-out epoch issued before the owner gave up (visibility) or after (scheduling / ordering)?
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5e_probe 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 $R
step r5e_probe_noretag 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_PROBE=1 NLS_AR_RETAG=0 $R
for f in probe probe_noretag; do
  echo "== $f"; grep -h -o "'addnorm_timeout_detail': {.*'probe_hist_self': [^]]*]]\|'pusher_view_of_rank0': {.*'probe_hist_pusher': [^]]*]]" gpurun_out/r5e_$f.log | cut -c1-1500 | head -4 || true
done
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
