#!/bin/bash
# round 5, call A: root-causing the eager one-shot timeout after decode-graph replays (2 ranks on one GPU).
# Each variant: greedy TP2 rehearsal with batch churn + a second round whose eager prefill follows the graph
# replays, eager calls on the IPC kernels (NLS_ONESHOT_EAGER=1), extended timeout diagnostics (NLS_TP_TRACE=1):
#   base          the round-4 protocol
#   eprmw         epoch counters read / written by atomic read-modify-writes
#   pollrmw       peer granules polled by atomic read-modify-writes
#   noreplay      graphs captured on every rank but every step run eagerly
# then the GPU test suite and the driver's bench command as a sanity check of the tree.
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5a_base 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 $R
step r5a_eprmw 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_EP_RMW=1 $R
step r5a_pollrmw 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_AR_POLL_RMW=1 $R
step r5a_noreplay 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 NLS_GRAPH_NO_REPLAY=1 $R
for f in base eprmw pollrmw noreplay; do
  echo "== $f"; grep -h -o "error words.*\|'timeout_addnorm': \[[0-9, -]*\]\|'addnorm_timeout_detail': {[^}]*}[^}]*}" gpurun_out/r5a_$f.log | head -6 || true
done
step r5a_gputests 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r5a_smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step r5a_bench 300 python3 -u bench.py --steps 20 --warmup 5
grep -h '^{' gpurun_out/r5a_bench.log | cut -c1-400
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
