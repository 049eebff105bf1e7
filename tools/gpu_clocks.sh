#!/bin/bash
# Sample SCLK / power while the headline bench runs (is sustained MFMA load clock-limited?)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-rtt --steps 200 --warmup 5 > gpurun_out/bench_clk.log 2>&1 &
pid=$!
for i in $(seq 1 40); do
  sleep 2
  kill -0 $pid 2>/dev/null || break
  { date +%s.%N; timeout 10 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|mclk|Power|Temperature \(Sensor junction"; } >> gpurun_out/clocks.txt
done
wait $pid
rc=$?
tail -1 gpurun_out/bench_clk.log
exit $rc
