#!/usr/bin/env bash
# A/B of bench.py runs under env overrides, one JSON result line each -> gpurun_out/bench_ab.jsonl.
# Cases come on stdin, one per line: "<name>|<env assignments>|<extra bench args>", e.g.
#   echo 'fuse_norm|NLS_FUSE_NORM=1|--concurrency 1' | bash tools/bench_ab.sh
# Every run has its own time limit; a crash / timeout ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/bench_ab.jsonl
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue ;; esac
  log=gpurun_out/ab_${name}.log
  env $envs timeout -k 10 ${STEP_TIMEOUT:-240} python -u bench.py --no-rtt --serve-load 0 --tp-leg 0 $args > $log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $log; exit $rc; fi
  line=$(grep '^{' $log | tail -1)
  CASE="$name" ENVS="$envs" ARGS="$args" LINE="$line" python3 -c 'import json, os; print(json.dumps({"case": os.environ["CASE"], "env": os.environ["ENVS"], "args": os.environ["ARGS"], "bench": json.loads(os.environ["LINE"])}))' >> $out
  echo "$name $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "tok/s", d["ms_per_step"], "ms/step")')"
done
