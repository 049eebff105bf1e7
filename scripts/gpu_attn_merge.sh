#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in 4 8; do
  NLS_ATTN_WAVES=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_kernels_gpu.py -k "attention_paged" > gpurun_out/am_w$w.log 2>&1 || { tail -20 gpurun_out/am_w$w.log; exit 1; }
  echo "waves=$w $(tail -1 gpurun_out/am_w$w.log)"
done
run() {  # tag concurrency prompt
  timeout -k 10 300 python -u bench.py --concurrency $2 --prompt-len $3 --steps 100 --warmup 10 --no-rtt \
      --serve-load 0 > gpurun_out/am.log 2>&1 || { tail -5 gpurun_out/am.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/am.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run "b512 p128" 512 128
run "b1 p4096" 1 4096
run "b16 p4096" 16 4096
run "b256 p1024" 256 1024
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
rm -rf gpurun_out/prof_am
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_am -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 > gpurun_out/prof_am.log 2>&1 || exit $?
python3 tools/analyze_trace.py $(find gpurun_out/prof_am -name "*kernel_trace.csv" | head -1) | head -8
