#!/bin/bash
# round 6, call B: model-level xnorm test, per-config dense timings (mode 14 vs 4/5/10), xnorm tuning, B=512 kernel trace.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6b_model 600 $T tests/test_model_gpu.py -k "xnorm"
step r6b_kern 600 $T tests/test_kernels_gpu.py -k "hgemm14 or split_rmsnorm_chain or rope_kv_dense_rin or topc"
step r6b_dtune 600 python3 -u tools/dense_tune.py --M 512 --roles qkv,o,down --rounds 3
step r6b_xtune 600 python3 -u tools/dense_tune.py --xnorm --M 256,512 --roles qkv,o,gateup,down,lm_head --rounds 3 --emit
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step r6b_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6b -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0
python3 tools/analyze_trace.py $(find gpurun_out/prof_r6b -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_r6b_breakdown.txt 2>&1
head -30 gpurun_out/prof_r6b_breakdown.txt
exit $STEPS_RC
