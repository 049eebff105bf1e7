#!/bin/bash
# round 4, call Q: Mixtral-8x7B batch-1 GEMV re-tune (r04 candidates), then Mixtral-8x7B batch-1 decode with the
# current table vs the re-tuned M=1 entries
source tools/gpu_steps.sh
step tunemx1 400 python3 -u tools/tune_gemv.py --model mixtral-8x7b --base q5_k --ms 1 --out gpurun_out/tunemx1.json --log gpurun_out/tunemx1.log
python3 - > gpurun_out/tunemx1_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tunemx1.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.endswith(":1") and (k.split(":")[0].startswith("13") or k.startswith("14:32000:")) and "28672" not in k and "14336" not in k}))
PY
cat gpurun_out/tunemx1_extra.json
step mx_b1_base 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 1 --steps 60 --warmup 5
step mx_b1_tuned 300 env NLS_TUNING_EXTRA="$(cat gpurun_out/tunemx1_extra.json)" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 1 --steps 60 --warmup 5
step mx_b1_base2 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 1 --steps 60 --warmup 5
grep -h '^{' gpurun_out/mx_b1_base.log gpurun_out/mx_b1_tuned.log gpurun_out/mx_b1_base2.log | cut -c150-240
# Mixtral B=256: alternative grouped-expert GEMM configs (NLS_MOE_QCFG_GU/_DN = mode,waves,rt)
run() { local n=$1; shift; step mx256_$n 400 env "$@" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model mixtral-8x7b --ftype Q5_K_M --concurrency 256 --steps 20 --warmup 3; }
run base NLS_X=0
run gu282 NLS_MOE_QCFG_GU=2,8,2
run gu181 NLS_MOE_QCFG_GU=1,8,1
run dn181 NLS_MOE_QCFG_DN=1,8,1
for f in base gu282 gu181 dn181; do echo "$f $(grep -h '^{' gpurun_out/mx256_$f.log | cut -c150-230)"; done
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
