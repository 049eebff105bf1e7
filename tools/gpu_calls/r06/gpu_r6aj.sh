#!/bin/bash
# round 6, call AJ: sustained (200 timed steps) quantised-only vs f16 copies at B=512 -- the copies run into the package
# power limit harder (more HBM bytes per step); does the 20-step gap hold over a sustained window?
source tools/gpu_steps.sh
B="python3 -u bench.py --warmup 5 --no-rtt --serve-load 0"
step r6aj_copies_200 600 $B --steps 200
NLS_DENSE_WEIGHTS=0 step r6aj_quant_200 600 $B --steps 200
step r6aj_copies_20 300 $B --steps 20
NLS_DENSE_WEIGHTS=0 step r6aj_quant_20 300 $B --steps 20
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
