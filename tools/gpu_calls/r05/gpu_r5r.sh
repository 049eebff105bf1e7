#!/bin/bash
# round 5, call R: Mixtral B=256 expert GEMMs on path B (mode 1: waves split rows, LDS-staged activations) vs mode 2.
source tools/gpu_steps.sh
for p in gateup down; do
  for c in 2,8,4,1 1,8,1,1 1,8,2,1 1,4,1,1 1,4,2,1; do
    step r5r_${p}_${c//,/_} 120 python3 -u tools/diag/moe_probe.py --proj $p --T 256 --cfg $c
  done
done
exit $STEPS_RC
