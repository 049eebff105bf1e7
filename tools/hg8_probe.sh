#!/usr/bin/env bash
# Build and run the mode-8 speed-of-light probes (tools/hg8_probe.hip) on the GPU box.
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/h8
PROBES=${PROBES:-0 1 2 4 3}
# PROBES: H8 bits (mode 8), PROBES9: H9 bits (mode 9; binaries q<bits>)
for P in $PROBES; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -DH8_PROBE=$P tools/hg8_probe.hip -o gpurun_out/h8/p$P 2>/dev/null & done
for P in ${PROBES9:-}; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -DH9_PROBE=$P tools/hg8_probe.hip -o gpurun_out/h8/q$P 2>/dev/null & done
wait
for P in $PROBES; do
  while read -r args; do timeout -k 5 60 gpurun_out/h8/p$P $args; done <<< "${SHAPES:-512 224 28672 4096 3}"
done
for P in ${PROBES9:-}; do
  while read -r args; do timeout -k 5 60 gpurun_out/h8/q$P $args; done <<< "${SHAPES9:-512 256 28672 4096 3 1 12}"
done
