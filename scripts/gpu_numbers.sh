#!/bin/bash
# Round numbers: context sweep on Llama-3-8B, then the other north-star families
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ctx_sweep.sh || exit $?
RUNS=${RUNS:-"mixtral_b1 mixtral_b256 l70b_b1 l70b_b128 qwen7b_b512"} bash tools/gpu_models.sh
