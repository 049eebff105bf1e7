#!/usr/bin/env bash
# Launch workers on this node.
#   --gpus N            N independent replicas, one per GPU, same NATS queue group (README.md:478-484)
#   --tp N --model M    one tensor-parallel worker: torchrun, one rank per GPU, rank 0 on NATS
#   --ep                with --tp: MoE experts expert-parallel instead of TP-sharded
# Extra arguments are passed to `python -m nats_llm_studio_amd.worker`.
set -euo pipefail
cd "$(dirname "$0")/.."
GPUS=1
TP=1
EXTRA=()
while [ $# -gt 0 ]; do
  case "$1" in
    --gpus) GPUS=$2; shift 2 ;;
    --tp) TP=$2; shift 2 ;;
    *) EXTRA+=("$1"); shift ;;
  esac
done
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$TP" -gt 1 ]; then
  exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$TP" --master-addr 127.0.0.1 \
       --master-port "${MASTER_PORT:-29511}" -m nats_llm_studio_amd.worker --tp "$TP" "${EXTRA[@]}"
fi
pids=()
for ((i = 0; i < GPUS; i++)); do
  HIP_VISIBLE_DEVICES=$i python3 -m nats_llm_studio_amd.worker --device cuda:0 "${EXTRA[@]}" \
      > "worker_gpu$i.log" 2>&1 &
  pids+=($!)
  echo "worker on GPU $i: pid ${pids[-1]} (log worker_gpu$i.log)"
done
trap 'kill "${pids[@]}" 2>/dev/null' INT TERM
wait
