#!/usr/bin/env bash
# Host bootstrap (replaces the reference's scripts/setup_unix.sh, which installed LM Studio +
# a downloaded nats-server binary): build the native parts in-tree, write .env with the README's
# variables, and start the native NATS server (JetStream on, file store) unless one is running.
#
#   scripts/setup_host.sh [--port 4222] [--store-dir ./nats_data] [--models-dir ~/.lmstudio/models]
#                         [--no-server]
set -euo pipefail
cd "$(dirname "$0")/.."
PORT=4222
STORE=./nats_data
MODELS="${MODELS_DIR:-${LMSTUDIO_MODELS_DIR:-$HOME/.lmstudio/models}}"
START=1
while [ $# -gt 0 ]; do
  case "$1" in
    --port) PORT=$2; shift 2 ;;
    --store-dir) STORE=$2; shift 2 ;;
    --models-dir) MODELS=$2; shift 2 ;;
    --no-server) START=0; shift ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
done

echo "[setup] building HIP kernels (gfx950), natscore extension and the nls-nats CLI"
python3 -m nats_llm_studio_amd.build

mkdir -p "$MODELS" "$STORE"
if [ ! -f .env ]; then
  cat > .env <<ENV
NATS_URL=nats://127.0.0.1:${PORT}
MODELS_DIR=${MODELS}
# LMSTUDIO_MODELS_DIR is accepted as an alias of MODELS_DIR
NATS_QUEUE_GROUP=lmstudio-workers
BUCKET=llm-models
# BACKEND=engine | stub | http (http = proxy to an LM Studio server at LMSTUDIO_BASE_URL)
BACKEND=engine
LMSTUDIO_BASE_URL=http://127.0.0.1:1234
MAX_BATCH=64
ENV
  echo "[setup] wrote .env"
fi

if [ "$START" = 1 ]; then
  if bin/nls-nats --server "nats://127.0.0.1:${PORT}" pub _setup.probe x --timeout 1 >/dev/null 2>&1; then
    echo "[setup] a NATS server already answers on :${PORT}"
  else
    nohup bin/nls-nats server --port "$PORT" --store-dir "$STORE" > nats_server.log 2>&1 &
    echo "[setup] nls-nats server (JetStream, store ${STORE}) started on :${PORT}, pid $!"
  fi
fi
cat <<MSG
[setup] done. Start workers with:
  scripts/run_workers.sh --gpus 8                   # 8 replicas (one per GPU) in the queue group
  scripts/run_workers.sh --tp 8 --model <id|path>   # one tensor-parallel worker over 8 GPUs
MSG
