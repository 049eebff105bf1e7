"""MI355X-native NATS LLM worker (capabilities of Dsouza10082/nats-llm-studio, rebuilt from scratch).

Layers: natsio (C++ NATS wire core) -> service (subjects/envelope) ->
engine (scheduler, paged KV, hipGraph decode) -> models (llama/granite/mixtral) ->
ops (hand-written gfx950 HIP kernels) -> parallel (RCCL TP/EP over xGMI).
"""
__version__ = "0.1.0"
