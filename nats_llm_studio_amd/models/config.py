"""Model hyper-parameters read from GGUF metadata (llama / mixtral / granite families)."""
from __future__ import annotations

from dataclasses import dataclass

SUPPORTED_ARCHS = ("llama", "granite", "mistral", "mixtral", "qwen2")
NEOX_ARCHS = ("qwen2",)           # llama.cpp LLAMA_ROPE_TYPE_NEOX families


@dataclass
class ModelConfig:
    arch: str
    n_layer: int
    d_model: int
    n_head: int
    n_kv_head: int
    head_dim: int
    d_ff: int
    vocab: int
    ctx: int
    rope_base: float
    eps: float
    n_expert: int = 0
    n_expert_used: int = 0
    tied_embeddings: bool = False
    embedding_scale: float = 1.0
    residual_scale: float = 1.0
    attention_scale: float = 0.0
    logit_scale: float = 1.0
    rope_neox: bool = False
    rope_pos_scale: float = 1.0      # 1 / rope.scaling.factor for linear scaling

    @property
    def attn_softmax_scale(self) -> float:
        return self.attention_scale if self.attention_scale > 0 else self.head_dim ** -0.5

    @property
    def q_dim(self) -> int:
        return self.n_head * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_head * self.head_dim

    @classmethod
    def from_gguf(cls, md: dict, tensor_names=()) -> "ModelConfig":
        a = str(md["general.architecture"])
        if a not in SUPPORTED_ARCHS:
            raise NotImplementedError(f"architecture {a!r} not supported (supported: {SUPPORTED_ARCHS})")

        def g(k, d=None):
            return md.get(f"{a}.{k}", d)

        d = int(g("embedding_length"))
        nh = int(g("attention.head_count"))
        nkv = int(g("attention.head_count_kv", nh))
        hd = int(g("attention.key_length", d // nh))
        vocab = g("vocab_size")
        if vocab is None:
            vocab = len(md.get("tokenizer.ggml.tokens", []))
        return cls(
            arch=a, n_layer=int(g("block_count")), d_model=d, n_head=nh, n_kv_head=nkv, head_dim=hd,
            d_ff=int(g("feed_forward_length")), vocab=int(vocab), ctx=int(g("context_length", 4096)),
            rope_base=float(g("rope.freq_base", 10000.0)), eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
            n_expert=int(g("expert_count", 0) or 0), n_expert_used=int(g("expert_used_count", 0) or 0),
            tied_embeddings="output.weight" not in set(tensor_names) if tensor_names else False,
            embedding_scale=float(g("embedding_scale", 1.0)), residual_scale=float(g("residual_scale", 1.0)),
            attention_scale=float(g("attention.scale", 0.0)), logit_scale=float(g("logit_scale", 1.0)),
            rope_neox=a in NEOX_ARCHS,
            rope_pos_scale=(1.0 / float(g("rope.scaling.factor", 1.0) or 1.0)
                            if str(g("rope.scaling.type", "none")) == "linear" else 1.0),
        )
