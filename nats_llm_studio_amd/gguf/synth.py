"""Random-init GGUF checkpoints of the north-star architectures.

BASELINE.json configs: Llama-3-8B Q4_K, Llama-3-70B Q4_K, Mixtral-8x7B Q5_K,
Granite-3.0-2B (stub backend). Shapes follow the public HF configs; the
quantisation mix follows llama.cpp's Q4_K_M / Q5_K_M recipe (attn_v and
ffn_down get Q6_K on the "more bits" layers, output.weight is Q6_K).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, replace
from typing import Dict, Optional

import numpy as np

from .constants import FILE_TYPE_IDS, GGMLType
from .quants import random_blocks
from .writer import GGUFWriter
from ..tokenizer import synthetic as tsyn


@dataclass(frozen=True)
class ModelSpec:
    name: str
    arch: str                     # gguf general.architecture
    n_layer: int
    d_model: int
    n_head: int
    n_kv_head: int
    d_ff: int
    vocab: int
    ctx: int = 8192
    rope_base: float = 500000.0
    eps: float = 1e-5
    n_expert: int = 0
    n_expert_used: int = 0
    tokenizer: str = "gpt2"       # gpt2 (byte-level BPE) | llama (SPM)
    tied_embeddings: bool = False
    # granite multipliers
    embedding_scale: float = 1.0
    residual_scale: float = 1.0
    attention_scale: float = 0.0  # 0 -> 1/sqrt(head_dim)
    logit_scale: float = 1.0
    publisher: str = "synthetic"
    rope_freqs: bool = False      # Llama-3.1-style `rope_freqs.weight` frequency factors

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_head


SPECS: Dict[str, ModelSpec] = {
    "llama-3-8b": ModelSpec("llama-3-8b", "llama", 32, 4096, 32, 8, 14336, 128256, 8192, 500000.0),
    # Llama-3.1-8B: the same shapes with the 128K context and rope_freqs scaling (long-context sweeps)
    "llama-3.1-8b": ModelSpec("llama-3.1-8b", "llama", 32, 4096, 32, 8, 14336, 128256, 131072, 500000.0,
                              rope_freqs=True),
    "llama-3-70b": ModelSpec("llama-3-70b", "llama", 80, 8192, 64, 8, 28672, 128256, 8192, 500000.0),
    "mixtral-8x7b": ModelSpec("mixtral-8x7b", "llama", 32, 4096, 32, 8, 14336, 32000, 32768, 1e6,
                              n_expert=8, n_expert_used=2, tokenizer="llama"),
    "granite-3.0-2b": ModelSpec("granite-3.0-2b", "granite", 40, 2048, 32, 8, 8192, 49155, 4096, 10000.0,
                                tied_embeddings=True, embedding_scale=12.0, residual_scale=0.22,
                                attention_scale=0.015625, logit_scale=8.0),
    # tiny shapes for CPU / kernel tests (all dims multiples of 256)
    "tiny-llama": ModelSpec("tiny-llama", "llama", 2, 512, 4, 2, 768, 1024, 512, 10000.0),
    # TP-shardable tiny shape (TP=2: per-rank FFN 512, one kv head each) for CPU multi-rank benches
    "tiny-llama-tp": ModelSpec("tiny-llama-tp", "llama", 2, 512, 4, 2, 1024, 1024, 512, 10000.0),
    # Llama-3-70B per-layer shapes (d 8192, 64 q / 8 kv heads, FFN 28672) with ONE layer and a 4K vocab: the
    # CPU rehearsal of the TP=4/8 data plane (bench.py TP leg on --device cpu, tests/test_parallel_shapes.py)
    "llama-3-70b-1layer": ModelSpec("llama-3-70b-1layer", "llama", 1, 8192, 64, 8, 28672, 4096, 512, 500000.0),
    # two Llama-3-70B layers / one Mixtral-8x7B layer with a 32K vocab: the multi-process, one-GPU rehearsal of
    # the TP / EP decode graphs (parallel/rehearsal.py, tests/test_tp_rehearsal_gpu.py)
    "llama-3-70b-2layer": ModelSpec("llama-3-70b-2layer", "llama", 2, 8192, 64, 8, 28672, 32000, 1024, 500000.0),
    "mixtral-8x7b-1layer": ModelSpec("mixtral-8x7b-1layer", "llama", 1, 4096, 32, 8, 14336, 32000, 1024, 1e6,
                                     n_expert=8, n_expert_used=2, tokenizer="llama"),
    "tiny-mixtral-tp": ModelSpec("tiny-mixtral-tp", "llama", 2, 512, 4, 2, 512, 1024, 512, 10000.0,
                                 n_expert=4, n_expert_used=2, tokenizer="llama"),
    "tiny-mixtral": ModelSpec("tiny-mixtral", "llama", 2, 512, 4, 2, 512, 1024, 512, 10000.0,
                              n_expert=4, n_expert_used=2, tokenizer="llama"),
    "qwen2.5-7b": ModelSpec("qwen2.5-7b", "qwen2", 28, 3584, 28, 4, 18944, 152064, 32768, 1e6, eps=1e-6),
    "tiny-qwen2": ModelSpec("tiny-qwen2", "qwen2", 2, 512, 4, 2, 768, 1000, 512, 1e6, eps=1e-6, tied_embeddings=True),
    "tiny-llama31": ModelSpec("tiny-llama31", "llama", 2, 512, 4, 2, 768, 1024, 512, 500000.0, rope_freqs=True),
    "tiny-granite": ModelSpec("tiny-granite", "granite", 2, 512, 8, 2, 768, 1000, 512, 10000.0,
                              tied_embeddings=True, embedding_scale=12.0, residual_scale=0.22,
                              attention_scale=0.015625, logit_scale=8.0),
}

QUANT_MIX = {
    # ftype name: (base type, "more bits" type, output type, token_embd type)
    "Q4_K_M": (GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q6_K, GGMLType.Q4_K),
    "Q5_K_M": (GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q6_K, GGMLType.Q5_K),
    "Q6_K": (GGMLType.Q6_K, GGMLType.Q6_K, GGMLType.Q6_K, GGMLType.Q6_K),
    "Q8_0": (GGMLType.Q8_0, GGMLType.Q8_0, GGMLType.Q8_0, GGMLType.Q8_0),
    # the legacy 32-block types and the low-bit K mixes (llama.cpp keeps output.weight at Q6_K)
    "Q4_0": (GGMLType.Q4_0, GGMLType.Q4_0, GGMLType.Q6_K, GGMLType.Q4_0),
    "Q4_1": (GGMLType.Q4_1, GGMLType.Q4_1, GGMLType.Q6_K, GGMLType.Q4_1),
    "Q5_0": (GGMLType.Q5_0, GGMLType.Q5_0, GGMLType.Q6_K, GGMLType.Q5_0),
    "Q5_1": (GGMLType.Q5_1, GGMLType.Q5_1, GGMLType.Q6_K, GGMLType.Q5_1),
    "Q3_K_M": (GGMLType.Q3_K, GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q3_K),
    "Q2_K": (GGMLType.Q2_K, GGMLType.Q3_K, GGMLType.Q6_K, GGMLType.Q2_K),
    "F16": (GGMLType.F16, GGMLType.F16, GGMLType.F16, GGMLType.F16),
    "F32": (GGMLType.F32, GGMLType.F32, GGMLType.F32, GGMLType.F32),
}


def use_more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_plan(spec: ModelSpec, ftype: str):
    """Yield (name, np_shape, ggml_type, std) for every tensor of the checkpoint."""
    base, more, out_t, emb_t = QUANT_MIX[ftype]
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    std = 0.02
    plan = [("token_embd.weight", (spec.vocab, d), emb_t, std * 2)]
    if spec.rope_freqs:
        plan.append(("rope_freqs.weight", (hd // 2,), GGMLType.F32, -2.0))
    for i in range(spec.n_layer):
        p = f"blk.{i}."
        mb = use_more_bits(i, spec.n_layer)
        plan += [
            (p + "attn_norm.weight", (d,), GGMLType.F32, -1.0),
            (p + "attn_q.weight", (nq, d), base, std),
            (p + "attn_k.weight", (nkv, d), base, std),
            (p + "attn_v.weight", (nkv, d), more if mb else base, std),
            (p + "attn_output.weight", (d, nq), base, std / np.sqrt(2 * spec.n_layer) * 4),
        ] + ([(p + "attn_q.bias", (nq,), GGMLType.F32, -3.0), (p + "attn_k.bias", (nkv,), GGMLType.F32, -3.0),
              (p + "attn_v.bias", (nkv,), GGMLType.F32, -3.0)] if spec.arch == "qwen2" else []) + [
            (p + "ffn_norm.weight", (d,), GGMLType.F32, -1.0),
        ]
        if spec.n_expert:
            e = spec.n_expert
            plan += [
                (p + "ffn_gate_inp.weight", (e, d), GGMLType.F32, std * 4),
                (p + "ffn_gate_exps.weight", (e, spec.d_ff, d), base, std),
                (p + "ffn_up_exps.weight", (e, spec.d_ff, d), base, std),
                (p + "ffn_down_exps.weight", (e, d, spec.d_ff), more if mb else base, std),
            ]
        else:
            plan += [
                (p + "ffn_gate.weight", (spec.d_ff, d), base, std),
                (p + "ffn_up.weight", (spec.d_ff, d), base, std),
                (p + "ffn_down.weight", (d, spec.d_ff), more if mb else base, std / np.sqrt(2 * spec.n_layer) * 4),
            ]
    plan.append(("output_norm.weight", (d,), GGMLType.F32, -1.0))
    if not spec.tied_embeddings:
        plan.append(("output.weight", (spec.vocab, d), out_t, std))
    return plan


def _metadata(w: GGUFWriter, spec: ModelSpec, ftype: str, name: str):
    a = spec.arch
    w.add("general.name", name)
    w.add("general.type", "model")
    w.add("general.organization", spec.publisher)
    w.add("general.file_type", FILE_TYPE_IDS[ftype])
    w.add("general.quantization_version", 2)
    w.add(f"{a}.context_length", spec.ctx)
    w.add(f"{a}.embedding_length", spec.d_model)
    w.add(f"{a}.block_count", spec.n_layer)
    w.add(f"{a}.feed_forward_length", spec.d_ff)
    w.add(f"{a}.attention.head_count", spec.n_head)
    w.add(f"{a}.attention.head_count_kv", spec.n_kv_head)
    w.add(f"{a}.rope.freq_base", float(spec.rope_base))
    w.add(f"{a}.rope.dimension_count", spec.head_dim)
    w.add(f"{a}.attention.layer_norm_rms_epsilon", float(spec.eps))
    w.add(f"{a}.vocab_size", spec.vocab)
    if spec.n_expert:
        w.add(f"{a}.expert_count", spec.n_expert)
        w.add(f"{a}.expert_used_count", spec.n_expert_used)
    if a == "granite":
        w.add(f"{a}.embedding_scale", float(spec.embedding_scale))
        w.add(f"{a}.residual_scale", float(spec.residual_scale))
        w.add(f"{a}.attention.scale", float(spec.attention_scale))
        w.add(f"{a}.logit_scale", float(spec.logit_scale))
    if spec.tokenizer == "gpt2":
        if a == "qwen2":
            tokens, types, merges, ids = tsyn.bytelevel_vocab(spec.vocab, tsyn.QWEN2_SPECIALS)
            bos, eos = ids["<|endoftext|>"], ids["<|im_end|>"]
            tmpl, add_bos = tsyn.CHATML_TEMPLATE, False
            pre = "qwen2"
        elif a == "granite":
            specials = ["<|end_of_text|>", "<|start_of_role|>", "<|end_of_role|>", "<|tool_call|>"]
            tokens, types, merges, ids = tsyn.bytelevel_vocab(spec.vocab, specials)
            bos = eos = ids["<|end_of_text|>"]
            tmpl, add_bos = tsyn.GRANITE_TEMPLATE, False
            pre = "refact"
        else:
            tokens, types, merges, ids = tsyn.bytelevel_vocab(spec.vocab)
            bos, eos = ids["<|begin_of_text|>"], ids["<|eot_id|>"]
            tmpl, add_bos = tsyn.LLAMA3_TEMPLATE, True
            pre = "llama-bpe"
        w.add("tokenizer.ggml.model", "gpt2")
        w.add("tokenizer.ggml.pre", pre)
        w.add("tokenizer.ggml.tokens", tokens)
        w.add("tokenizer.ggml.token_type", np.asarray(types, np.int32))
        w.add("tokenizer.ggml.merges", merges)
        w.add("tokenizer.ggml.bos_token_id", bos)
        w.add("tokenizer.ggml.eos_token_id", eos)
        w.add("tokenizer.ggml.add_bos_token", add_bos)
        w.add("tokenizer.chat_template", tmpl)
    else:
        tokens, types, scores = tsyn.spm_vocab(spec.vocab)
        w.add("tokenizer.ggml.model", "llama")
        w.add("tokenizer.ggml.tokens", tokens)
        w.add("tokenizer.ggml.scores", np.asarray(scores, np.float32))
        w.add("tokenizer.ggml.token_type", np.asarray(types, np.int32))
        w.add("tokenizer.ggml.bos_token_id", 1)
        w.add("tokenizer.ggml.eos_token_id", 2)
        w.add("tokenizer.ggml.add_bos_token", True)
        w.add("tokenizer.chat_template", tsyn.MISTRAL_TEMPLATE)


def llama3_rope_factors(head_dim: int, base: float, factor: float = 8.0, low: float = 1.0, high: float = 4.0,
                        orig_ctx: int = 8192) -> np.ndarray:
    """Per-frequency divisors of Llama-3.1 RoPE scaling (what convert_hf_to_gguf stores in rope_freqs)."""
    inv = 1.0 / (base ** (np.arange(0, head_dim, 2, dtype=np.float64) / head_dim))
    wl = 2 * np.pi / inv
    lo_wl, hi_wl = orig_ctx / low, orig_ctx / high
    smooth = (orig_ctx / wl - low) / (high - low)
    return np.where(wl < hi_wl, 1.0, np.where(wl > lo_wl, factor, 1.0 / ((1 - smooth) / factor + smooth)))


def write_synthetic_gguf(path: str, spec_name: str, ftype: str = "Q4_K_M", seed: int = 0,
                         progress=None, spec: Optional[ModelSpec] = None) -> str:
    spec = spec or SPECS[spec_name]
    rng = np.random.default_rng(seed)
    w = GGUFWriter(path, spec.arch)
    _metadata(w, spec, ftype, os.path.splitext(os.path.basename(path))[0])
    for name, shape, gt, std in tensor_plan(spec, ftype):
        n = int(np.prod(shape))
        if std == -2.0:   # rope frequency factors (llama.cpp llama3 recipe: factor 8, low/high 1/4)
            def prod(n=n):
                return llama3_rope_factors(2 * n, spec.rope_base).astype(np.float32).view(np.uint8)
        elif std == -3.0:   # projection biases: small
            def prod(n=n):
                return (0.1 * rng.standard_normal(n)).astype(np.float32).view(np.uint8)
        elif std < 0:   # norm weights: ~1
            def prod(n=n):
                return (1.0 + 0.1 * rng.standard_normal(n).astype(np.float32)).view(np.uint8)
        else:
            def prod(gt=gt, n=n, std=std):
                return random_blocks(gt, n, std, rng)
        w.add_tensor(name, shape, gt, prod)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".part"
    w.path = tmp
    w.write(progress)
    os.replace(tmp, path)
    return path


def model_dir_name(spec_name: str, ftype: str) -> str:
    return f"{spec_name}-{ftype}-GGUF"


def materialize(models_dir: str, spec_name: str, ftype: str = "Q4_K_M", seed: int = 0,
                publisher: str = "synthetic") -> str:
    """Write `<models_dir>/<publisher>/<model>-GGUF/<model>-<ftype>.gguf` if absent (LM Studio tree)."""
    d = os.path.join(models_dir, publisher, model_dir_name(spec_name, ftype))
    path = os.path.join(d, f"{spec_name}-{ftype}.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(path, spec_name, ftype, seed)
    return path
