"""Independent fp32 PyTorch reference forward (the correctness oracle).

Reads weights straight from the GGUF via the numpy ggml codecs (no device
layouts, no paging, no fused epilogues) and runs a textbook decoder over a full
token sequence. Engine/kernels are compared against this.
"""
from __future__ import annotations

import numpy as np
import torch

from ..gguf.reader import GGUFReader
from .config import ModelConfig


class ReferenceModel:
    def __init__(self, reader: GGUFReader):
        self.r = reader
        self.cfg = ModelConfig.from_gguf(reader.metadata, reader.tensors.keys())
        self._cache = {}

    def w(self, name) -> torch.Tensor:
        if name not in self._cache:
            self._cache[name] = torch.from_numpy(self.r.dequantized(name).astype(np.float32).copy())
        return self._cache[name]

    @staticmethod
    def _rms(x, w, eps):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w

    def _rope(self, x, pos):   # x [S, H, D], adjacent-pair (GGUF llama) rotation
        cfg = self.cfg
        D = x.shape[-1]
        inv = 1.0 / (cfg.rope_base ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
        if "rope_freqs.weight" in self.r.tensors:         # Llama-3.1+ frequency factors
            inv = inv / self.w("rope_freqs.weight").double().reshape(-1)[:D // 2]
        ang = ((pos.double() * cfg.rope_pos_scale)[:, None] * inv[None, :]).float()
        c, s = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
        if cfg.rope_neox:                                  # (i, i + D/2) pairs (Qwen2)
            x0, x1 = x[..., :D // 2], x[..., D // 2:]
            return torch.cat([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1)
        x0, x1 = x[..., 0::2], x[..., 1::2]
        return torch.stack([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1).flatten(-2)

    @torch.no_grad()
    def logits(self, ids) -> torch.Tensor:
        """ids: list[int] -> logits [S, V] for every position (causal)."""
        cfg = self.cfg
        S = len(ids)
        H, Hkv, D = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        G = H // Hkv
        x = self.w("token_embd.weight")[torch.tensor(ids)] * cfg.embedding_scale
        pos = torch.arange(S)
        mask = torch.full((S, S), float("-inf")).triu(1)
        for i in range(cfg.n_layer):
            p = f"blk.{i}."
            h = self._rms(x, self.w(p + "attn_norm.weight"), cfg.eps)
            q, k, v = (h @ self.w(p + f"attn_{n}.weight").t() + (self.w(p + f"attn_{n}.bias")
                       if p + f"attn_{n}.bias" in self.r.tensors else 0.0) for n in "qkv")
            q, k, v = q.view(S, H, D), k.view(S, Hkv, D), v.view(S, Hkv, D)
            q, k = self._rope(q, pos), self._rope(k, pos)
            k = k.repeat_interleave(G, dim=1)
            v = v.repeat_interleave(G, dim=1)
            sc = torch.einsum("shd,thd->hst", q, k) * cfg.attn_softmax_scale + mask
            o = torch.einsum("hst,thd->shd", torch.softmax(sc, -1), v).reshape(S, H * D)
            x = x + cfg.residual_scale * (o @ self.w(p + "attn_output.weight").t())
            h = self._rms(x, self.w(p + "ffn_norm.weight"), cfg.eps)
            if cfg.n_expert:
                rl = h @ self.w(p + "ffn_gate_inp.weight").t()
                pr = torch.softmax(rl, -1)
                tw, te = torch.topk(pr, cfg.n_expert_used, -1)
                tw = tw / tw.sum(-1, keepdim=True)
                gw, uw, dw = self.w(p + "ffn_gate_exps.weight"), self.w(p + "ffn_up_exps.weight"), \
                    self.w(p + "ffn_down_exps.weight")
                out = torch.zeros_like(x)
                for s in range(S):
                    for j in range(cfg.n_expert_used):
                        e = int(te[s, j])
                        a = torch.nn.functional.silu(h[s] @ gw[e].t()) * (h[s] @ uw[e].t())
                        out[s] += tw[s, j] * (a @ dw[e].t())
                x = x + cfg.residual_scale * out
            else:
                a = torch.nn.functional.silu(h @ self.w(p + "ffn_gate.weight").t()) * (h @ self.w(p + "ffn_up.weight").t())
                x = x + cfg.residual_scale * (a @ self.w(p + "ffn_down.weight").t())
        h = self._rms(x, self.w("output_norm.weight"), cfg.eps)
        head = "token_embd.weight" if cfg.tied_embeddings else "output.weight"
        return (h @ self.w(head).t()) / cfg.logit_scale

    def greedy(self, ids, n_new: int):
        ids = list(ids)
        out = []
        for _ in range(n_new):
            nxt = int(self.logits(ids)[-1].argmax())
            out.append(nxt)
            ids.append(nxt)
        return out
