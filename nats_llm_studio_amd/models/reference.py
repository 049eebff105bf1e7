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
    """device: where the fp32 math runs (a GPU oracle for full-size models; the weights are still decoded
    by the numpy codecs of gguf/quants.py, never by the kernels under test). cache=False streams them
    (each tensor decoded when used, then dropped: an 8B model never sits in host memory as fp32);
    workers > 1 decodes a tensor's row ranges in parallel threads."""

    def __init__(self, reader: GGUFReader, device=None, cache: bool = True, workers: int = 1,
                 storage_rounding: bool = False):
        """storage_rounding: round the tensors the engine STORES in narrower types at the same points
        (GEMM inputs h / attention output / SwiGLU output to f16, q and the K/V cache to bf16), all math
        still fp32 -- separates the engine's storage precision from kernel error in a comparison."""
        self.rnd = storage_rounding
        self.r = reader
        self.cfg = ModelConfig.from_gguf(reader.metadata, reader.tensors.keys())
        self._cache = {}
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.cache = cache
        self.workers = max(1, int(workers))
        self._pool = None

    def _decode(self, name, r0=None, r1=None) -> np.ndarray:
        """fp32 rows [r0, r1) of a tensor (all rows by default), straight from its GGUF bytes."""
        from ..gguf.quants import dequantize
        ti = self.r.tensors[name]
        shape = ti.np_shape
        rows = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
        r0, r1 = (0, rows) if r0 is None else (r0, r1)
        rb = ti.nbytes // rows
        K = shape[-1]
        n = r1 - r0
        if self.workers == 1 or n < 2 * self.workers:
            out = dequantize(ti.data[r0 * rb:r1 * rb], ti.ggml_type, (n, K))
        else:
            from concurrent.futures import ThreadPoolExecutor
            if self._pool is None:
                self._pool = ThreadPoolExecutor(self.workers)
            cuts = np.linspace(r0, r1, self.workers + 1).astype(int)
            parts = self._pool.map(lambda c: dequantize(ti.data[c[0] * rb:c[1] * rb], ti.ggml_type, (c[1] - c[0], K)),
                                   [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:]) if b > a])
            out = np.concatenate(list(parts), axis=0)
        if r0 == 0 and r1 == rows:
            out = out.reshape(shape)
        return out.astype(np.float32, copy=False)

    def w(self, name) -> torch.Tensor:
        if name in self._cache:
            return self._cache[name]
        t = torch.from_numpy(np.ascontiguousarray(self._decode(name))).to(self.device)
        if self.cache:
            self._cache[name] = t
        return t

    def rows(self, name, ids) -> torch.Tensor:
        """Gathered rows of a 2-D tensor (embedding lookup) without decoding the whole table."""
        if name in self._cache:
            return self._cache[name][torch.as_tensor(ids, device=self.device)]
        out = [torch.from_numpy(self._decode(name, int(i), int(i) + 1)) for i in ids]
        return torch.cat(out, 0).to(self.device)

    def _st(self, t, dtype):
        return t.to(dtype).float() if self.rnd else t

    @staticmethod
    def _rms(x, w, eps):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w

    def _rope(self, x, pos):   # x [S, H, D], adjacent-pair (GGUF llama) rotation
        cfg = self.cfg
        D = x.shape[-1]
        inv = 1.0 / (cfg.rope_base ** (torch.arange(0, D, 2, dtype=torch.float64, device=x.device) / D))
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
        dev = self.device
        x = self.rows("token_embd.weight", ids) * cfg.embedding_scale
        pos = torch.arange(S, device=dev)
        mask = torch.full((S, S), float("-inf"), device=dev).triu(1)
        for i in range(cfg.n_layer):
            p = f"blk.{i}."
            h = self._st(self._rms(x, self.w(p + "attn_norm.weight"), cfg.eps), torch.float16)
            q, k, v = (h @ self.w(p + f"attn_{n}.weight").t() + (self.w(p + f"attn_{n}.bias")
                       if p + f"attn_{n}.bias" in self.r.tensors else 0.0) for n in "qkv")
            q, k, v = q.view(S, H, D), k.view(S, Hkv, D), v.view(S, Hkv, D)
            q, k = self._rope(q, pos), self._rope(k, pos)
            q, k, v = (self._st(t, torch.bfloat16) for t in (q, k, v))
            k = k.repeat_interleave(G, dim=1)
            v = v.repeat_interleave(G, dim=1)
            sc = torch.einsum("shd,thd->hst", q, k) * cfg.attn_softmax_scale + mask
            o = self._st(torch.einsum("hst,thd->shd", torch.softmax(sc, -1), v).reshape(S, H * D), torch.float16)
            x = x + cfg.residual_scale * (o @ self.w(p + "attn_output.weight").t())
            h = self._st(self._rms(x, self.w(p + "ffn_norm.weight"), cfg.eps), torch.float16)
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
                a = self._st(a, torch.float16)
                x = x + cfg.residual_scale * (a @ self.w(p + "ffn_down.weight").t())
        h = self._st(self._rms(x, self.w("output_norm.weight"), cfg.eps), torch.float16)
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
