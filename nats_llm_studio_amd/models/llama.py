"""Llama-family decoder (Llama-3, Mistral/Mixtral MoE, Granite) executing on GGUF
quantised weights with the gfx950 kernels of `nats_llm_studio_amd.ops`.

This is the co-located engine that replaces LM Studio's llama.cpp runtime behind
`POST /api/v0/chat/completions` (`/root/reference/nats_llm_studio.go:158-179`).

Per layer a few-row decode step (single GPU) is 5 launches:
  QKV GEMV (Q|K|V segments, per-tensor quant type) with RoPE + paged KV append in its epilogue
  -> paged GQA attention (flash-decoding splits merged in-kernel by the last split)
  -> O GEMV + residual, the next RMSNorm run by its last workgroup
  -> gate|up GEMV with fused SwiGLU -> down GEMV + residual + next RMSNorm (last workgroup)
Large batches use the split-K / LDS GEMMs with fused reduce+RoPE and reduce+residual+RMSNorm
kernels instead. The whole step is captured once per batch bucket in a hipGraph by the engine.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..gguf.constants import GGMLType, GGML_BLOCK
from ..gguf.reader import GGUFReader
from ..ops import QWeight, Seg, tuning
from .config import ModelConfig


# flash-decoding splits per (token, kv head): up to 64 (only batch <= 2 reaches it; the kernel's context-adaptive
# chunk keeps 4K context at 16 x 256 keys, which beat 32 x 128 -- profiles/attn_split_cap_4k.txt -- and gives
# 8K-32K contexts 32-64 splits; profiles/ctx_sweep_r03_splits.jsonl)
_SPLIT_CAP = int(os.environ.get("NLS_ATTN_SPLIT_CAP", "64"))
# target workgroups of a decode attention launch: 256 = one 8-wave workgroup per CU (attention.hip picks 8 waves
# for grids of <= 256 workgroups); batch 1 then splits 32 ways, batch 16 two ways
_SPLIT_WG = int(os.environ.get("NLS_ATTN_SPLIT_WG", "256"))
# fewest keys per flash-decoding split (0: the kernel's context-adaptive policy, attention.hip
# split_chunk: 64 keys below 1K of context, 128 above)
_MIN_CHUNK = int(os.environ.get("NLS_ATTN_MIN_CHUNK", "0"))
# MoE: tokens per step above which the experts run as ONE grouped LDS-dequant GEMM launch (below: path-A
# GEMVs over each expert's gathered rows)
# (Mixtral-8x7B: B=64 15.2 vs 28.9 ms/step, B=32 15.2 vs 15.6, B=16 14.8 vs 9.7; round-2 sweep)
_MOE_GEMM_T = int(os.environ.get("NLS_MOE_GEMM_T", "16"))
# MoE decode at up to this many tokens (<= 4) fuses the FFN input RMSNorm, the router and the route
# into one launch (ops.moe_norm_route); 0 disables
_MOE_NORM_ROUTE_T = min(4, int(os.environ.get("NLS_MOE_NORM_ROUTE", "4")))
# ... and with NLS_MOE_FOLD_ROUTE=1 that launch is folded into the o projection's last workgroup. Off: the
# last-arriver tail (norm, E router dot products, route on one workgroup) measured slower than the launch it
# removes (Mixtral batch 1: 3.50 vs 3.25 ms/token, batch 4: 7.38 vs 6.85; profiles/mixtral_b1_r03.txt)
_MOE_FOLD_ROUTE = os.environ.get("NLS_MOE_FOLD_ROUTE", "0") == "1"
# MoE decode (path-A expert GEMVs): launch config (mode, waves, rt, ks) of the DOWN projection, whose
# K (d_ff) is 3.5x the gate/up's; empty: ops.MOE_GEMV like gate/up
_MOE_GEMV_DN = tuple(int(v) for v in os.environ.get("NLS_MOE_GEMV_DN", "").split(",") if v)
# MoE expert GEMMs on the experts' f16 copies: (mode, waves, rt[, ks]) of gate/up and down
_MOE_DENSE_GU = tuple(int(v) for v in os.environ.get("NLS_MOE_DENSE_GU", "5,8,2").split(","))
_MOE_DENSE_DN = tuple(int(v) for v in os.environ.get("NLS_MOE_DENSE_DN", "5,8,2,4").split(","))
# expert parallelism: eager steps of >= NLS_EP_A2A_T tokens that the IPC row exchange does not cover dispatch /
# combine over all-to-all (LlamaModel._moe_a2a); NLS_EP_A2A=0 keeps the combine-then-all-reduce everywhere
_EP_A2A = os.environ.get("NLS_EP_A2A", "1")
_EP_A2A_T = int(os.environ.get("NLS_EP_A2A_T", "64"))
# tokens per step the EP row exchange covers (receive buffers: 2 x tokens x top-k x d_model floats per rank; 2048 =
# the engine's default prefill chunk: 134 MB per rank for Mixtral), decode AND prefill: no host-side split sizes, no
# RCCL call. NLS_EP_PREFILL=a2a sends eager steps of >= NLS_EP_A2A_T tokens to the all-to-all instead.
_EPX_TOKENS = int(os.environ.get("NLS_EPX_TOKENS", "2048"))
_EP_PREFILL = os.environ.get("NLS_EP_PREFILL", "exchange")
# MoE router logits through ops.router_logits (E-row kernel) rather than the GEMV/GEMM tiles; 0 = the GEMV
_ROUTER_KERNEL = os.environ.get("NLS_ROUTER_KERNEL", "1") == "1"


# device buffers superseded by larger ones; captured hipGraphs may still point at them
_RETIRED: List[torch.Tensor] = []


@dataclass
class ShardSpec:
    """Model shard of this process (rank of size); size 1 = whole model.

    Attention and dense FFNs are tensor-parallel (QKV / gate|up column-split, O / down
    row-split, lm_head vocab-split). MoE experts are TP-sharded along their FFN dim by
    default; with `ep=True` each rank instead owns E/size whole experts (expert parallel)."""
    rank: int = 0
    size: int = 1
    ep: bool = False


def _raw_rows(raw: np.ndarray, ggml_type: int, rows: int, K: int, r0: int, r1: int) -> np.ndarray:
    rb = ops.row_bytes(ggml_type, K)
    return np.asarray(raw).view(np.uint8).reshape(rows, rb)[r0:r1].reshape(-1)


def neox_pair_perm(n_heads: int, D: int) -> np.ndarray:
    """Row order that turns NEOX RoPE pairs (i, i + D/2) of every head into adjacent pairs (2i, 2i + 1): new row
    2i <- i, 2i + 1 <- i + D/2. Applied to the Q and K projection rows (and biases) at load, it leaves every q.k dot
    product unchanged (the same permutation on both sides) and lets Qwen2's RoPE run in the Q|K|V GEMV epilogue, which
    rotates adjacent pairs with pair i's frequency -- the frequency NEOX gives pair (i, i + D/2)."""
    h = np.stack([np.arange(D // 2), np.arange(D // 2) + D // 2], 1).reshape(-1)
    return (np.arange(n_heads)[:, None] * D + h[None, :]).reshape(-1)


def _raw_perm_rows(raw: np.ndarray, ggml_type: int, rows: int, K: int, perm: np.ndarray) -> np.ndarray:
    rb = ops.row_bytes(ggml_type, K)
    return np.ascontiguousarray(np.asarray(raw).view(np.uint8).reshape(rows, rb)[perm]).reshape(-1)


def _raw_cols(raw: np.ndarray, ggml_type: int, rows: int, K: int, k0: int, k1: int) -> np.ndarray:
    blk, nbytes = GGML_BLOCK[GGMLType(ggml_type)]
    if k0 % 256 or k1 % 256:
        raise ValueError("column shards must be multiples of 256")
    b = np.asarray(raw).view(np.uint8).reshape(rows, K // blk, nbytes)
    return np.ascontiguousarray(b[:, k0 // blk:k1 // blk]).reshape(-1)


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    ffn_norm: torch.Tensor
    qkv: List[Seg]
    wo: QWeight
    gateup: Optional[QWeight] = None
    down: Optional[QWeight] = None
    qkv_bias: Optional[torch.Tensor] = None     # Qwen2: f32 [(Hq + 2*Hkv) * D] (this shard)
    # MoE
    router: Optional[QWeight] = None
    router16: Optional[torch.Tensor] = None     # f16 [E, d] row-major copy for the fused norm + route kernel
    exp_gateup: List[QWeight] = field(default_factory=list)
    exp_down: List[QWeight] = field(default_factory=list)


@dataclass
class StepBuffers:
    """Device buffers for one forward of up to `cap` tokens (static for hipGraph capture)."""
    cap: int
    ids: torch.Tensor
    pos: torch.Tensor
    slot: torch.Tensor
    tok_seq: torch.Tensor
    ctx_len: torch.Tensor
    block_tables: torch.Tensor
    use_prev: torch.Tensor
    x: torch.Tensor
    h: torch.Tensor
    qkv: torch.Tensor
    q: torch.Tensor
    ao: torch.Tensor
    act: torch.Tensor
    logits: torch.Tensor
    keys: torch.Tensor
    next_ids: torch.Tensor
    attn_ws: torch.Tensor
    moe: Dict[str, torch.Tensor] = field(default_factory=dict)
    meta: Optional[torch.Tensor] = None
    pad: int = 0
    attn_cnt: Optional[torch.Tensor] = None    # int32 [pad*Hkv] split-merge tickets (zero between launches)
    part: Optional[torch.Tensor] = None        # f32 [pad, d] row-parallel partial sums (TP fused all-reduce)
    cnt: Optional[torch.Tensor] = None         # int32 tickets of the last-workgroup residual+RMSNorm GEMVs
    ssq: Optional[torch.Tensor] = None         # f32 [pad, ldss] split-RMSNorm partial sums of squares
    ldss: int = 0


class LlamaModel:
    def __init__(self, reader: GGUFReader, device="cpu", shard: ShardSpec = ShardSpec(), comm=None,
                 fuse_norm: Optional[bool] = None):
        self.reader = reader
        # RMSNorm folded into the consuming GEMVs for few-row decode steps, split between the O / down
        # GEMVs (per-workgroup shares of sum(x^2)) and the consumers (no norm launch, no reduction pass).
        # Round 2 measured it neutral at batch 1 (profiles/b1_split_rmsnorm_ab.txt): the consumers read the
        # shares and the residual row in loop-carried L2 round trips issued after their weight prologue.
        # With the one-row staging issued ahead of the weights (qgemv_impl.h xpre / xput) batch 1 gains
        # (2.11 -> 2.05 ms/token, profiles/b1_latency_r03.txt) while batch 4 still loses, so the default
        # ("auto") folds the norms at batch 1 only; NLS_FUSE_NORM=1 / 0 forces it on / off.
        env = os.environ.get("NLS_FUSE_NORM", "auto")
        self.fuse_norm = (env if env == "auto" else bool(int(env))) if fuse_norm is None else fuse_norm
        self.device = torch.device(device)
        self.cfg = cfg = ModelConfig.from_gguf(reader.metadata, reader.tensors.keys())
        self.shard = shard
        self.comm = comm
        n = shard.size
        if cfg.n_head % n or cfg.n_kv_head % n:
            raise ValueError(f"TP={n} must divide head counts ({cfg.n_head}/{cfg.n_kv_head})")
        self.Hq = cfg.n_head // n
        self.Hkv = cfg.n_kv_head // n
        self.D = cfg.head_dim
        self.ffn = cfg.d_ff // n
        self.ep = bool(shard.ep and cfg.n_expert and n > 1)
        if self.ep and cfg.n_expert % n:
            raise ValueError(f"EP={n} must divide the expert count ({cfg.n_expert})")
        self.exp_ffn = cfg.d_ff if self.ep else self.ffn
        per = cfg.n_expert // n if self.ep else cfg.n_expert
        self.experts = list(range(shard.rank * per, (shard.rank + 1) * per)) if self.ep else list(range(cfg.n_expert))
        if (self.Hq * self.D) % 256 or self.exp_ffn % 256 or (not cfg.n_expert and self.ffn % 256):
            raise ValueError("TP shard widths must be multiples of 256 (K-quant super-blocks)")
        self.vocab_lo, self.vocab_hi = self._vocab_range()
        self.weight_bytes = 0
        self._load()
        # expert parallelism on GPUs: decode-size MoE steps exchange the experts' output rows over the IPC buffers
        # (parallel/oneshot.py ep_exchange) instead of all-reducing [T, d] partial combines (NLS_EP_EXCHANGE=0: off)
        self.ep_exchange = False
        os_ = getattr(comm, "oneshot", None) if comm is not None else None
        if (self.ep and os_ is not None and self.device.type == "cuda"
                and os.environ.get("NLS_EP_EXCHANGE", "1") == "1"):
            os_.ep_setup(_EPX_TOKENS * cfg.n_expert_used, cfg.d_model)
            self.ep_exchange = True
        ff = reader.dequantized("rope_freqs.weight") if "rope_freqs.weight" in reader.tensors else None
        self.cs = ops.rope_table(cfg.ctx, self.D, cfg.rope_base, self.device, ff, cfg.rope_pos_scale)

    # ------------------------------------------------------------------ loading
    def _vocab_range(self):
        n, r, V = self.shard.size, self.shard.rank, self.cfg.vocab
        per = (V + n - 1) // n
        per = (per + 15) // 16 * 16
        self.vocab_per = per
        return min(V, r * per), min(V, (r + 1) * per)

    def _t(self, name):
        return self.reader.tensor(name)

    def _qw(self, raw, gt, rows, K, name, layout="tiled") -> QWeight:
        w = QWeight(raw, gt, rows, K, self.device, name, layout)
        self.weight_bytes += w.nbytes
        return w

    def _matrix(self, name, rows_sl=None, cols_sl=None, expert=None, layout="tiled", perm=None) -> QWeight:
        ti = self._t(name)
        shape = ti.np_shape
        raw = ti.data
        if expert is not None:
            E = shape[0]
            per = ti.nbytes // E
            raw = np.asarray(raw)[expert * per:(expert + 1) * per]
            shape = shape[1:]
        rows, K = shape
        if rows_sl is not None:
            raw = _raw_rows(raw, ti.ggml_type, rows, K, *rows_sl)
            rows = rows_sl[1] - rows_sl[0]
        if cols_sl is not None:
            raw = _raw_cols(raw, ti.ggml_type, rows, K, *cols_sl)
            K = cols_sl[1] - cols_sl[0]
        if perm is not None:
            raw = _raw_perm_rows(raw, ti.ggml_type, rows, K, perm)
        return self._qw(raw, ti.ggml_type, rows, K, name, layout)

    def _vec(self, name) -> torch.Tensor:
        return torch.from_numpy(self.reader.dequantized(name).astype(np.float32).copy()).to(self.device)

    def _gateup(self, gname, uname, expert=None, ffn=None) -> QWeight:
        cfg, r = self.cfg, self.shard.rank
        ffn = ffn or self.ffn
        sl = (0, ffn) if ffn == cfg.d_ff else (r * ffn, (r + 1) * ffn)
        gt, ut = self._t(gname).ggml_type, self._t(uname).ggml_type
        if gt != ut:
            raise NotImplementedError("gate/up with different quant types")
        raw = ops.interleave_gate_up(self._raw_of(gname, sl, expert), self._raw_of(uname, sl, expert), gt,
                                     ffn, cfg.d_model)
        return self._qw(raw, gt, 2 * ffn, cfg.d_model, gname + "|up")

    def _raw_of(self, name, rows_sl, expert=None):
        ti = self._t(name)
        shape = ti.np_shape
        raw = ti.data
        if expert is not None:
            per = ti.nbytes // shape[0]
            raw = np.asarray(raw)[expert * per:(expert + 1) * per]
            shape = shape[1:]
        return _raw_rows(raw, ti.ggml_type, shape[0], shape[1], *rows_sl)

    def _load(self):
        cfg, r = self.cfg, self.shard.rank
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        self.tok_embd = self._matrix("token_embd.weight", layout="rows")      # gathered, not streamed
        self.layers: List[LayerWeights] = []
        # NEOX RoPE (Qwen2): Q / K rows reordered so the pairs are adjacent (neox_pair_perm); the kernels then rotate
        # adjacent pairs, fused into the Q|K|V GEMV / GEMM epilogue like Llama's (NLS_NEOX_PERMUTE=0: the separate
        # NEOX RoPE launch, original row order)
        permute = cfg.rope_neox and os.environ.get("NLS_NEOX_PERMUTE", "1") == "1"
        self.rope_neox = cfg.rope_neox and not permute
        pq = neox_pair_perm(Hq, D) if permute else None
        pk = neox_pair_perm(Hkv, D) if permute else None
        for i in range(cfg.n_layer):
            p = f"blk.{i}."
            wq = self._matrix(p + "attn_q.weight", (r * Hq * D, (r + 1) * Hq * D), perm=pq)
            wk = self._matrix(p + "attn_k.weight", (r * Hkv * D, (r + 1) * Hkv * D), perm=pk)
            wv = self._matrix(p + "attn_v.weight", (r * Hkv * D, (r + 1) * Hkv * D))
            if ops.kernel_set([wq.type, wk.type, wv.type]) is None:   # e.g. Q2_K (-> F16) with a Q3_K V
                wq, wk, wv = wq.to_f16(), wk.to_f16(), wv.to_f16()
            qkv = [Seg(wq, 0), Seg(wk, Hq * D), Seg(wv, (Hq + Hkv) * D)]
            wo = self._matrix(p + "attn_output.weight", None, (r * Hq * D, (r + 1) * Hq * D))
            lw = LayerWeights(self._vec(p + "attn_norm.weight"), self._vec(p + "ffn_norm.weight"), qkv, wo)
            if p + "attn_q.bias" in self.reader.tensors:
                bq = self.reader.dequantized(p + "attn_q.bias").reshape(-1)[r * Hq * D:(r + 1) * Hq * D]
                bk = self.reader.dequantized(p + "attn_k.bias").reshape(-1)[r * Hkv * D:(r + 1) * Hkv * D]
                bv = self.reader.dequantized(p + "attn_v.bias").reshape(-1)[r * Hkv * D:(r + 1) * Hkv * D]
                if permute:
                    bq, bk = bq[pq], bk[pk]
                lw.qkv_bias = torch.from_numpy(np.concatenate([bq, bk, bv]).astype(np.float32)).to(self.device)
            if cfg.n_expert:
                lw.router = self._matrix(p + "ffn_gate_inp.weight")
                if self.device.type == "cuda" and cfg.n_expert in (2, 4, 8):
                    lw.router16 = lw.router.dense(torch.float16).contiguous()
                F = self.exp_ffn
                ksl = None if self.ep else (r * F, (r + 1) * F)
                for e in self.experts:          # local experts (all of them unless EP)
                    lw.exp_gateup.append(self._gateup(p + "ffn_gate_exps.weight", p + "ffn_up_exps.weight", e, F))
                    lw.exp_down.append(self._matrix(p + "ffn_down_exps.weight", None, ksl, expert=e))
            else:
                lw.gateup = self._gateup(p + "ffn_gate.weight", p + "ffn_up.weight")
                lw.down = self._matrix(p + "ffn_down.weight", None, (r * self.ffn, (r + 1) * self.ffn))
            self.layers.append(lw)
        self.out_norm = self._vec("output_norm.weight")
        head = "token_embd.weight" if cfg.tied_embeddings else "output.weight"
        self.lm_head = self._matrix(head, (self.vocab_lo, self.vocab_hi))

    def dense_matrices(self, experts: bool = False) -> List[QWeight]:
        """The projection matrices that get an f16 copy for the large-M dense GEMM (modes 4/5):
        attention, dense FFN and the LM head; experts=True: the local MoE experts (their grouped GEMM
        gathers rows through the same maps on the f16 copies)."""
        out = []
        for lw in self.layers:
            if experts:
                out += list(lw.exp_gateup) + list(lw.exp_down)
                continue
            out += [s.w for s in lw.qkv] + [lw.wo]
            if lw.gateup is not None:
                out += [lw.gateup, lw.down]
        if not experts:
            out.append(self.lm_head)
        return out

    def dense_decode_fraction(self, M: int) -> float:
        """Share of a decode step's dense-capable weight bytes whose launch at M rows would take the f16 copies
        (ops.tuning.select_dense: tuned "d:" entries, -1 = the quantised GEMM measured faster). 0 below
        ops.DENSE_MIN_M. Llama-3-70B at M = 128: 0 (every shape -1), so its 139 GB of copies would serve prompt
        chunks only; Llama-3-8B at 512: 1."""
        if M < ops.DENSE_MIN_M or not self.layers:
            return 0.0
        lw = self.layers[0]
        groups = [list(lw.qkv), [Seg(lw.wo)]]
        if lw.gateup is not None:
            groups += [[Seg(lw.gateup)], [Seg(lw.down)]]
        groups.append([Seg(self.lm_head)])
        tot = used = 0
        for segs in groups:
            b = sum(s.w.dense_bytes for s in segs)
            tot += b
            if tuning.select_dense(segs, M) is not None:
                used += b
        return used / tot if tot else 0.0

    def expand_dense(self, budget_bytes: Optional[int] = None, experts: bool = False) -> int:
        """Give the dense_matrices() their f16 copies (ops.QWeight.expand_dense) in all-or-nothing
        tiers -- attention/dense FFN/LM head, then (experts=True) the MoE experts -- each only when it
        fits in what is left of `budget_bytes` (None: no limit), so every large-M launch of one kind
        takes one path. Returns the bytes added (0 if skipped or already expanded)."""
        if self.device.type != "cuda":
            return 0
        added = 0
        for tier in ((False, True) if experts else (False,)):
            ws = self.dense_matrices(experts=tier)
            need = sum(w.dense_bytes for w in ws if w.d16 is None)
            if need == 0:
                continue
            if budget_bytes is not None and need > budget_bytes - added:
                break
            if not tier:   # each layer's Q|K|V copies as one buffer: one dense segment per launch
                added += sum(QWeight.expand_dense_group([s.w for s in lw.qkv]) for lw in self.layers)
            added += sum(w.expand_dense() for w in ws)
        self.dense_bytes = getattr(self, "dense_bytes", 0) + added
        return added

    # ------------------------------------------------------------------ buffers
    @property
    def kv_dtype(self) -> torch.dtype:
        """Paged KV cache element type: NLS_KV_DTYPE=bf16 (default) | fp8 (OCP e4m3, half the bytes)."""
        name = os.environ.get("NLS_KV_DTYPE", "bf16")
        if name not in ops.KV_DTYPES:
            raise ValueError(f"NLS_KV_DTYPE={name}: one of {sorted(ops.KV_DTYPES)}")
        return ops.KV_DTYPES[name]

    def kv_cache(self, num_blocks: int, block_size: int = 16):
        L, slots = self.cfg.n_layer, num_blocks * block_size
        k = torch.zeros(L, slots, self.Hkv, self.D, dtype=self.kv_dtype, device=self.device)
        v = torch.zeros_like(k)
        return k, v

    def step_buffers(self, cap: int, max_seqs: int, max_blocks: int) -> StepBuffers:
        """All int32 step metadata lives in ONE tensor (`meta`) so the engine refreshes it
        with a single host->device copy per step: [ids|pos|slot|tok_seq|ctx_len|use_prev|block_tables].
        use_prev[i] != 0: row i's input token is next_ids[i] of the previous step (chained decode)."""
        cfg, dev = self.cfg, self.device
        pad = (cap + 63) // 64 * 64
        Vs = self.vocab_hi - self.vocab_lo
        nq = self.Hq * self.D
        k = max(1, cfg.n_expert_used)
        meta = torch.zeros(6 * pad + max_seqs * max_blocks, dtype=torch.int32, device=dev)
        f = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=torch.bfloat16, device=dev)     # q (attention operand, like the KV cache)
        act = dict(dtype=ops.ACT_DTYPE, device=dev)     # GEMM inputs: h, attention output, SwiGLU output
        b = StepBuffers(
            cap=cap,
            ids=meta[0:pad], pos=meta[pad:2 * pad], slot=meta[2 * pad:3 * pad],
            tok_seq=meta[3 * pad:4 * pad], ctx_len=meta[4 * pad:5 * pad], use_prev=meta[5 * pad:6 * pad],
            block_tables=meta[6 * pad:].view(max_seqs, max_blocks),
            x=torch.zeros(pad, cfg.d_model, **f),
            h=torch.zeros(pad, cfg.d_model, **act),
            qkv=torch.zeros(pad, (self.Hq + 2 * self.Hkv) * self.D, **f),
            q=torch.zeros(pad, nq, **bf),
            ao=torch.zeros(pad, nq, **act),
            act=torch.zeros(pad * (k if cfg.n_expert else 1), self.exp_ffn if cfg.n_expert else self.ffn, **act),
            logits=torch.zeros(min(pad, max(64, max_seqs)), Vs, **f),
            keys=torch.zeros(pad, dtype=torch.int64, device=dev),
            next_ids=torch.zeros(pad, dtype=torch.int32, device=dev),
            # flash-decoding partials for the split policy's largest T * n_split (attn_splits keeps
            # T * Hkv * n_split <= _SPLIT_WG): allocated once, because captured decode graphs hold it
            attn_ws=torch.zeros(max(1, (_SPLIT_WG // self.Hkv + 1) * self.Hq * (self.D + 2)), **f),
        )
        b.meta = meta
        b.pad = pad
        # keys hold the reset value (argmax_unpack(rearm=True) leaves them so): the next step skips the reset.
        # Device keys start zeroed; a CPU buffer starts at zero too, which is not its reset value.
        b.keys_clean = dev.type == "cuda"
        b.attn_cnt = torch.zeros(pad * self.Hkv, dtype=torch.int32, device=dev)
        if self.shard.size > 1:
            b.part = torch.zeros(pad, cfg.d_model, dtype=torch.float32, device=dev)
        b.cnt = torch.zeros(16, dtype=torch.int32, device=dev)
        b.ldss = (cfg.d_model + 15) // 16       # one share per 16-row path-A tile of an O / down GEMV
        b.ssq = torch.zeros(pad * b.ldss, dtype=torch.float32, device=dev)
        b.slot.fill_(-1)
        if cfg.n_expert:
            E = cfg.n_expert
            b.moe = dict(
                rlogits=torch.zeros(pad, E, dtype=torch.float32, device=dev),
                topw=torch.zeros(pad * k, dtype=torch.float32, device=dev),
                counts=torch.zeros(E, dtype=torch.int32, device=dev),
                xrows=torch.zeros(E * pad, dtype=torch.int32, device=dev),
                yrows=torch.zeros(E * pad, dtype=torch.int32, device=dev),
                sel=torch.zeros(pad * k, dtype=torch.int32, device=dev),
                yexp=torch.zeros(pad * k, cfg.d_model, dtype=torch.float32, device=dev),
            )
        return b

    @staticmethod
    def attn_splits(T: int, Hkv: int) -> int:
        """Flash-decoding splits per (token, kv head): enough workgroups to cover the chip. The kernel
        sizes each split from the actual context (>= 64 keys) and skips splits past it, so a large
        split count only costs parallelism headroom for long contexts."""
        wg = T * Hkv
        if wg >= _SPLIT_WG:
            return 1
        return int(min(_SPLIT_CAP, max(1, _SPLIT_WG // wg)))

    # ------------------------------------------------------------------ forward
    def forward(self, b: StepBuffers, kc: torch.Tensor, vc: torch.Tensor, T: int, block_size: int,
                n_split: int = 1, logit_rows: Optional[torch.Tensor] = None, n_logits: Optional[int] = None,
                qblocks: Optional[torch.Tensor] = None, nqb: int = 0, feed_prev: bool = False,
                need_logits: bool = True):
        """Runs T tokens through the model; leaves greedy ids in b.next_ids[:n] and logits in b.logits[:n].
        With `qblocks` (prompt chunks, ops.prefill_blocks) attention runs the MFMA flash-prefill kernel."""
        cfg = self.cfg
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        x = b.x
        # chained decode: the previous step's tokens are picked on the device inside the embedding launch
        ops.embed(b.ids, self.tok_embd, x, T, cfg.embedding_scale, prev=(b.next_ids, b.use_prev) if feed_prev else None)
        need = T * Hq * n_split * (D + 2)
        if n_split > 1 and b.attn_ws.numel() < need:
            # a larger explicit split than the policy's: grow, but keep the old buffer alive -- a graph
            # captured earlier still writes its partials there (freeing it let a later allocation, e.g.
            # prefill metadata, land under a replaying graph: the 256 x 1K-context fault of this round)
            _RETIRED.append(b.attn_ws)
            b.attn_ws = torch.zeros(need, dtype=torch.float32, device=self.device)
        fused = self.shard.size == 1            # row-parallel GEMM + residual + next RMSNorm in one pass
        # few-row decode steps: every RMSNorm is folded into the GEMV that consumes it (no norm launches)
        fuse = (T == 1 and x.is_cuda) if self.fuse_norm == "auto" else self.fuse_norm
        fnorm = (fuse and fused and not cfg.n_expert and qblocks is None
                 and ops.norm_fusable(T, cfg.d_model))
        if fnorm:
            return self._forward_fused_norm(b, kc, vc, T, block_size, n_split, logit_rows, n_logits, need_logits)
        fused_prev = True                       # layer 0's input norm is applied just below
        ops.rmsnorm(x, self.layers[0].attn_norm, b.h, T, cfg.eps)
        for L, lw in enumerate(self.layers):
            if L > 0 and not fused_prev:
                ops.rmsnorm(x, lw.attn_norm, b.h, T, cfg.eps)
            ops.qkv_rope_kv(lw.qkv, b.h, b.qkv, b.pos, b.slot, self.cs, b.q, kc[L], vc[L], T, Hq, Hkv, D,
                            self.rope_neox, bias=lw.qkv_bias)
            if qblocks is not None and nqb > 0 and ops.attention_prefill_ok(Hq, Hkv, D):
                ops.attention_prefill(b.q, kc[L], vc[L], b.block_tables, qblocks, nqb, b.tok_seq, b.ctx_len, b.ao,
                                      T, Hq, Hkv, D, block_size, cfg.attn_softmax_scale)
            else:
                ops.attention(b.q, kc[L], vc[L], b.block_tables, b.tok_seq, b.ctx_len, b.ao, T, Hq, Hkv, D,
                              block_size, cfg.attn_softmax_scale, chunk=-_MIN_CHUNK, n_split=n_split, workspace=b.attn_ws,
                              counters=b.attn_cnt)
            moe_norm = fused and lw.router16 is not None and T <= _MOE_NORM_ROUTE_T
            moe_routed = False
            if moe_norm and _MOE_FOLD_ROUTE and x.is_cuda:
                # the o projection's last workgroup applies the FFN norm, the router and the route
                m = b.moe
                use_sel = T * cfg.n_expert_used < len(self.experts)
                moe_routed = ops.qgemv_add_norm_route(
                    Seg(lw.wo), b.ao, x, lw.ffn_norm, b.h, T, cfg.residual_scale, cfg.eps, b.cnt, lw.router16,
                    m["rlogits"], cfg.n_expert_used, m["topw"], m["counts"], m["xrows"], m["yrows"], x.shape[0],
                    sel=m["sel"] if use_sel else None)
            if moe_routed:
                pass
            elif moe_norm:
                # the FFN input norm runs inside the MoE router/route launch (ops.moe_norm_route)
                ops.qgemv([Seg(lw.wo)], b.ao, x, T, alpha=cfg.residual_scale, epi="add")
            elif fused:
                ops.qgemv_add_rmsnorm(Seg(lw.wo), b.ao, x, lw.ffn_norm, b.h, T, cfg.residual_scale, cfg.eps,
                                      counter=b.cnt)
            elif not self.comm.row_parallel_add_norm(lw.wo, b.ao, b.part, x, lw.ffn_norm, b.h, T,
                                                     cfg.residual_scale, cfg.eps):
                self._row_parallel(lw.wo, b.ao, x, T, cfg.residual_scale)
                ops.rmsnorm(x, lw.ffn_norm, b.h, T, cfg.eps)
            nxt = self.layers[L + 1].attn_norm if L + 1 < len(self.layers) else self.out_norm
            fused_prev = False
            if cfg.n_expert:
                fused_prev = self._moe(lw, b, T, nxt if (fused or self.ep_exchange) else None,
                                       lw.ffn_norm if moe_norm and not moe_routed else None, routed=moe_routed)
            else:
                ops.qgemv([Seg(lw.gateup)], b.h, b.act, T, epi="swiglu")
                if fused:
                    ops.qgemv_add_rmsnorm(Seg(lw.down), b.act, x, nxt, b.h, T, cfg.residual_scale, cfg.eps,
                                          counter=b.cnt)
                    fused_prev = True
                elif self.comm.row_parallel_add_norm(lw.down, b.act, b.part, x, nxt, b.h, T, cfg.residual_scale,
                                                     cfg.eps):
                    fused_prev = True
                else:
                    self._row_parallel(lw.down, b.act, x, T, cfg.residual_scale)
        if not fused_prev:
            ops.rmsnorm(x, self.out_norm, b.h, T, cfg.eps)
        h = b.h
        n = T
        if logit_rows is not None:
            n = int(n_logits)
            h = b.h.index_select(0, logit_rows[:n].long())
            h = torch.cat([h, h.new_zeros((-n) % 16, h.shape[1])]) if n % 16 else h
        if not b.keys_clean:
            ops.argmax_reset(b.keys)
        # greedy-only steps keep just the fused arg-max keys (no [n, V] logits written)
        ops.qgemv([Seg(self.lm_head, 0)], h, b.logits, n, alpha=1.0 / cfg.logit_scale, argmax=b.keys,
                  epi="f32" if need_logits else "argmax")
        # the unpack (or the vocab-parallel arg-max) re-arms the keys it read: the next step's arg-max needs no
        # reset launch (under TP it was the one PyTorch kernel left in the decode graphs)
        if self.shard.size == 1:
            ops.argmax_unpack(b.keys, n, b.next_ids, rearm=True)
        else:
            self.comm.vocab_parallel_argmax(b.keys, n, self.vocab_lo, b.next_ids)
        b.keys_clean = b.keys.is_cuda
        return n

    def _forward_fused_norm(self, b: StepBuffers, kc, vc, T: int, block_size: int, n_split: int, logit_rows,
                            n_logits, need_logits: bool):
        """Decode of a few rows with no RMSNorm launches: QKV, gate|up and the lm_head GEMVs normalise
        their input rows themselves (ops.qgemv(norm=...)); O / down add into the f32 residual."""
        cfg = self.cfg
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        x = b.x
        # split RMSNorm: each O / down launch leaves per-workgroup shares of sum(x^2) in b.ssq and the
        # consuming GEMV sums them instead of re-reading the whole row (ops.qgemv_add_ssq)
        ssq, ldss = b.ssq, b.ldss

        def nrm(w, parts):
            return (x, w, cfg.eps, ssq if parts else None, ldss, parts or 0)

        parts = None
        for L, lw in enumerate(self.layers):
            ops.qkv_rope_kv(lw.qkv, b.h, b.qkv, b.pos, b.slot, self.cs, b.q, kc[L], vc[L], T, Hq, Hkv, D,
                            self.rope_neox, bias=lw.qkv_bias, norm=nrm(lw.attn_norm, parts))
            ops.attention(b.q, kc[L], vc[L], b.block_tables, b.tok_seq, b.ctx_len, b.ao, T, Hq, Hkv, D,
                          block_size, cfg.attn_softmax_scale, chunk=-_MIN_CHUNK, n_split=n_split, workspace=b.attn_ws,
                          counters=b.attn_cnt)
            parts = ops.qgemv_add_ssq(Seg(lw.wo), b.ao, x, T, cfg.residual_scale, ssq, ldss)
            ops.qgemv([Seg(lw.gateup)], b.h, b.act, T, epi="swiglu", norm=nrm(lw.ffn_norm, parts))
            parts = ops.qgemv_add_ssq(Seg(lw.down), b.act, x, T, cfg.residual_scale, ssq, ldss)
        n = T
        if logit_rows is not None:             # (prefill-style row pick: normalise, then gather)
            ops.rmsnorm(x, self.out_norm, b.h, T, cfg.eps)
            n = int(n_logits)
            h = b.h.index_select(0, logit_rows[:n].long())
            h = torch.cat([h, h.new_zeros((-n) % 16, h.shape[1])]) if n % 16 else h
            if not b.keys_clean:
                ops.argmax_reset(b.keys)
            ops.qgemv([Seg(self.lm_head, 0)], h, b.logits, n, alpha=1.0 / cfg.logit_scale, argmax=b.keys,
                      epi="f32" if need_logits else "argmax")
        else:
            if not b.keys_clean:
                ops.argmax_reset(b.keys)
            ops.qgemv([Seg(self.lm_head, 0)], b.h, b.logits, n, alpha=1.0 / cfg.logit_scale, argmax=b.keys,
                      epi="f32" if need_logits else "argmax", norm=nrm(self.out_norm, parts))
        ops.argmax_unpack(b.keys, n, b.next_ids, rearm=True)
        b.keys_clean = b.keys.is_cuda
        return n

    def _row_parallel(self, w: QWeight, xin: torch.Tensor, resid: torch.Tensor, T: int, alpha: float):
        if self.shard.size == 1:
            ops.qgemv([Seg(w)], xin, resid, T, alpha=alpha, epi="add")
        else:
            self.comm.row_parallel_add(w, xin, resid, T, alpha)

    @staticmethod
    def _router(lw: LayerWeights, h: torch.Tensor, logits: torch.Tensor, T: int,
                counts: Optional[torch.Tensor] = None) -> bool:
        """Router logits of T tokens: the dedicated E-row kernel on the router's f16 copy (GPU), else the GEMV.
        True when the kernel also zeroed `counts` (the following moe_route can skip its memset)."""
        if lw.router16 is not None and _ROUTER_KERNEL:
            ops.router_logits(h, lw.router16, logits, T, zero=counts)
            return counts is not None
        ops.qgemv([Seg(lw.router)], h, logits, T)
        return False

    @staticmethod
    def _moe_gemm_cfg(lw: LayerWeights, rows: int, n_exp: int):
        """Launch configs (gate/up, down, down split-K) of the grouped expert GEMMs for `rows` routed rows
        over `n_exp` experts."""
        if all(w.d16 is not None for w in lw.exp_gateup + lw.exp_down):
            # f16 expert copies (expand_dense tier 2): the dense DMA GEMM, bandwidth- rather than
            # dequant-bound at ~64 rows per expert (NLS_MOE_DENSE_GU/_DN = mode,waves,rt)
            gu = dict(zip(("mode", "waves", "rt"), _MOE_DENSE_GU[:3]), ks=1)
            dn = dict(zip(("mode", "waves", "rt"), _MOE_DENSE_DN[:3]), ks=1)
            return gu, dn, (_MOE_DENSE_DN[3] if len(_MOE_DENSE_DN) > 3 else 1)
        # few routed rows per expert: 128-row blocks (64 KiB of LDS, two workgroups per CU hide each
        # other's dequant/barrier waits; Mixtral B=64: 13.8 vs 15.2 ms/step), else 256-row blocks
        rt = 2 if rows < 32 * n_exp else 4
        gu = dict(mode=2, waves=8, rt=int(os.environ.get("NLS_MOE_RT_GU", rt)), ks=1)
        dn = dict(mode=2, waves=8, rt=int(os.environ.get("NLS_MOE_RT_DN", rt)), ks=1)
        kdn = int(os.environ.get("NLS_MOE_KS_DN", "1"))
        kquant = all(int(w.type) in (12, 13, 14) for w in lw.exp_gateup + lw.exp_down)   # the DMA GEMM's types
        if kquant and 32 * n_exp <= rows <= 96 * n_exp and os.environ.get("NLS_MOE_DMA", "1") == "1":
            # ~32-96 routed rows per expert (Mixtral B=128-384): gate|up on the LDS-DMA GEMM over 96-row blocks at
            # two workgroups per CU, the DMA gathering each expert's rows (286 -> 260 us per launch in the model).
            # The down projection stays on mode 2 unsplit: in the model (Mixtral-8x7B B=256, one box) 16.45
            # ms/step vs 16.63 with mode 3 split 4 and 18.24 split 2 (profiles/moe_dma_r06.txt; the isolated
            # probe's 168 vs 285 us did not carry over -- the model's mode-2 down runs at ~144 us)
            gu = dict(mode=3, waves=4, rt=6, ks=1)
        if os.environ.get("NLS_MOE_QCFG_GU"):      # explicit (mode, waves, rt) overrides
            gu = dict(zip(("mode", "waves", "rt"), (int(v) for v in os.environ["NLS_MOE_QCFG_GU"].split(","))), ks=1)
        if os.environ.get("NLS_MOE_QCFG_DN"):
            dn = dict(zip(("mode", "waves", "rt"), (int(v) for v in os.environ["NLS_MOE_QCFG_DN"].split(","))), ks=1)
        return gu, dn, kdn

    def _ep_a2a(self, T: int) -> bool:
        """Take the all-to-all dispatch / combine (_moe_a2a) for this MoE step? Eager EP steps of
        >= NLS_EP_A2A_T tokens (prefill chunks, large eager batches) that the IPC row exchange does not cover
        (no exchange: CPU / no IPC, or more than NLS_EPX_TOKENS tokens); captured decode graphs never (the
        all-to-all needs its split sizes on the host)."""
        if not self.ep or _EP_A2A == "0" or T < _EP_A2A_T:
            return False
        if (self.ep_exchange and _EP_PREFILL != "a2a"
                and self.comm.oneshot.ep_ok(T * self.cfg.n_expert_used, self.cfg.d_model)):
            return False                     # the row exchange covers this step (_moe, exch)
        if self.device.type == "cuda":
            # grouped-GEMM path only (the path-A GEMVs take <= 64 rows) and never inside a capture
            return T > _MOE_GEMM_T and not torch.cuda.is_current_stream_capturing()
        return True

    def _moe_a2a(self, lw: LayerWeights, b: StepBuffers, T: int) -> bool:
        """Expert parallelism as dispatch / combine over all-to-all (BASELINE config 5, "expert all-to-all on
        xGMI"). Rank r routes its 1/W slice of the (replicated) tokens, sends each (token, slot) row to the rank
        owning that slot's expert (RCCL all-to-all: each pair of ranks exchanges only its own rows on its own
        xGMI link), runs its local experts as ONE grouped GEMM over the rows it received, sends the expert
        outputs back (all-to-all), combines its slice's k slots in slot order -- the single-GPU combine, so the
        result does not depend on the rank count -- and all-gathers the residual slices. Per rank and layer:
        (T/W) k d (2 + 4) bytes each way plus the f32 residual all-gather, against the 2 T d 4 (W-1)/W of the
        combine-then-all-reduce path (profiles/ep_alltoall_model_r04.md)."""
        cfg, m, comm = self.cfg, b.moe, self.comm
        k, d = cfg.n_expert_used, cfg.d_model
        W, r = self.shard.size, self.shard.rank
        per, e0 = len(self.experts), self.experts[0]
        cap = b.x.shape[0]
        ts = -(-T // W)                                   # tokens per rank slice
        t0 = min(T, r * ts)
        n = min(T, t0 + ts) - t0
        sel = m["sel"]
        if n:
            zeroed = self._router(lw, b.h[t0:], m["rlogits"], n, counts=m["counts"])
            ops.moe_route(m["rlogits"], n, k, m["topw"], m["counts"], m["xrows"], m["yrows"], cap, sel=sel,
                          counts_zeroed=zeroed)
        # dispatch: the slice's (token, slot) rows grouped by the rank owning the slot's expert
        eid = sel[:n * k].long()
        dest = torch.div(eid, per, rounding_mode="floor")
        order = torch.argsort(dest, stable=True)
        send = torch.bincount(dest, minlength=W).tolist()
        recv = comm.exchange_counts(send)
        nr = sum(recv)
        xr = comm.all_to_all_rows(b.h[t0:t0 + n].index_select(0, torch.div(order, k, rounding_mode="floor")),
                                  send, recv)
        er = comm.all_to_all_rows(eid.index_select(0, order).to(torch.int32), send, recv).long() - e0
        # local experts' row lists over the received rows (expert i: rows[i * cap:], counts[i]); the GEMMs
        # gather their inputs and place their outputs by the same received-row index
        o2 = torch.argsort(er, stable=True)
        cnt = torch.bincount(er, minlength=per)
        le = er.index_select(0, o2)
        pos = torch.arange(nr, device=er.device) - (torch.cumsum(cnt, 0) - cnt).index_select(0, le)
        rows, counts = m["xrows"], m["counts"]
        rows[le * cap + pos] = o2.to(torch.int32)
        counts[:per] = cnt.to(torch.int32)
        if nr:
            gu, dn, _ = self._moe_gemm_cfg(lw, nr, per) if self.device.type == "cuda" else ({}, {}, 1)
            M = min(nr, T)                                # an expert gets each token at most once
            segs = [Seg(w, 0, rows[i * cap:], rows[i * cap:], counts[i:i + 1]) for i, w in enumerate(lw.exp_gateup)]
            for s0 in range(0, per, 8):
                ops.qgemv(segs[s0:s0 + 8], xr, b.act, M, epi="swiglu", **gu)
            segs = [Seg(w, 0, rows[i * cap:], rows[i * cap:], counts[i:i + 1]) for i, w in enumerate(lw.exp_down)]
            for s0 in range(0, per, 8):
                ops.qgemv(segs[s0:s0 + 8], b.act, m["yexp"], M, epi="f32", **dn)
        # combine: the outputs return to the slice's rank in dispatch order -> slot order -> weighted sum
        yb = comm.all_to_all_rows(m["yexp"][:nr], recv, send)
        ys = torch.empty_like(yb)
        ys.index_copy_(0, order, yb)
        blk = b.x.new_zeros(ts, d)
        if n:
            ops.moe_combine(ys, m["topw"], n, k, b.x[t0:t0 + n], cfg.residual_scale)
            blk[:n] = b.x[t0:t0 + n]
        b.x[:T] = comm.all_gather_rows(blk)[:T]
        return False

    def _moe(self, lw: LayerWeights, b: StepBuffers, T: int, next_norm: Optional[torch.Tensor] = None,
             in_norm: Optional[torch.Tensor] = None, routed: bool = False) -> bool:
        """Top-k routed experts: router GEMV -> route kernel (per-expert row lists on device)
        -> grouped expert GEMVs (tiles of experts with no routed rows exit before reading
        weights) -> deterministic weighted combine into the residual. `in_norm` (<= 4 tokens): b.h is
        not normalised yet; the FFN input RMSNorm, the router and the route run as ONE launch."""
        if in_norm is None and not routed and self._ep_a2a(T):
            return self._moe_a2a(lw, b, T)
        cfg = self.cfg
        normed = False
        m = b.moe
        k, E = cfg.n_expert_used, cfg.n_expert
        cap = b.x.shape[0]
        # routed: the o projection already normalised b.h and routed the tokens (ops.qgemv_add_norm_route)
        if in_norm is not None and not routed:
            use_sel = self.device.type == "cuda" and T * k < len(self.experts)
            routed = ops.moe_norm_route(b.x, in_norm, cfg.eps, lw.router16, b.h, m["rlogits"], T, k, m["topw"],
                                        m["counts"], m["xrows"], m["yrows"], cap, sel=m["sel"] if use_sel else None)
            if not routed:
                ops.rmsnorm(b.x, in_norm, b.h, T, cfg.eps)
        zeroed = False
        if not routed:
            zeroed = self._router(lw, b.h, m["rlogits"], T, counts=m["counts"])
        # few tokens: path-A GEMV over each expert's gathered rows; many tokens: ONE route and the
        # LDS-dequant GEMM (mode 2) over all experts, each m-block of an expert gathering its rows
        # through xrows and exiting when it lies past the expert's device-side count
        gemm = T > _MOE_GEMM_T and self.device.type == "cuda"
        # path-A chunks of <= 32 tokens: the mapped GEMV then runs with <= 2 activation tiles, whose
        # kernels keep every fragment in registers (3-4 tiles spill: -Rpass-analysis scratch > 0)
        step = T if gemm else 32
        # m-block = 64*rt rows. Every m-block re-dequantises the expert's weights, so the largest block
        # wins; the GEMM multiplies only the block's real 16-row tiles (qgemm_impl.h NA), so ~64 routed
        # rows in a 256-row block cost 64 rows of MFMA (Mixtral B=256, round-2 sweep: gate/up
        # rt 4 / down rt 4 = 19.6 ms/step, 4/2 = 20.7, 2/2 = 28.3, 1/1 = 43.0)
        gu = dn = {}
        if not gemm and len(_MOE_GEMV_DN) == 4:
            dn = dict(zip(("mode", "waves", "rt", "ks"), _MOE_GEMV_DN))
        dn_rows = T
        if gemm:
            gu, dn, kdn = self._moe_gemm_cfg(lw, T * k, E)
            # down projection (K = d_ff): split K over workgroups when ONE launch covers every routed row
            # (<= 8 local experts, no EP: every y row written by exactly one expert in every K slice);
            # the slabs are indexed by the y row, so that launch's M is the T*k output rows
            # (Mixtral-8x7B before the NA tiles: B=256 28.5 vs 30.9 ms/step at 4 slices; with them the
            # unsplit rt-4 launch is faster, 19.6 vs 20.6: off by default, profiles/moe_down_splitk.txt)
            if kdn > 1 and len(self.experts) <= 8 and not self.ep and T * k >= 48 * len(self.experts):
                dn["ks"] = kdn
                dn_rows = T * k
            elif dn.get("mode") == 3:
                dn = dict(mode=2, waves=8, rt=4, ks=1)      # unsplit, the LDS-dequant GEMM is ahead (285 vs 300 us)
        for c0 in range(0, T, step):
            n = min(step, T - c0)
            # few tokens: the route kernel also lists each (token, slot)'s expert and the expert GEMVs
            # launch only those experts' tiles (k of E; the rest would be launched just to exit)
            use_sel = not gemm and self.device.type == "cuda" and n * k < len(self.experts)
            # the EP exchange needs every (token, slot)'s expert: its owner rank pushes the row
            exch = self.ep_exchange and self.comm.oneshot.ep_ok(n * k, cfg.d_model)
            if not (routed and c0 == 0 and n == T):
                ops.moe_route(m["rlogits"][c0:], n, k, m["topw"], m["counts"], m["xrows"], m["yrows"], cap,
                              sel=m["sel"] if (use_sel or exch) else None, counts_zeroed=zeroed and c0 == 0)
            loc = list(zip(self.experts, lw.exp_gateup, lw.exp_down))
            segs = [Seg(gu, 0, m["xrows"][e * cap:], m["yrows"][e * cap:], m["counts"][e:e + 1]) for e, gu, _ in loc]

            def sel(s0):
                return (m["sel"], n * k, self.experts[0] + s0) if use_sel else None
            for s0 in range(0, len(segs), 8):
                ops.qgemv(segs[s0:s0 + 8], b.h[c0:], b.act, n, epi="swiglu", sel=sel(s0), **gu)
            if self.ep and not exch:           # rows routed to other ranks' experts stay zero
                m["yexp"][:n * k].zero_()
            segs = [Seg(dn, 0, m["yrows"][e * cap:], m["yrows"][e * cap:], m["counts"][e:e + 1]) for e, _, dn in loc]
            for s0 in range(0, len(segs), 8):
                ops.qgemv(segs[s0:s0 + 8], b.act, m["yexp"], dn_rows if dn.get("ks", 1) > 1 else n, epi="f32",
                          sel=sel(s0), **dn)
            xs = b.x[c0:c0 + n]
            if exch:
                # every rank ends with all n * k expert rows (its own pushed, the peers' received): the single-GPU
                # combine, identical on every rank, no all-reduce
                self.comm.oneshot.ep_exchange(m["yexp"], n * k, m["sel"], len(self.experts))
                self.comm.stats["ep_exchange"] = self.comm.stats.get("ep_exchange", 0) + 1
                if next_norm is not None and n == T:
                    ops.moe_combine_norm(m["yexp"], m["topw"], n, k, xs, cfg.residual_scale, next_norm, cfg.eps, b.h)
                    normed = True
                else:
                    ops.moe_combine(m["yexp"], m["topw"], n, k, xs, cfg.residual_scale)
            elif self.shard.size > 1:
                # combine locally first, then ONE all-reduce of the combined [n, d] rows (k x fewer bytes
                # than reducing the per-slot expert outputs): rank 0 adds into the residual, the others
                # contribute their partial combine from zero (EP: own experts; TP: own FFN slice)
                ops.moe_combine(m["yexp"], m["topw"], n, k, xs, cfg.residual_scale, set_=self.shard.rank != 0)
                self.comm.all_reduce(xs)
            elif next_norm is not None and n == T:
                # one chunk: the combine and the next layer's input RMSNorm share a launch
                ops.moe_combine_norm(m["yexp"], m["topw"], n, k, xs, cfg.residual_scale, next_norm, cfg.eps, b.h)
                normed = True
            else:
                ops.moe_combine(m["yexp"], m["topw"], n, k, xs, cfg.residual_scale)
        return normed
