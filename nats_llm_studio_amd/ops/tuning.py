"""Launch-configuration selection for the quantised GEMV/GEMM kernels.

Measured per-shape winners (tools/tune_gemv.py on MI355X) live in `gemv_tuning.json`
next to this file: {"<type>:<rows>:<K>:<Mbucket>": [mode, waves, rt, ks]}. Shapes not in
the table use the heuristic below.
"""
from __future__ import annotations

import json
import os

_TABLE = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemv_tuning.json")
MBUCKETS = (1, 2, 4, 8, 16, 32, 48, 64, 128, 256, 512, 1024, 2048)


def _mb(M: int) -> int:
    for b in MBUCKETS:
        if M <= b:
            return b
    return MBUCKETS[-1]


def key(segs, M: int) -> str:
    t = "+".join(str(s.w.type) for s in segs)
    rows = sum(s.w.rows for s in segs)
    return f"{t}:{rows}:{segs[0].w.K}:{_mb(M)}"


def table():
    global _TABLE
    if _TABLE is None:
        _TABLE = {}
        if os.path.exists(_PATH):
            with open(_PATH) as f:
                _TABLE = {k: tuple(v) for k, v in json.load(f).items()}
        # A/B overrides without editing the table: NLS_TUNING_EXTRA='{"<key>": [..], ...}'
        # ... or from a file (NLS_TUNING_EXTRA_FILE, e.g. a fresh tune_gemv.py --out table), applied first
        path = os.environ.get("NLS_TUNING_EXTRA_FILE")
        if path:
            with open(path) as f:
                _TABLE.update({k: tuple(v) for k, v in json.load(f).items()})
        extra = os.environ.get("NLS_TUNING_EXTRA")
        if extra:
            _TABLE.update({k: tuple(v) for k, v in json.loads(extra).items()})
    return _TABLE


def heuristic(segs, M: int):
    rows = sum(s.w.rows for s in segs)
    K = segs[0].w.K
    if M <= 8:
        # the batch-1 winners of every measured family (Llama-3-8B / -70B, Qwen2.5-7B, Mixtral; r03 sweeps,
        # profiles/b1_latency_r03.txt, profiles/b1_models_r03.txt): 4-wave workgroups; wide matrices (gate|up,
        # LM head) on path B's staged-x stream, fused Q|K|V on 32-row path-A tiles, the rest on 16-row ones.
        # The old (0, 8, 1, 1) default cost Llama-3-70B / Qwen2.5-7B ~30 % at batch 1.
        if rows >= 4 * K:
            return (1, 4, 2, 2) if rows >= 16 * K and K >= 1024 else (1, 4, 2, 1)
        return (0, 4, 2, 1) if len(segs) > 1 else (0, 4, 1, 1)
    if M > 64:
        if all(int(s.w.type) in (12, 13, 14) for s in segs):
            if M >= 256 and (rows >= 4 * K or K >= 2 * rows):
                # wide (gate|up, LM head) and down-projection shapes: the quantised GEMM on the raw tile-blocks
                # (mode 9, 256 weight rows x 256 activation rows) won every measured one at M >= 256 -- Llama-3-8B
                # gate|up / LM head, Llama-3-70B gate|up / down / LM head by 10-20 % over mode 2
                # (profiles/tune_quant_70b_r05.txt); split K until the grid covers the 256 CUs
                tiles = sum((s.w.rows + 255) // 256 for s in segs) * ((M + 255) // 256)
                ks, nb = 1, K // 256
                while tiles * ks < 256 and ks * 2 <= min(8, max(1, nb // 4)):    # (ks <= 8: the tuned range)
                    ks *= 2
                return (9, 8, 2, ks)
            # LDS-dequant GEMM (mode 2): 128 weight rows x 256 (or 128) activation rows per workgroup;
            # split K until the grid covers the 256 CUs (the measured winners on the 8B shapes)
            tiles = sum((s.w.rows + 127) // 128 for s in segs) * ((M + 255) // 256)
            ks, nb = 1, K // 256
            while tiles * ks < 256 and ks * 2 <= max(1, nb // 4):
                ks *= 2
            return (2, 8, 4 if M >= 192 else 2, ks)
        return (1, 8, 1, 1)      # MFMA GEMM: 128 weight rows x 128 activation rows per workgroup
    waves, rt = 8, 1
    tiles = sum((s.w.rows + waves * rt * 16 - 1) // (waves * rt * 16) for s in segs)
    ks = 1
    nb = K // 256
    while tiles * ks < 256 and ks * 2 <= max(1, nb // 2):
        ks *= 2
    return (1, waves, rt, ks)


def dense_key(segs, M: int) -> str:
    return f"d:{sum(s.w.rows for s in segs)}:{segs[0].w.K}:{_mb(M)}"


def dense_heuristic(segs, M: int):
    """Modes 4/5/6 (dense f16 GEMM) for shapes without a tuned "d:" entry. Decode batches (M < 1024): 128 x 128 tiles
    on 16 waves (mode 4, wm 2) -- what the tuner picked for nearly every Llama-3-8B / Granite-3.0-2B shape at M = 256 /
    512, where the r05 rule (256 x 256 tiles from M >= 192) ran Granite's B=512 GEMMs 1.3-1.7x slower
    (profiles/granite_r06.txt); prefill chunks (M >= 1024): 256-row activation blocks with 256-row weight tiles
    (mode 5). Then the split-K that minimises (workgroup rounds over the 256 CUs) / ks, with a small per-slice cost."""
    if M < 1024:
        mode, bn, wm, waves = (4, 128, 2, 16) if M >= 128 else (4, 128, 2, 8)
    else:
        mode, bn, wm, waves = 5, 256, 4, 8
    bm = 64 * wm
    tiles = sum((s.w.rows + bn - 1) // bn for s in segs) * ((M + bm - 1) // bm)
    nkt = segs[0].w.K // 64
    best, best_ks = None, 1
    for ks in range(1, 9):
        if ks > 1 and nkt // ks < 8:
            break
        cost = -(-tiles * ks // 256) / ks + 0.03 * ks
        if best is None or cost < best - 1e-9:
            best, best_ks = cost, ks
    return (mode, waves, wm, best_ks)


def select_dense(segs, M: int):
    """Dense config, or None where the tuner measured the quantised GEMM faster (entry [-1])."""
    hit = table().get(dense_key(segs, M))
    if hit is not None and hit[0] < 0:
        return None
    return hit if hit is not None else dense_heuristic(segs, M)


# Llama-3-8B Q4_K_M shapes per projection role: the tuned entries an untuned shape of the same role borrows at
# the same batch bucket (M <= 64), e.g. Llama-3-70B / Qwen2.5-7B / Mixtral attention and dense FFN shapes
_ROLE_KEYS = {"qkv": "12+12+12:6144:4096", "o": "12:4096:4096", "gateup": "12:28672:4096", "down": "12:4096:14336",
              "lm_head": "14:128256:4096"}


def _role(segs) -> str:
    rows = sum(s.w.rows for s in segs)
    K = segs[0].w.K
    if len(segs) > 1:
        return "qkv"
    if rows >= 16 * K:
        return "lm_head"
    if rows >= 4 * K:
        return "gateup"
    if K >= 2 * rows:
        return "down"
    return "o"


def _role_entry(segs, M: int):
    """The Llama-3-8B entry of this shape's role and batch bucket, for a shape within 1.5x of that role's
    Llama-3-8B rows and K (Qwen2.5-7B, Mixtral attention: batch 16 / 64 2.70 / 4.30 vs 3.57 / 5.06 ms/step
    with the generic heuristic). Larger shapes keep the heuristic, whose split-K follows their own tile
    count (Llama-3-70B batch 64: 22.7 vs 24.4 ms/step borrowing); profiles/b1_models_r03.txt."""
    ref = _ROLE_KEYS[_role(segs)]
    _, rrows, rk = ref.split(":")
    rows, K = sum(s.w.rows for s in segs), segs[0].w.K
    near = lambda a, b: max(a, b) < 1.5 * min(a, b)
    if not (near(rows, int(rrows)) and near(K, int(rk))):
        return None
    return table().get(f"{ref}:{_mb(M)}")


def select(segs, M: int):
    hit = table().get(key(segs, M))
    if hit is None and M <= 64 and os.environ.get("NLS_TUNING_ROLE", "1") == "1":
        hit = _role_entry(segs, M)
    return hit if hit is not None else heuristic(segs, M)
