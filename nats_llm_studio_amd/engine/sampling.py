"""Sampling parameters (OpenAI / LM Studio chat fields) and the batched sampler.

Greedy rows never leave the device: the lm-head GEMV fuses the arg-max. Only
rows that ask for temperature / top-k / top-p / min-p / penalties go through
a sampler on their logits rows.

Every sampling path draws the SAME way: the kept tokens (penalties -> temperature -> top-k ->
min-p -> top-p) are walked in index order and the token where the cumulative mass passes u * Z
is taken, with u = uniform01(seed, position) -- the counter-based splitmix64 variate of
csrc/kernels/sample.hip. A seeded request therefore yields the same tokens whether it is sampled
in the decode hipGraph, by the batched GPU sampler on the host-driven path (tensor parallel,
logits requested) or by this module's CPU reference.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch


@dataclass
class SamplingParams:
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    min_p: float = 0.0
    repeat_penalty: float = 1.0
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    seed: Optional[int] = None
    max_tokens: int = 256
    stop: List[str] = field(default_factory=list)
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False

    @property
    def greedy(self) -> bool:
        return (self.temperature <= 0.0 and self.repeat_penalty == 1.0 and self.presence_penalty == 0.0
                and self.frequency_penalty == 0.0)

    @classmethod
    def from_request(cls, req: dict, default_max: int = 256, profile: Optional[str] = None) -> "SamplingParams":
        """OpenAI / LM Studio chat fields -> params. Fields the request omits come from `profile`
        (default: env NLS_SAMPLING_DEFAULTS, else "lmstudio"); see DEFAULT_PROFILES."""
        stop = req.get("stop") or []
        if isinstance(stop, str):
            stop = [stop]
        mt = req.get("max_tokens", req.get("max_completion_tokens"))
        if mt is None or int(mt) < 0:
            mt = default_max
        d = defaults_for(req, profile)

        def get(key, conv):
            v = req.get(key)
            return conv(d[key]) if v is None else conv(v)
        rp = get("repeat_penalty", float)
        if not rp > 0.0:        # 0 / negative / NaN: clients send 0 for "off"; v / 0 would make the logits inf
            rp = 1.0
        return cls(
            temperature=get("temperature", float),
            top_k=get("top_k", int),
            top_p=get("top_p", float),
            min_p=get("min_p", float),
            repeat_penalty=rp,
            presence_penalty=float(req.get("presence_penalty", 0.0) or 0.0),
            frequency_penalty=float(req.get("frequency_penalty", 0.0) or 0.0),
            seed=req.get("seed"),
            max_tokens=int(mt),
            stop=list(stop),
            ignore_eos=bool(req.get("ignore_eos", False)),
        )


# Values of the sampling fields a chat request omits. The reference forwards the request verbatim to LM Studio
# (`/root/reference/nats_llm_studio.go:348`), whose server fills omitted fields from its preset: temperature 0.8,
# top-k 40, top-p 0.95, min-p 0.05, repeat penalty 1.1 [ext: LM Studio defaults; no fixture in the reference pins
# them -- parity unpinned]. Decision (round 5):
#   "lmstudio" (default): a request that SAMPLES (temperature > 0) gets LM Studio's top-k / top-p / min-p /
#       repeat-penalty preset for the fields it omits -- the reference README's own payload `{"temperature":
#       0.7}` (README.md:196-204) samples as LM Studio would sample it. A request that omits temperature, or sends
#       0, decodes greedily with neutral penalties: deterministic output is this API's documented default (LM
#       Studio would sample at 0.8 there -- the one deliberate deviation).
#   "lmstudio-full": every omitted field from the preset, temperature 0.8 included (LM Studio's behaviour).
#   "neutral": the round-4 behaviour: omitted fields are neutral (top-k 0, top-p 1, min-p 0, penalty 1).
LMSTUDIO_PRESET = dict(temperature=0.8, top_k=40, top_p=0.95, min_p=0.05, repeat_penalty=1.1)
NEUTRAL = dict(temperature=0.0, top_k=0, top_p=1.0, min_p=0.0, repeat_penalty=1.0)
DEFAULT_PROFILES = ("lmstudio", "lmstudio-full", "neutral")


def defaults_for(req: dict, profile: Optional[str] = None) -> dict:
    import os
    profile = profile or os.environ.get("NLS_SAMPLING_DEFAULTS", "lmstudio")
    if profile == "lmstudio-full":
        return LMSTUDIO_PRESET
    if profile == "lmstudio":
        t = req.get("temperature")
        if t is not None and float(t) > 0.0:
            return dict(LMSTUDIO_PRESET, temperature=0.0)
        return NEUTRAL
    if profile == "neutral":
        return NEUTRAL
    raise ValueError(f"NLS_SAMPLING_DEFAULTS: unknown profile {profile!r} (one of {DEFAULT_PROFILES})")


_M64 = (1 << 64) - 1


def uniform01(seed: int, pos: int) -> float:
    """Counter-based uniform in [0, 1) of (seed, position): bit-exact twin of sample.hip uniform01."""
    z = (int(seed) + 0x9E3779B97F4A7C15 * (int(pos) + 1)) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    z ^= z >> 31
    return (z >> 40) * (1.0 / 16777216.0)


def sample_rows(logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                uniforms: Sequence) -> List[int]:
    """logits [n, V] -> one token per row (CPU reference of the GPU sampler; `uniforms`: one variate per
    row -- a float in [0, 1), a torch.Generator, or None for a fresh random one)."""
    out = []
    for i, p in enumerate(params):
        l = logits[i].float()
        hist = histories[i]
        if hist and (p.repeat_penalty != 1.0 or p.presence_penalty or p.frequency_penalty):
            ids = torch.tensor(list(hist[-64:]), device=l.device, dtype=torch.long)
            uniq, cnt = torch.unique(ids, return_counts=True)
            vals = l[uniq]
            if p.repeat_penalty != 1.0:
                vals = torch.where(vals > 0, vals / p.repeat_penalty, vals * p.repeat_penalty)
            vals = vals - p.presence_penalty - p.frequency_penalty * cnt.float()
            l = l.clone()
            l[uniq] = vals
        if p.temperature <= 0.0:
            out.append(int(l.argmax()))
            continue
        l = l.double()
        mx = l.max()
        lo = torch.tensor(float("-inf"), dtype=l.dtype)
        if p.top_k and 0 < p.top_k < l.numel():
            lo = torch.topk(l, p.top_k).values[-1]          # k-th largest logit (ties kept)
        if p.min_p > 0.0:
            lo = torch.maximum(lo, mx + p.temperature * math.log(p.min_p))
        w = torch.where(l >= lo, torch.exp((l - mx) / p.temperature), torch.zeros_like(l))
        if p.top_p < 1.0:                                   # smallest top set whose mass reaches top_p
            sw, si = torch.sort(w, descending=True)
            cum = torch.cumsum(sw, 0)
            n_keep = int(torch.searchsorted(cum, p.top_p * cum[-1]).item()) + 1
            thr = sw[min(n_keep, sw.numel()) - 1]
            w = torch.where(w >= thr, w, torch.zeros_like(w))
        cdf = torch.cumsum(w, 0)
        target = uniform(uniforms[i]) * float(cdf[-1])
        tok = int(torch.searchsorted(cdf, torch.tensor(target, dtype=cdf.dtype), right=True).item())
        kept = torch.nonzero(w > 0).flatten()
        if tok >= l.numel() or w[tok] <= 0:                  # rounding at the very end: last kept token
            tok = int(kept[-1]) if kept.numel() else 0
        out.append(tok)
    return out


HIST = 64      # penalty window (last tokens)


def uniform(u) -> float:
    """A row's variate: a float as given, a draw from a torch.Generator, or a fresh random one (None)."""
    if isinstance(u, float):
        return u
    if u is not None:
        return float(torch.rand(1, generator=u).item())
    import random
    return random.random()


def sample_rows_gpu(logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                    uniforms: Sequence) -> List[int]:
    """All sampled rows of a step in ONE kernel launch (csrc/kernels/sample.hip).
    `logits` [n, V] fp32 on the GPU is used as scratch (penalties are applied in place)."""
    return sample_rows_dev(logits, params, histories, uniforms).cpu().tolist()


def sample_rows_dev(logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                    uniforms: Sequence) -> torch.Tensor:
    """sample_rows_gpu without the read-back: the drawn ids as an int32 device tensor, stream-ordered."""
    import ctypes
    import numpy as np
    from ..ops import _lib
    n, V = len(params), logits.shape[1]
    if logits.shape[0] < n:
        raise ValueError(f"{logits.shape[0]} logit rows for {n} sampling requests")
    logits = logits[:n]
    lg = logits if logits.is_contiguous() and logits.dtype == torch.float32 else logits.float().contiguous()
    P = (_lib.SampleParams * n)()
    hist = np.full((n, HIST), -1, dtype=np.int32)
    for i, p in enumerate(params):
        h = list(histories[i])[-HIST:]
        hist[i, :len(h)] = h
        P[i] = _lib.SampleParams(p.temperature, p.top_p, p.min_p, p.repeat_penalty, p.presence_penalty,
                                 p.frequency_penalty, uniform(uniforms[i]), int(p.top_k or 0), len(h), 0)
    dev = lg.device
    # pinned, non_blocking uploads: a pageable upload would wait for the whole stream (the prefill chunk)
    pbytes = torch.frombuffer(bytearray(bytes(P)), dtype=torch.uint8).pin_memory().to(dev, non_blocking=True)
    hd = torch.from_numpy(hist).pin_memory().to(dev, non_blocking=True)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.lib().nls_sample(lg.data_ptr(), lg.stride(0), n, V, pbytes.data_ptr(), hd.data_ptr(), HIST,
                                     out.data_ptr(), stream), "nls_sample")
    return out
