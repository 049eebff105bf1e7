"""Sampling parameters (OpenAI / LM Studio chat fields) and the batched sampler.

Greedy rows never leave the device: the lm-head GEMV fuses the arg-max. Only
rows that ask for temperature / top-k / top-p / min-p / penalties go through
this torch sampler on their logits rows.
"""
from __future__ import annotations

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
    def from_request(cls, req: dict, default_max: int = 256) -> "SamplingParams":
        stop = req.get("stop") or []
        if isinstance(stop, str):
            stop = [stop]
        mt = req.get("max_tokens", req.get("max_completion_tokens"))
        if mt is None or int(mt) < 0:
            mt = default_max
        temp = req.get("temperature")
        return cls(
            temperature=0.0 if temp is None else float(temp),
            top_k=int(req.get("top_k", 0) or 0),
            top_p=float(req.get("top_p", 1.0) if req.get("top_p") is not None else 1.0),
            min_p=float(req.get("min_p", 0.0) or 0.0),
            repeat_penalty=float(req.get("repeat_penalty", 1.0) or 1.0),
            presence_penalty=float(req.get("presence_penalty", 0.0) or 0.0),
            frequency_penalty=float(req.get("frequency_penalty", 0.0) or 0.0),
            seed=req.get("seed"),
            max_tokens=int(mt),
            stop=list(stop),
            ignore_eos=bool(req.get("ignore_eos", False)),
        )


def sample_rows(logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                generators: Sequence[Optional[torch.Generator]]) -> List[int]:
    """logits [n, V] (device) -> one token per row."""
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
        l = l / p.temperature
        if p.top_k and p.top_k > 0:
            kth = torch.topk(l, min(p.top_k, l.numel())).values[-1]
            l = torch.where(l < kth, torch.full_like(l, float("-inf")), l)
        probs = torch.softmax(l, dim=-1)
        if p.min_p > 0.0:
            probs = torch.where(probs < p.min_p * probs.max(), torch.zeros_like(probs), probs)
        if p.top_p < 1.0:
            sp, si = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            keep = cum - sp < p.top_p
            keep[0] = True
            mask = torch.zeros_like(probs, dtype=torch.bool)
            mask[si[keep]] = True
            probs = torch.where(mask, probs, torch.zeros_like(probs))
        probs = probs / probs.sum()
        g = generators[i]
        if g is not None and g.device != probs.device:
            tok = int(torch.multinomial(probs.cpu(), 1, generator=g))
        else:
            tok = int(torch.multinomial(probs, 1, generator=g))
        out.append(tok)
    return out


HIST = 64      # penalty window (last tokens)


def uniform(gen: Optional[torch.Generator]) -> float:
    if gen is not None:
        return float(torch.rand(1, generator=gen).item())
    import random
    return random.random()


def sample_rows_gpu(logits: torch.Tensor, params: Sequence[SamplingParams], histories: Sequence[Sequence[int]],
                    generators: Sequence[Optional[torch.Generator]]) -> List[int]:
    """All sampled rows of a step in ONE kernel launch (csrc/kernels/sample.hip).
    `logits` [n, V] fp32 on the GPU is used as scratch (penalties are applied in place)."""
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
                                 p.frequency_penalty, uniform(generators[i]), int(p.top_k or 0), len(h), 0)
    dev = lg.device
    pbytes = torch.frombuffer(bytearray(bytes(P)), dtype=torch.uint8).to(dev)
    hd = torch.from_numpy(hist).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.lib().nls_sample(lg.data_ptr(), lg.stride(0), n, V, pbytes.data_ptr(), hd.data_ptr(), HIST,
                                     out.data_ptr(), stream), "nls_sample")
    return out.cpu().tolist()
