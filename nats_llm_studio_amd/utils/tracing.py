"""Per-request tracing (SURVEY.md §5 "Tracing / profiling": the reference only has three
log.Printf calls, `nats_llm_studio.go:95, 210, 215`).

A chat request is traced as monotonic spans
    recv -> validate -> tokenize (chat template + BPE, model pin) -> queue (engine admission wait)
         -> prefill (admission -> first token) -> decode -> respond (reply JSON + publish)
kept in a bounded ring (exposed by `lmstudio.metrics`, phase percentiles + the last traces)
and, with NLS_TRACE=1, written as one JSON log line per request.
"""
from __future__ import annotations

import collections
import os
import threading
from typing import Dict, List, Optional

from .metrics import LatencyHistogram, log

PHASES = ("validate", "tokenize", "queue", "prefill", "decode", "respond", "total")


class Tracer:
    def __init__(self, keep: int = 256):
        self._lock = threading.Lock()
        self.recent: "collections.deque[dict]" = collections.deque(maxlen=keep)
        self.phase = {p: LatencyHistogram() for p in PHASES}
        self.emit = os.environ.get("NLS_TRACE", "0") == "1"

    def record(self, subject: str, request_id: str, marks: Dict[str, float], extra: Optional[dict] = None):
        """marks: monotonic timestamps recv, validated, queued?, admitted?, first_token?, done?, responded."""
        t0 = marks["recv"]
        spans = {}

        def span(name, a, b):
            if a in marks and b in marks and marks[b] >= marks[a]:
                spans[name] = marks[b] - marks[a]

        span("validate", "recv", "validated")
        span("tokenize", "validated", "queued")
        span("queue", "queued", "admitted")
        span("prefill", "admitted", "first_token")
        span("decode", "first_token", "done")
        span("respond", "done" if "done" in marks else "validated", "responded")
        span("total", "recv", "responded")
        rec = {"subject": subject, "request_id": request_id,
               "spans_ms": {k: round(v * 1e3, 3) for k, v in spans.items()},
               "t_rel_ms": {k: round((v - t0) * 1e3, 3) for k, v in marks.items()}}
        if extra:
            rec.update(extra)
        with self._lock:
            self.recent.append(rec)
        for k, v in spans.items():
            self.phase[k].add(v)
        if self.emit:
            log("trace", **rec)
        return rec

    def summary(self, last: int = 10) -> dict:
        with self._lock:
            tail: List[dict] = list(self.recent)[-last:] if last > 0 else []
        return {"phases_ms": {k: h.summary_ms() for k, h in self.phase.items() if h.count},
                "recent": tail}
