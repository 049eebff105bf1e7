"""Small observability helpers: latency histograms and structured (JSON) logs."""
from __future__ import annotations

import json
import sys
import threading
import time


class LatencyHistogram:
    """Keeps the last `cap` samples (seconds) for exact percentiles."""

    def __init__(self, cap: int = 8192):
        self.cap = cap
        self.samples = []
        self.count = 0
        self._lock = threading.Lock()

    def add(self, s: float):
        with self._lock:
            self.count += 1
            if len(self.samples) >= self.cap:
                self.samples.pop(0)
            self.samples.append(s)

    def percentile(self, p: float) -> float:
        with self._lock:
            if not self.samples:
                return 0.0
            xs = sorted(self.samples)
        k = min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))
        return xs[k]

    def summary_ms(self) -> dict:
        return {"count": self.count, "p50": round(self.percentile(50) * 1e3, 4),
                "p90": round(self.percentile(90) * 1e3, 4), "p99": round(self.percentile(99) * 1e3, 4)}


def log(event: str, **kw):
    rec = {"ts": round(time.time(), 6), "event": event, **kw}
    sys.stderr.write(json.dumps(rec, default=str) + "\n")
    sys.stderr.flush()
