"""GPU clock / power / temperature telemetry for the benchmark record (amdsmi, read-only).

The headline number moves with the package power limit: the B=512 step draws ~1.4 kW and the
GFX clock then drops from ~2.4 GHz (`profiles/clocks_power_b512.txt`). `GpuTelemetry` samples
the GPU that a torch device maps to (matched by PCI bus id, so it works when the container sees a
subset of the node's GPUs) at both brackets of a timed region and, from a background thread,
in between. Everything here is best effort: any amdsmi failure yields `None` fields, never an
exception in the bench.
"""
from __future__ import annotations

import threading
import time


def _handle_for(device_index: int):
    import amdsmi
    amdsmi.amdsmi_init()
    handles = amdsmi.amdsmi_get_processor_handles()
    if not handles:
        return None
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        bus = int(getattr(p, "pci_bus_id"))
        dev = int(getattr(p, "pci_device_id", 0))
        for h in handles:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)       # "dddd:bb:dd.f"
            _, b, df = bdf.split(":")
            if int(b, 16) == bus and int(df.split(".")[0], 16) == dev:
                return h
    except Exception:
        pass
    return handles[device_index] if device_index < len(handles) else handles[0]


class GpuTelemetry:
    """`snap()` -> {"gfx_mhz", "mem_mhz", "power_w", "hotspot_c", "throttle"}; `start()`/`stop()` bracket
    a region and `summary()` reports the two bracket snapshots plus min/mean/max of the samples."""

    FIELDS = ("gfx_mhz", "mem_mhz", "power_w", "hotspot_c")

    def __init__(self, device_index: int = 0, period_s: float = 0.05):
        self.period = period_s
        self.err = None
        try:
            self.h = _handle_for(device_index)
        except Exception as e:         # amdsmi missing / no permission: report why, keep going
            self.h, self.err = None, f"{type(e).__name__}: {e}"[:160]
        self.samples = []
        self._stop = threading.Event()
        self._thr = None
        self.begin = self.end = None

    def snap(self) -> dict:
        out = dict.fromkeys(self.FIELDS)
        if self.h is None:
            return out
        import amdsmi
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        except Exception:
            m = {}

        def num(v):
            return v if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF) else None
        gfx = m.get("current_gfxclk")
        if num(gfx) is None:
            clks = [c for c in (m.get("current_gfxclks") or []) if num(c)]
            gfx = max(clks) if clks else None
        out["gfx_mhz"] = num(gfx)
        out["mem_mhz"] = num(m.get("current_uclk"))
        out["power_w"] = num(m.get("current_socket_power")) or num(m.get("average_socket_power"))
        out["hotspot_c"] = num(m.get("temperature_hotspot"))
        if out["power_w"] is None:
            try:
                p = amdsmi.amdsmi_get_power_info(self.h)
                out["power_w"] = num(p.get("current_socket_power")) or num(p.get("average_socket_power"))
            except Exception:
                pass
        if out["gfx_mhz"] is None:
            try:
                out["gfx_mhz"] = num(amdsmi.amdsmi_get_clock_info(self.h, amdsmi.AmdSmiClkType.GFX)["clk"])
            except Exception:
                pass
        if out["hotspot_c"] is None:
            try:
                out["hotspot_c"] = num(amdsmi.amdsmi_get_temp_metric(
                    self.h, amdsmi.AmdSmiTemperatureType.HOTSPOT, amdsmi.AmdSmiTemperatureMetric.CURRENT))
            except Exception:
                pass
        thr = m.get("throttle_status")
        out["throttle"] = thr if isinstance(thr, int) and thr != 0xFFFFFFFF else None
        # residency counters (ticks of `accumulation_counter`) in package-power (PPT) and thermal limiting
        for k in ("accumulation_counter", "ppt_residency_acc", "socket_thm_residency_acc"):
            v = m.get(k)
            out[k] = v if isinstance(v, int) else None
        return out

    def _run(self):
        while not self._stop.wait(self.period):
            self.samples.append(self.snap())

    def start(self):
        self.begin = self.snap()
        self.samples = []
        self._stop.clear()
        if self.h is not None:
            self._thr = threading.Thread(target=self._run, daemon=True, name="gpu-telemetry")
            self._thr.start()

    def stop(self):
        self._stop.set()
        if self._thr is not None:
            self._thr.join(timeout=2.0)
        self.end = self.snap()

    def summary(self) -> dict:
        s = {"source": "amdsmi" if self.h is not None else None, "begin": self.begin, "end": self.end,
             "n_samples": len(self.samples)}
        if self.err:
            s["error"] = self.err
        # a timed region shorter than one sampling period (batch-1 runs) has no periodic samples: its begin / end
        # snapshots stand in, so every record carries the clock it ran at
        pts = self.samples or [x for x in (self.begin, self.end) if x]
        for f in self.FIELDS:
            xs = [x[f] for x in pts if x.get(f) is not None]
            if xs:
                s[f] = {"min": min(xs), "mean": round(sum(xs) / len(xs), 1), "max": max(xs)}
        b, e = self.begin or {}, self.end or {}
        try:       # fraction of the region the package spent power- / thermally-limited
            dt = e["accumulation_counter"] - b["accumulation_counter"]
            if dt > 0:
                s["ppt_limited_frac"] = round((e["ppt_residency_acc"] - b["ppt_residency_acc"]) / dt, 3)
                s["thermal_limited_frac"] = round(
                    (e["socket_thm_residency_acc"] - b["socket_thm_residency_acc"]) / dt, 3)
        except (KeyError, TypeError):
            pass
        for snap in (b, e):
            for k in ("accumulation_counter", "ppt_residency_acc", "socket_thm_residency_acc"):
                snap.pop(k, None)
        return s


def sample_once(device_index: int = 0) -> dict:
    t = GpuTelemetry(device_index)
    return {"t": time.time(), **t.snap()}
