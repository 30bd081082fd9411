"""Run-environment telemetry for benchmark lines (NS-09): what the GPU was doing while the timed
loop ran, and which GEMM selections were really in use.

* ``GpuSampler`` — a background thread that samples the device's graphics / memory clocks,
  socket power, power cap and temperature through amdsmi (ROCm's SMI library) every
  ``period`` seconds; ``summary()`` gives min / mean / max. MI355X boards differ by up to ~12 %
  in the clock they hold under an MFMA-dense load (MI355X_MICROARCH.md, 'DVFS give-back' item 5),
  so a throughput number is only comparable across boxes next to the clock it ran at.
* ``tunableop_status()`` — whether PyTorch TunableOp is enabled, how many tuned GEMM
  selections it holds (after the run: >0 only if the committed results file validated against
  this box's hipBLASLt / rocBLAS / PyTorch versions and was loaded), and the validator values.
* ``library_versions()`` — hipBLASLt / rocBLAS / HIP / torch versions.

Everything degrades to ``None`` fields when amdsmi or a counter is unavailable (CPU runs).
"""
from __future__ import annotations

import os
import statistics
import threading
import time


def _amdsmi_handle(device_index: int):
    import amdsmi

    amdsmi.amdsmi_init()
    handles = amdsmi.amdsmi_get_processor_handles()
    if not handles:
        return amdsmi, None
    target = None
    try:
        import torch

        props = torch.cuda.get_device_properties(device_index)
        bus = getattr(props, "pci_bus_id", None)
        dev = getattr(props, "pci_device_id", None)
        if bus is not None:
            for h in handles:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "0000:75:00.0"
                parts = bdf.split(":")
                if len(parts) >= 3 and int(parts[1], 16) == bus and (dev is None or int(parts[2].split(".")[0], 16) == dev):
                    target = h
                    break
    except Exception:
        target = None
    if target is None:
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
        idx = device_index
        if vis:
            try:
                idx = int(vis.split(",")[device_index])
            except Exception:
                idx = device_index
        target = handles[idx] if idx < len(handles) else handles[0]
    return amdsmi, target


def _read(amdsmi, h):
    out = {}
    try:
        out["sclk_mhz"] = float(amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)["clk"])
    except Exception:
        pass
    try:
        out["mclk_mhz"] = float(amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.MEM)["clk"])
    except Exception:
        pass
    try:
        p = amdsmi.amdsmi_get_power_info(h)
        for k in ("current_socket_power", "average_socket_power", "socket_power"):
            v = p.get(k)
            if isinstance(v, (int, float)) and v > 0:
                out["power_w"] = float(v)
                break
        cap = p.get("power_limit")
        if isinstance(cap, (int, float)) and cap > 0:
            out["power_cap_w"] = float(cap) / (1e6 if cap > 1e5 else 1.0)
    except Exception:
        pass
    try:
        t = amdsmi.amdsmi_get_temp_metric(h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                                          amdsmi.AmdSmiTemperatureMetric.CURRENT)
        out["temp_c"] = float(t)
    except Exception:
        pass
    return out


class GpuSampler:
    """Samples clocks / power in a daemon thread between start() and stop()."""

    def __init__(self, device_index: int = 0, period: float = 0.1):
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._thread = None
        try:
            self._smi, self._h = _amdsmi_handle(device_index)
        except Exception:
            self._smi, self._h = None, None

    @property
    def available(self):
        return self._h is not None

    def snapshot(self):
        return _read(self._smi, self._h) if self.available else {}

    def _loop(self):
        while not self._stop.is_set():
            s = _read(self._smi, self._h)
            if s:
                self.samples.append(s)
            self._stop.wait(self.period)

    def start(self):
        if self.available:
            self._thread = threading.Thread(target=self._loop, daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
        return self.summary()

    def summary(self):
        if not self.samples:
            return None
        out = {"samples": len(self.samples)}
        for key in ("sclk_mhz", "mclk_mhz", "power_w", "temp_c"):
            vals = [s[key] for s in self.samples if key in s]
            if vals:
                out[key] = {"min": round(min(vals), 1), "mean": round(statistics.fmean(vals), 1),
                            "max": round(max(vals), 1)}
        caps = [s["power_cap_w"] for s in self.samples if "power_cap_w" in s]
        if caps:
            out["power_cap_w"] = round(caps[-1], 1)
        return out


def tunableop_status():
    try:
        import torch

        t = torch.cuda.tunable
        enabled = bool(t.is_enabled())
        out = {"enabled": enabled, "tuning": bool(t.tuning_is_enabled())}
        try:
            out["results_loaded"] = len(t.get_results())
        except Exception:
            out["results_loaded"] = None
        try:
            out["validators"] = {k: v for k, v in t.get_validators()}
        except Exception:
            pass
        try:
            out["filename"] = os.path.basename(t.get_filename())
        except Exception:
            pass
        return out
    except Exception as e:  # pragma: no cover
        return {"error": repr(e)}


def committed_validators(path: str):
    """Validator lines of a committed TunableOp results file."""
    out = {}
    try:
        with open(path) as f:
            for line in f:
                if line.startswith("Validator,"):
                    _, k, v = line.rstrip("\n").split(",", 2)
                    out[k] = v
    except OSError:
        pass
    return out


def library_versions():
    out = {}
    try:
        import torch

        out["torch"] = torch.__version__
        out["hip"] = torch.version.hip
    except Exception:
        pass
    hdr = "/opt/rocm/include/hipblaslt/hipblaslt-version.h"
    try:
        with open(hdr) as f:
            txt = f.read()
        import re

        parts = [re.search(r"#define\s+hipblasLt_VERSION_%s\s+(\w+)" % k, txt) for k in ("MAJOR", "MINOR", "PATCH")]
        if all(parts):
            out["hipblaslt_header"] = ".".join(p.group(1) for p in parts)
    except OSError:
        pass
    return out


class StepTimer:
    """Per-step device time from HIP events recorded between steps (no host sync inside the
    loop); ``summary()`` after the final synchronize."""

    def __init__(self, enabled=True):
        self.events = []
        self.enabled = enabled

    def mark(self):
        if self.enabled:
            import torch

            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)

    def summary(self):
        if len(self.events) < 2:
            return None
        ms = [a.elapsed_time(b) for a, b in zip(self.events[:-1], self.events[1:])]
        return {"min": round(min(ms), 3), "median": round(statistics.median(ms), 3),
                "max": round(max(ms), 3), "first": round(ms[0], 3), "last": round(ms[-1], 3)}


def wall():
    return time.perf_counter()
