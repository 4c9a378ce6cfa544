"""GPU clock / power / temperature telemetry around a timed region (amdsmi).

The bench brackets its timed steps with :class:`GpuTelemetry` so every JSON
line says what the chip was doing while it was measured: the graphics clock
it held (per-XCD ``current_gfxclks``, sampled), socket power, hotspot and HBM
temperature, and how much of the region the firmware spent power-limited
(``ppt_residency_acc``) or thermally limited (``socket_thm_residency_acc``).
MI355X lowers its clock under MFMA load (guide: "DVFS give-back"), and boxes
differ by a few percent, so two runs of one binary are comparable only
together with these numbers.

Sampling runs on a daemon thread every ``period`` seconds; it reads firmware
counters only (no GPU work, no HIP calls).  Everything degrades to
``{"available": False, "error": ...}`` where amdsmi or the metrics table is
missing (CPU tests, containers without the driver).
"""
from __future__ import annotations

import threading
import time
from typing import Any, Dict, List, Optional

_NA = "N/A"


def _num(v) -> Optional[float]:
    if v is None or v == _NA or isinstance(v, str):
        return None
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def _stats(xs: List[float], nd: int = 1) -> Optional[Dict[str, float]]:
    xs = [x for x in xs if x is not None]
    if not xs:
        return None
    return {"mean": round(sum(xs) / len(xs), nd), "min": round(min(xs), nd), "max": round(max(xs), nd)}


class GpuTelemetry:
    """Samples one GPU's firmware metrics between :meth:`start` and :meth:`stop`."""

    def __init__(self, device_index: int = 0, period: float = 0.05):
        self.device_index = device_index
        self.period = period
        self._smi = None
        self._h = None
        self._err: Optional[str] = None
        self._samples: List[Dict[str, Any]] = []
        self._m0: Optional[Dict[str, Any]] = None
        self._t0 = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._open()

    # -- amdsmi handle for the torch device (matched by PCI bus id) ---------------
    def _open(self) -> None:
        try:
            import amdsmi  # noqa: WPS433
            import torch

            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            want = None
            try:
                props = torch.cuda.get_device_properties(self.device_index)
                want = int(getattr(props, "pci_bus_id", -1))
            except Exception:  # noqa: BLE001
                pass
            pick = None
            for h in handles:
                bdf = str(amdsmi.amdsmi_get_gpu_device_bdf(h))  # "dddd:bb:dd.f"
                try:
                    bus = int(bdf.split(":")[1], 16)
                except (IndexError, ValueError):
                    continue
                if want is not None and bus == want:
                    pick = h
                    break
            if pick is None and len(handles) == 1:
                pick = handles[0]
            if pick is None:
                raise RuntimeError(f"no amdsmi handle with PCI bus {want} among {len(handles)}")
            self._smi, self._h = amdsmi, pick
            self._metrics()  # probe once
        except Exception as exc:  # noqa: BLE001
            self._smi = self._h = None
            self._err = f"{type(exc).__name__}: {exc}"[:200]

    @property
    def available(self) -> bool:
        return self._h is not None

    def _metrics(self) -> Dict[str, Any]:
        return self._smi.amdsmi_get_gpu_metrics_info(self._h)

    def _sample(self) -> Dict[str, Any]:
        m = self._metrics()
        clks = [c for c in (_num(x) for x in (m.get("current_gfxclks") or [])) if c]
        return {
            "t": time.perf_counter(),
            "gfxclk": sum(clks) / len(clks) if clks else _num(m.get("current_gfxclk")),
            "power": _num(m.get("current_socket_power")),
            "hotspot": _num(m.get("temperature_hotspot")),
            "mem": _num(m.get("temperature_mem")),
            "uclk": _num(m.get("current_uclk")),  # HBM clock
            "fclk": _num(m.get("current_fclk")),  # data-fabric clock (absent on some firmware tables)
        }

    def _loop(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self._samples.append(self._sample())
            except Exception as exc:  # noqa: BLE001
                self._err = f"{type(exc).__name__}: {exc}"[:200]
                return

    # -- public ------------------------------------------------------------------
    def start(self) -> "GpuTelemetry":
        if not self.available:
            return self
        self._samples = []
        self._stop.clear()
        try:
            self._m0 = self._metrics()
        except Exception as exc:  # noqa: BLE001
            self._err = f"{type(exc).__name__}: {exc}"[:200]
            self._m0 = None
        self._t0 = time.perf_counter()
        self._thread = threading.Thread(target=self._loop, name="gpu-telemetry", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> Dict[str, Any]:
        if not self.available:
            return {"available": False, "error": self._err}
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2.0)
        out: Dict[str, Any] = {"available": True, "samples": len(self._samples),
                               "period_s": self.period, "source": "amdsmi gpu_metrics"}
        s = self._samples
        out["gfxclk_mhz"] = _stats([x["gfxclk"] for x in s], 0)
        out["socket_power_w"] = _stats([x["power"] for x in s], 0)
        out["hotspot_c"] = _stats([x["hotspot"] for x in s], 0)
        out["hbm_c"] = _stats([x["mem"] for x in s], 0)
        for key, name in (("uclk", "uclk_mhz"), ("fclk", "fclk_mhz")):
            st = _stats([x[key] for x in s], 0)
            if st is not None:
                out[name] = st
        try:
            m1 = self._metrics()
            m0 = self._m0 or {}
            acc0, acc1 = _num(m0.get("accumulation_counter")), _num(m1.get("accumulation_counter"))
            if acc0 is not None and acc1 is not None and acc1 > acc0:
                for key, name in (("ppt_residency_acc", "power_limited_pct"),
                                  ("socket_thm_residency_acc", "thermal_limited_pct"),
                                  ("prochot_residency_acc", "prochot_pct")):
                    a, b = _num(m0.get(key)), _num(m1.get(key))
                    if a is not None and b is not None:
                        out[name] = round(100.0 * (b - a) / (acc1 - acc0), 1)
            lim = self._smi.amdsmi_get_power_cap_info(self._h)
            cap = _num(lim.get("power_cap")) if isinstance(lim, dict) else None
            if cap:
                out["power_cap_w"] = round(cap / 1e6, 0) if cap > 1e4 else cap
        except Exception as exc:  # noqa: BLE001
            out["counters_error"] = f"{type(exc).__name__}: {exc}"[:200]
        if self._err:
            out["error"] = self._err
        return out
