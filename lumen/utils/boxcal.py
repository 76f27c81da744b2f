"""Box calibration for bench records (``extra.box``; VERDICT r5 "Next" #3).

The library GEMMs that make up ~80 % of a training step are power-limited on MI355X: the chip
holds 1.5-2.0 GHz under sustained MFMA load (profiles/r5_gemm_clock), and boards differ, so one
tree's step time moves 1-3 % from box to box.  A record that carries, from the same process and
the same lease:

* the GPU's clock and board power sampled from sysfs hwmon through the timed region;
* the time of a FIXED 8192^3 bf16 hipBLASLt GEMM (the compute-bound half of the step);
* the time of a FIXED 4 GiB non-temporal HBM read (kernels/calib.hip: the bandwidth-bound half)

lets a reader divide the box out: a record whose fixed GEMM ran 3 % slow was a slow box, one
whose fixed work matched the last record but whose step did not is the tree.  The reference's
only number is a single tqdm rate on one V100 (training/train.ipynb:442); ours must be
reproducible.
"""
from __future__ import annotations

import glob
import os
import threading
import time
from typing import Dict, List, Optional

import torch


def gpu_hwmon(device=None) -> Optional[str]:
    """The hwmon directory of ``device``'s PCI function (sysfs), or None where it cannot be
    found (CPU runs, containers without /sys/bus/pci)."""
    try:
        p = torch.cuda.get_device_properties(device if device is not None else 0)
        dom = getattr(p, "pci_domain_id", 0)
        bus, dv = getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None)
    except Exception:  # noqa: BLE001
        return None
    if bus is None or dv is None:
        return None
    for fn in range(8):
        hw = sorted(glob.glob(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dv:02x}.{fn}/hwmon/hwmon*"))
        if hw:
            return hw[0]
    return None


def _read_num(path: str) -> Optional[float]:
    try:
        with open(path) as f:
            return float(f.read().strip())
    except (OSError, ValueError):
        return None


class HwmonSampler:
    """Samples SCLK (``freq1_input``, Hz) and board power (``power1_average`` or
    ``power1_input``, microwatts) every ``period_s`` on a daemon thread between ``start()`` and
    ``stop()``.  File reads only: no GPU call, nothing on the device timeline."""

    def __init__(self, hwmon: Optional[str], period_s: float = 0.02):
        self.hwmon = hwmon
        self.period_s = period_s
        self.sclk: List[float] = []
        self.power: List[float] = []
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None
        pw = None
        if hwmon:
            for name in ("power1_average", "power1_input"):
                if os.path.exists(os.path.join(hwmon, name)):
                    pw = os.path.join(hwmon, name)
                    break
        self._pw = pw
        self._fq = os.path.join(hwmon, "freq1_input") if hwmon and os.path.exists(
            os.path.join(hwmon, "freq1_input")) else None

    def _run(self):
        while not self._stop.is_set():
            if self._fq:
                v = _read_num(self._fq)
                if v is not None:
                    self.sclk.append(v / 1e6)
            if self._pw:
                v = _read_num(self._pw)
                if v is not None:
                    self.power.append(v / 1e6)
            self._stop.wait(self.period_s)

    def start(self) -> "HwmonSampler":
        if self._fq or self._pw:
            self._t = threading.Thread(target=self._run, daemon=True, name="lumen-hwmon")
            self._t.start()
        return self

    def stop(self) -> Dict:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=1.0)
        return summarize(self.sclk, self.power, self.hwmon)


def summarize(sclk: List[float], power: List[float], hwmon: Optional[str]) -> Dict:
    out: Dict = {"hwmon": hwmon, "samples": max(len(sclk), len(power))}
    if sclk:
        s = sorted(sclk)
        out.update(sclk_mhz_mean=round(sum(s) / len(s), 1), sclk_mhz_min=round(s[0], 1),
                   sclk_mhz_p50=round(s[len(s) // 2], 1), sclk_mhz_max=round(s[-1], 1))
    if power:
        p = sorted(power)
        out.update(power_w_mean=round(sum(p) / len(p), 1), power_w_max=round(p[-1], 1))
    return out


def _batch_ms(fn, n: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


def fixed_work(device, gemm_n: int = 8192, hbm_gib: int = 4, reps: int = 5,
               hwmon: Optional[str] = None, batch: int = 60) -> Dict:
    """The fixed calibration work on ``device``: an n^3 bf16 GEMM (hipBLASLt, uniform [-1, 1)
    operands: the power-hungry case) and a ``hbm_gib`` GiB non-temporal read.  Each is run in
    back-to-back batches of ``batch`` launches (~55 ms for the GEMM, long enough for the clock
    and power to settle as they do in a training step) after a ~0.2 s warm-up; the medians of
    ``reps`` batches, with the clock / power sampled during the GEMM batches."""
    out: Dict = {}
    g = torch.Generator(device=device).manual_seed(7)
    a = torch.rand(gemm_n, gemm_n, device=device, generator=g, dtype=torch.float32).mul_(2).sub_(1)
    a = a.to(torch.bfloat16)
    b = torch.rand(gemm_n, gemm_n, device=device, generator=g, dtype=torch.float32).mul_(2).sub_(1)
    b = b.to(torch.bfloat16)
    c = torch.empty(gemm_n, gemm_n, device=device, dtype=torch.bfloat16)
    fn = lambda: torch.mm(a, b, out=c)  # noqa: E731
    _batch_ms(fn, 4 * batch)
    smp = HwmonSampler(hwmon, period_s=0.005).start()
    ts = sorted(_batch_ms(fn, batch) for _ in range(reps))
    clk = smp.stop()
    med = ts[len(ts) // 2]
    out["gemm"] = {"shape": f"{gemm_n}^3 bf16 (uniform [-1, 1))", "ms_med": round(med, 3),
                   "ms_min": round(ts[0], 3),
                   "pflops": round(2.0 * gemm_n ** 3 / (med * 1e-3) / 1e15, 3),
                   "sclk_mhz_mean": clk.get("sclk_mhz_mean"), "power_w_mean": clk.get("power_w_mean")}
    del a, b, c
    try:
        from ..ops._native import native

        C = native()
        if C is None or not hasattr(C, "hbm_read"):
            raise RuntimeError("native extension without hbm_read")
        nbytes = hbm_gib << 30
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        buf.fill_(1)
        sink = torch.zeros(1, dtype=torch.int32, device=device)
        blocks = 4096
        fn = lambda: C.hbm_read(buf, sink, blocks)  # noqa: E731
        _batch_ms(fn, batch)
        ts = sorted(_batch_ms(fn, batch) for _ in range(reps))
        med = ts[len(ts) // 2]
        out["hbm_read"] = {"gib": hbm_gib, "ms_med": round(med, 3), "ms_min": round(ts[0], 3),
                           "tbps": round(nbytes / (med * 1e-3) / 1e12, 3), "nontemporal": True}
        del buf
    except Exception as e:  # noqa: BLE001 - the GEMM number stands
        out["hbm_read"] = {"error": repr(e)[:200]}
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
    return out


def device_identity(device) -> Dict:
    try:
        p = torch.cuda.get_device_properties(device)
        return {"name": p.name, "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:"
                f"{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}",
                "cus": p.multi_processor_count, "host": os.uname().nodename}
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)[:200]}


def box_record(device, timed: Dict, fixed: Dict) -> Dict:
    return {"device": device_identity(device), "timed_region": timed, "fixed_work": fixed,
            "sampled_at": time.strftime("%Y-%m-%dT%H:%M:%S")}
