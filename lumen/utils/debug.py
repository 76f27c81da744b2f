"""Tracing, debug guards and fault injection (SURVEY.md section 5 aux subsystems).

The reference has none of these (its only knob is ``wall_clock_breakdown: false``,
configs/ds_config_zero1.json:48); lumen adds them behind environment variables so the hot path
pays nothing when they are off:

``LUMEN_PROFILE=1``        torch.profiler over optimizer steps ``LUMEN_PROFILE_WAIT`` (default 2)
                           .. +``LUMEN_PROFILE_ACTIVE`` (default 3); writes a Chrome trace per rank
                           to ``LUMEN_PROFILE_DIR`` (``./profiles/torch``) and prints the top
                           kernels on rank 0.  ``trace_range()`` ranges show up as roctx markers
                           in rocprofv3 ``--marker-trace`` and as user annotations in the trace.
``LUMEN_DEBUG=1``          synchronous kernel launches (``AMD_SERIALIZE_KERNEL=3``,
                           ``HIP_LAUNCH_BLOCKING=1``; must be set before the first HIP call, so
                           ``lumen.parallel.dist.init`` applies it), NaN/Inf guards on the loss and
                           on the flat gradient buffer after every backward, and a device sync
                           around collectives (stream-ordering bugs surface as errors at the
                           offending call instead of wrong numbers later).
``LUMEN_ZERO3_POISON=1``   race detector for the ZeRO-3 gather schedules (also on under
                           ``LUMEN_DEBUG``): every gathered-weight buffer is filled with NaN on the
                           compute stream right before it is (re-)gathered, so a kernel that reads
                           a buffer outside its live window -- a release-ring buffer already
                           handed to the next unit, a keep unit read before its first gather
                           landed -- turns the loss NaN at once instead of silently reading
                           identical-looking stale weights.
``LUMEN_FAULT_STEP=k``     fault injection: the rank(s) in ``LUMEN_FAULT_RANK`` (default 0) exit
                           with code 17 right after optimizer step k (after any checkpoint of
                           that step).  Used by the kill-and-resume equality test.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch

FAULT_EXIT_CODE = 17


def debug_enabled() -> bool:
    return os.environ.get("LUMEN_DEBUG", "0") not in ("", "0")


def apply_debug_env() -> None:
    """Call before any HIP runtime use (done by ``dist.init``)."""
    if debug_enabled():
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")


class NonFiniteError(FloatingPointError):
    pass


def check_finite(name: str, t: Optional[torch.Tensor], step: int = -1, rank: int = 0,
                 force: bool = False) -> None:
    """Raise ``NonFiniteError`` if ``t`` holds NaN/Inf (only in debug mode unless ``force``)."""
    if t is None or not (force or debug_enabled()):
        return
    if not bool(torch.isfinite(t.detach()).all()):
        bad = t.detach().float()
        raise NonFiniteError(f"[lumen debug] rank {rank} step {step}: non-finite values in {name} "
                             f"(nan={int(torch.isnan(bad).sum())}, inf={int(torch.isinf(bad).sum())})")


@contextlib.contextmanager
def trace_range(name: str):
    """Named range: torch.profiler annotation + roctx push/pop on GPU builds."""
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds
            pushed = True
        except Exception:  # noqa: BLE001 - markers are best-effort
            pushed = False
    with torch.autograd.profiler.record_function(name):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


class StepProfiler:
    """``LUMEN_PROFILE``-gated torch.profiler driven by optimizer steps."""

    def __init__(self, rank: int = 0, printer=print):
        self.enabled = os.environ.get("LUMEN_PROFILE", "0") not in ("", "0")
        self.rank = rank
        self.print = printer
        self.prof = None
        if not self.enabled:
            return
        from torch.profiler import ProfilerActivity, profile, schedule

        wait = int(os.environ.get("LUMEN_PROFILE_WAIT", "2"))
        active = int(os.environ.get("LUMEN_PROFILE_ACTIVE", "3"))
        self.out_dir = os.environ.get("LUMEN_PROFILE_DIR", os.path.join("profiles", "torch"))
        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)
        self.prof = profile(activities=acts, schedule=schedule(wait=wait, warmup=1, active=active,
                                                                repeat=1),
                            on_trace_ready=self._ready, record_shapes=False, with_stack=False)
        self.prof.__enter__()

    def _ready(self, p):
        os.makedirs(self.out_dir, exist_ok=True)
        path = os.path.join(self.out_dir, f"trace_rank{self.rank}.json")
        p.export_chrome_trace(path)
        if self.rank == 0:
            key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
            try:
                self.print(p.key_averages().table(sort_by=key, row_limit=25))
            except Exception:  # noqa: BLE001
                pass
            self.print(f"[lumen] profiler trace written to {path}")

    def step(self):
        if self.prof is not None:
            self.prof.step()

    def close(self):
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            self.prof = None


def maybe_inject_fault(step: int, rank: int) -> None:
    """Exit hard (no cleanup, like a crashed rank) when ``LUMEN_FAULT_STEP`` says so."""
    k = os.environ.get("LUMEN_FAULT_STEP")
    if not k or int(k) != step:
        return
    ranks = {int(r) for r in os.environ.get("LUMEN_FAULT_RANK", "0").split(",") if r.strip()}
    if rank in ranks:
        print(f"[lumen fault] rank {rank} exiting at step {step}", flush=True)
        os._exit(FAULT_EXIT_CODE)


HANG_EXIT_CODE = 19


class StepWatchdog:
    """Host-side progress watchdog: ends the process (exit code 19) when no ``kick()`` arrives
    within ``timeout_s`` -- a hung collective must end a multi-rank job with a message that
    names the escape hatch, not eat the job's time budget.  It fires before the RCCL watchdog
    (``LUMEN_DIST_TIMEOUT``), prints what the ZeRO-3 coordinator had in flight, and exits with
    ``os._exit`` (no re-exec, no cleanup that could block on the hung device)."""

    def __init__(self, timeout_s: float, rank: int = 0, coordinator=None, what: str = "step"):
        import threading
        import time

        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.coordinator = coordinator
        self.what = what
        self._time = time
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="lumen-watchdog", daemon=True)
            self._thread.start()

    @classmethod
    def from_env(cls, rank: int = 0, coordinator=None, what: str = "step"):
        """Timeout from ``LUMEN_WATCHDOG_S``, else 60 s under ``LUMEN_DIST_TIMEOUT`` (0: off)."""
        v = os.environ.get("LUMEN_WATCHDOG_S")
        if v is None:
            d = float(os.environ.get("LUMEN_DIST_TIMEOUT", "1800"))
            v = max(60.0, d - 60.0)
        return cls(float(v), rank, coordinator, what)

    def kick(self) -> None:
        self._last = self._time.monotonic()

    def message(self, waited: float) -> str:
        msg = (f"[lumen watchdog] rank {self.rank}: no {self.what} completed in {waited:.0f} s "
               f"(limit {self.timeout_s:.0f} s); a collective or kernel is hung.")
        c = self.coordinator
        if c is not None and not getattr(c, "identity", True):
            inflight = sum(u.state == "inflight" for u in c.units)
            msg += (f" ZeRO-3 schedule '{c.schedule}', {inflight} weight gather(s) in flight on "
                    f"{'a separate' if c.group is not None else 'the default'} communicator.")
            if c.group is not None:
                msg += (" If concurrent communicators hang on this system, rerun with "
                        "LUMEN_ZERO3_SHARED_GROUP=1 (weight gathers on the default group).")
        return msg

    def _run(self):
        import sys

        while not self._stop.wait(min(5.0, self.timeout_s / 4)):
            waited = self._time.monotonic() - self._last
            if waited > self.timeout_s:
                sys.stderr.write(self.message(waited) + "\n")
                sys.stderr.flush()
                os._exit(HANG_EXIT_CODE)

    def close(self) -> None:
        self._stop.set()


def zero3_poison_enabled() -> bool:
    return debug_enabled() or os.environ.get("LUMEN_ZERO3_POISON", "0") not in ("", "0")
