"""One overall wall deadline for bench.py's optional sections (VERDICT r5 "Next" #7).

After the timed headline region bench.py runs optional sections: the transport probe, the two
partitioned ZeRO-3 schedules, the TP = 1 serving bench (N = 1) or TP = N serving (N > 1).  On a
first 8-GPU node their costs are unknown, and the driver kills the whole run at its timeout
(600 s in every record so far) -- which would lose the headline line too.  ``WallBudget``
counts every section against one deadline measured from process start, skips a section whose
estimate does not fit in what is left (and says so in the record), and makes every rank take the
same decision (the remaining time is agreed as the minimum over ranks), because the sections
are collective.  Reference: training/train.ipynb:806 -- the reference's only multi-GPU run
crashed before producing a number; ours must always print one.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional


class WallBudget:
    def __init__(self, total_s: float, t0: float, agree_min: Optional[Callable[[float], float]] = None,
                 clock: Callable[[], float] = time.time):
        self.total_s = float(total_s)
        self.t0 = t0
        self.clock = clock
        self.agree_min = agree_min
        self.ran: List[Dict] = []
        self.skipped: List[Dict] = []
        self._open: Optional[Dict] = None

    def left(self) -> float:
        """Seconds left, the same value on every rank (min over ranks when ``agree_min``)."""
        x = self.total_s - (self.clock() - self.t0)
        return float(self.agree_min(x)) if self.agree_min is not None else x

    def allow(self, name: str, est_s: float) -> bool:
        """Run section ``name`` (estimated ``est_s``) only if it fits in what is left.  Collective
        when ``agree_min`` is set: every rank must call it at the same point."""
        left = self.left()
        if est_s > left:
            self.skipped.append({"section": name, "est_s": round(est_s, 1),
                                 "left_s": round(left, 1)})
            return False
        self._open = {"section": name, "est_s": round(est_s, 1), "left_s": round(left, 1),
                      "t": self.clock()}
        return True

    def done(self, name: str) -> None:
        o = self._open
        if o is not None and o["section"] == name:
            o["took_s"] = round(self.clock() - o.pop("t"), 1)
            self.ran.append(o)
            self._open = None

    def record(self) -> Dict:
        return {"wall_budget_s": self.total_s,
                "left_at_record_s": round(self.total_s - (self.clock() - self.t0), 1),
                "ran": list(self.ran), "skipped": list(self.skipped)}


def partitioned_estimate_s(ms_per_step: float, steps: int, warmup: int, build_s: float,
                           slowdown: float = 1.5) -> float:
    """A partitioned run: a fresh model + engine, then (warmup + steps) steps that re-gather
    weights (``slowdown`` x the headline step), plus teardown."""
    return 10.0 + 2.0 * build_s + (steps + warmup) * ms_per_step / 1000.0 * slowdown
