"""Failure detection and fault injection for the multi-process runtime.

* Watchdog: before every coordination round, `faulthandler.dump_traceback_later`
  is armed with `watchdog_s`; a round that does not complete in time (a peer that
  died or hangs inside a collective, a stuck device) dumps every thread's stack
  plus this rank's state to stderr, and aborts the process when asked to.
* Fault injection (environment, identical semantics to the native runner):
    TTS_FAULT_DELAY_US=<us>        random delay in [0, us] before each round (per rank)
    TTS_FAULT_STEAL_FAIL_PCT=<pct> planned transfers dropped with this probability;
                                   the draw is seeded by the round number, so every
                                   rank drops the same ones (the plan stays consistent)
    TTS_FAULT_SEED=<int>
"""
from __future__ import annotations

import faulthandler
import os
import random
import sys
import time


class Faults:
    def __init__(self, rank: int, delay_us: int | None = None, steal_fail_pct: int | None = None,
                 seed: int | None = None):
        env = os.environ.get
        self.delay_us = int(env("TTS_FAULT_DELAY_US", "0") or 0) if delay_us is None else int(delay_us)
        self.steal_fail_pct = (int(env("TTS_FAULT_STEAL_FAIL_PCT", "0") or 0) if steal_fail_pct is None
                               else int(steal_fail_pct))
        self.seed = int(env("TTS_FAULT_SEED", "12345") or 12345) if seed is None else int(seed)
        self._rank = rank
        self._rng = None  # created on first use (a Random costs ~10 us; the runtime builds Faults per solve)
        self.dropped = 0

    @property
    def active(self) -> bool:
        return bool(self.delay_us or self.steal_fail_pct)

    def before_round(self) -> None:
        if self.delay_us:
            if self._rng is None:
                self._rng = random.Random(self.seed * 7919 + self._rank)
            time.sleep(self._rng.randint(0, self.delay_us) * 1e-6)

    def filter_plan(self, plan, round_no: int):
        if not self.steal_fail_pct or not plan:
            return plan
        rng = random.Random(self.seed * 1_000_003 + round_no)  # same draw on every rank
        kept = []
        for t in plan:
            if rng.randrange(100) < self.steal_fail_pct:
                self.dropped += 1
            else:
                kept.append(t)
        return kept


class Watchdog:
    """Watches each coordination round. On timeout: a state line for this rank
    (best effort, from a timer thread) and the stacks of every thread (from
    faulthandler's C thread, which works even if the GIL is stuck); with
    abort=True (or TTS_WATCHDOG_ABORT=1) the process then aborts."""

    def __init__(self, timeout_s: float = 0.0, abort: bool = False):
        self.timeout_s = float(timeout_s or float(os.environ.get("TTS_WATCHDOG_S", "0") or 0))
        self.abort = abort or os.environ.get("TTS_WATCHDOG_ABORT", "0") not in ("", "0")
        self.events = 0
        self._timer = None

    @property
    def enabled(self) -> bool:
        return self.timeout_s > 0

    def arm(self, state: str) -> None:
        if self.timeout_s <= 0:
            return
        import threading

        def fire():
            self.events += 1
            sys.stderr.write(f"[tts watchdog] round exceeded {self.timeout_s:.3f} s: {state}\n")
            sys.stderr.flush()

        self._timer = threading.Timer(self.timeout_s, fire)
        self._timer.daemon = True
        self._timer.start()
        faulthandler.dump_traceback_later(self.timeout_s * 1.5, repeat=False, file=sys.stderr, exit=self.abort)

    def disarm(self) -> None:
        if self.timeout_s <= 0:
            return
        faulthandler.cancel_dump_traceback_later()
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
