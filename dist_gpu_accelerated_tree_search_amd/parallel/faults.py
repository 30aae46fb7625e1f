"""Fault-injection settings of the multi-process runtime.

The injection itself runs in the native round loop (csrc/core/dist_rounds.hpp) and in
the single-process runner (csrc/core/runner.hpp), with the same semantics:

    TTS_FAULT_DELAY_US=<us>        random delay in [0, us] before each round (per rank)
    TTS_FAULT_STEAL_FAIL_PCT=<pct> planned transfers dropped with this probability; the
                                   draw is seeded by the round number, so every rank
                                   drops the same ones (the plan stays consistent)
    TTS_FAULT_SEED=<int>

Failure detection (stuck-phase watchdogs, TTS_WATCHDOG_S / TTS_WATCHDOG_ABORT; a peer
that misses a shared-memory round within the timeout raises) is native as well; this
module only resolves the settings from DistConfig and the environment.
"""
from __future__ import annotations

import os


class Faults:
    def __init__(self, rank: int, delay_us: int | None = None, steal_fail_pct: int | None = None,
                 seed: int | None = None):
        env = os.environ.get
        self.rank = rank
        self.delay_us = int(env("TTS_FAULT_DELAY_US", "0") or 0) if delay_us is None else int(delay_us)
        self.steal_fail_pct = (int(env("TTS_FAULT_STEAL_FAIL_PCT", "0") or 0) if steal_fail_pct is None
                               else int(steal_fail_pct))
        self.seed = int(env("TTS_FAULT_SEED", "12345") or 12345) if seed is None else int(seed)

    @property
    def active(self) -> bool:
        return bool(self.delay_us or self.steal_fail_pct)
