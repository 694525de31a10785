"""Rank-side fault-tolerance helpers.

Heartbeat          daemon thread that stamps <dir>/hb_<rank> every `interval` s; the supervisor
                   (minips_amd.elastic) declares a rank failed when its stamp is older than
                   3 x interval (master/heartbeat_check_thread.cpp:29) or the process exited.
FaultInjector      --fail_rank/--fail_step: that rank fails when it reaches the step, on the first
                   attempt only -- --fail_mode=exit: the process dies (os._exit; detected from the
                   exit status); --fail_mode=hang: it stops heartbeating and stalls, like a machine
                   that stops answering (detected only by the 3 x interval heartbeat timeout, the
                   reference's only detector); --with_injected_straggler: a 5% chance per step of
                   sleeping U(0, 100) ms (lr_example.cpp:347-353).
"""
from __future__ import annotations

import os
import random
import threading
import time


class Heartbeat:
    def __init__(self, directory: str, rank: int, interval: float):
        self.path = os.path.join(directory, f"hb_{rank}")
        self.interval = interval
        os.makedirs(directory, exist_ok=True)
        self._stop = threading.Event()
        self._beat()
        self._th = threading.Thread(target=self._loop, name="minips-heartbeat", daemon=True)
        self._th.start()

    def _beat(self):
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            f.write(f"{time.time():.3f}")
        os.replace(tmp, self.path)

    def _loop(self):
        while not self._stop.wait(self.interval):
            self._beat()

    def stop(self, quit_: bool = True):
        """kQuitHeartBeat: mark a clean exit so the supervisor does not treat silence as failure."""
        self._stop.set()
        self._th.join(timeout=5)
        if quit_:
            with open(self.path + ".quit", "w") as f:
                f.write(f"{time.time():.3f}")


class FaultInjector:
    def __init__(self, rank: int, fail_rank: int = -1, fail_step: int = -1, straggler: bool = False,
                 seed: int = 0, mode: str = "exit", heartbeat: Heartbeat | None = None):
        self.rank = rank
        self.mode, self.heartbeat = mode, heartbeat
        self.fail_rank, self.fail_step = fail_rank, fail_step
        self.straggler = straggler
        self.first_attempt = int(os.environ.get("MINIPS_RESTART_COUNT", "0")) == 0
        self.rng = random.Random(seed * 7919 + rank)

    def step(self, step: int):
        if self.first_attempt and self.rank == self.fail_rank and step == self.fail_step:
            print(f"[fault injection][{int(time.time() * 1000)}] rank {self.rank} {self.mode} at step {step}",
                  flush=True)
            if self.mode == "hang":
                if self.heartbeat is not None:
                    self.heartbeat.stop(quit_=False)  # silence, no clean-exit marker
                while True:
                    time.sleep(3600)
            os._exit(17)
        if self.straggler and self.rng.random() < 0.05:
            time.sleep(self.rng.uniform(0.0, 0.1))
