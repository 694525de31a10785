"""Rank-side fault-tolerance helpers.

Heartbeat          daemon thread that stamps <dir>/hb_<rank> every `interval` s with JSON
                   {t, step, state}: ``step`` is the last iteration the TRAINING LOOP completed
                   (``progress()``), ``state`` is "run", "comm" (blocked in a collective / on a
                   collective's result, see ps.comm.Comm.waiting) or "recover" (rolling back).
                   The supervisor (minips_amd.elastic) declares a rank failed when the stamp is
                   older than 3 x interval (master/heartbeat_check_thread.cpp:29: the process is
                   gone or frozen) OR when its step has not advanced for the progress timeout
                   while it is not waiting on a peer (it is stuck inside a step: a hung kernel,
                   a deadlock, a sleep), so a live thread can no longer mask a hung rank.
FaultInjector      --fail_rank/--fail_step: that rank fails when it reaches the step, on the first
                   attempt only -- --fail_mode=exit: the process dies (os._exit; detected from the
                   exit status); --fail_mode=hang: it stops heartbeating and stalls (a machine that
                   stops answering); --fail_mode=hang_in_step: it blocks INSIDE the step with the
                   heartbeat thread untouched (detected by the progress check only);
                   --with_injected_straggler: a 5% chance per step of sleeping U(0, 100) ms
                   (lr_example.cpp:347-353).
"""
from __future__ import annotations

import json
import os
import random
import threading
import time


class Heartbeat:
    def __init__(self, directory: str, rank: int, interval: float, state_fn=None):
        self.path = os.path.join(directory, f"hb_{rank}")
        self.interval = interval
        self.step = -1
        self.state = "run"
        self.state_fn = state_fn  # optional: returns "comm" while the rank waits on its peers
        os.makedirs(directory, exist_ok=True)
        self._stop = threading.Event()
        self._beat()
        self._th = threading.Thread(target=self._loop, name="minips-heartbeat", daemon=True)
        self._th.start()

    def write_caps(self, **caps):
        """Recovery capabilities of this rank (<dir>/caps_<rank>.json), read by the supervisor."""
        d = os.path.dirname(self.path)
        r = os.path.basename(self.path)[3:]
        tmp = os.path.join(d, f"caps_{r}.json.tmp")
        with open(tmp, "w") as f:
            json.dump(caps, f)
        os.replace(tmp, os.path.join(d, f"caps_{r}.json"))

    def progress(self, step: int):
        """Called by the training loop after each completed iteration (and at long phases:
        start-up, restore, checkpoint), so the stamp carries real progress."""
        self.step = int(step)

    def _beat(self):
        state = self.state
        if state == "run" and self.state_fn is not None:
            state = self.state_fn() or "run"
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            f.write(json.dumps({"t": round(time.time(), 3), "step": self.step, "state": state}))
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


def read_heartbeat(path: str):
    """-> (mtime-free stamp time, step, state) of a heartbeat file, or None."""
    try:
        d = json.loads(open(path).read())
        return float(d["t"]), int(d.get("step", -1)), str(d.get("state", "run"))
    except (OSError, ValueError, KeyError):
        return None


class FaultInjector:
    def __init__(self, rank: int, fail_rank: int = -1, fail_step: int = -1, straggler: bool = False,
                 seed: int = 0, mode: str = "exit", heartbeat: Heartbeat | None = None):
        self.rank = rank
        self.mode, self.heartbeat = mode, heartbeat
        self.fail_rank, self.fail_step = fail_rank, fail_step
        self.straggler = straggler
        self.first_attempt = int(os.environ.get("MINIPS_RESTART_COUNT", "0")) == 0 and \
            int(os.environ.get("MINIPS_GENERATION", "0")) == 0
        self.rng = random.Random(seed * 7919 + rank)

    def _hit(self, step: int) -> bool:
        return self.first_attempt and self.rank == self.fail_rank and step == self.fail_step

    def step(self, step: int):
        """Called at the top of an iteration (exit / hang / straggler)."""
        if self._hit(step) and self.mode in ("exit", "hang"):
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

    def in_step(self, step: int):
        """Called INSIDE the step (between the Get and the Clock): hang_in_step blocks here while
        the heartbeat thread keeps stamping."""
        if self._hit(step) and self.mode == "hang_in_step":
            print(f"[fault injection][{int(time.time() * 1000)}] rank {self.rank} hangs inside step {step}",
                  flush=True)
            while True:
                time.sleep(3600)


def slow_io_delay(rank: int):
    """Fault injection for long-phase tests: MINIPS_FAULT_SLOW_IO="<rank>:<seconds>" makes each
    checkpoint write and restore of that rank take that much longer (a slow disk / network FS)."""
    spec = os.environ.get("MINIPS_FAULT_SLOW_IO", "")
    if not spec:
        return
    r, secs = spec.split(":")
    if int(r) == rank:
        time.sleep(float(secs))


def slow_pause_delay(rank: int):
    """Fault injection: MINIPS_FAULT_SLOW_PAUSE="<rank>:<seconds>" delays that rank between the
    checkpoint's clock all-gather and the pause of its asynchronous servers (the window in which a
    fast peer could otherwise resume and push into a not-yet-paused owner)."""
    spec = os.environ.get("MINIPS_FAULT_SLOW_PAUSE", "")
    if not spec:
        return
    r, secs = spec.split(":")
    if int(r) == rank:
        time.sleep(float(secs))
