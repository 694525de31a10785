"""Supervisor of a PS job: one process per rank, heartbeat + progress failure detection, recovery
from the last checkpoint (reference master/heartbeat_check_thread.cpp, the
master's kRollBack broadcast and the launcher's relaunch verb).

    python -m minips_amd.elastic --nproc 8 --heartbeat_interval 2 --max_restarts 3 -- \\
        python -m minips_amd.train --model widedeep --checkpoint_toggle=1 --checkpoint_every 50

Detection (the reference's rule, plus progress):
  * a rank whose process exited non-zero is failed;
  * a rank whose heartbeat stamp is older than 3 x interval is failed (process gone or frozen:
    heartbeat_check_thread.cpp:29);
  * a rank whose completed-step counter has not advanced for ``progress_timeout`` (default
    3 x interval) while it is NOT waiting on a peer is failed: it is stuck inside a step (a hung
    kernel, a deadlock, an injected sleep) although its heartbeat thread still stamps. When every
    stalled rank is waiting on peers the culprit is ambiguous and the lowest stalled rank is
    blamed (the whole rank set is then restarted).
  -> "[Fault Tolerance][Phase2]" (detect).
Recovery (at most one at a time; after ``max_restarts`` recoveries the job fails):
  * inplace (default): only the failed rank is killed and relaunched (--use_weight_file=1, same
    GPU); the survivors, whose collectives failed, roll back in their own processes: they read
    the rollback directive (a new generation + rendezvous port) this supervisor writes to
    <run_dir>/attempt<k>/rollback.json (the reference's kRollBack broadcast), re-form the group
    with the relaunched rank and restore the last committed checkpoint -> "[Phase3]" restart of
    the failed rank, "[Phase4]" its restore, "[Phase5]" the survivors' in-place rollback.
  * restart: every rank is stopped and the whole set relaunched on a fresh rendezvous (also the
    fallback when the culprit is ambiguous or a survivor dies during an in-place recovery).
A rank that exits 0 (finished, or kForceQuit for lack of data) is done, not failed.

Live scale-out / scale-in (the reference's kScaleRollback, comm/mailbox.cpp:197-219, and
Engine::UpdateAndRestart, driver/engine.cpp:96-112):

    python -m minips_amd.elastic scale --run_dir <run_dir> --world M

asks the running job to change its rank count to M. The supervisor writes a "scale" directive
(new generation, rendezvous port, world M) next to the heartbeats and, for M > N, starts ranks
N..M-1 with --use_weight_file=1. The running ranks agree on the iteration at which they saw it
(a max all-reduce every --scale_check_every steps), save and commit a checkpoint there, leave the
old group, and -- without leaving their processes -- ranks < M re-form the group at world M,
rebuild their tables on the new shard ranges and restore that checkpoint (any N -> M reshard);
ranks >= M retire (exit 0). The new ranks restore the same checkpoint and the job continues.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

from .ps.fault import read_heartbeat
from .utils.metrics import fault_tolerance_phase


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Supervisor:
    def __init__(self, cmd: list[str], nproc: int, heartbeat_interval: float = 1.0, max_restarts: int = 3,
                 run_dir: str | None = None, log_dir: str | None = None, startup_grace: float = 120.0,
                 recovery: str = "inplace", progress_timeout: float | None = None):
        self.cmd = cmd
        self.nproc = nproc
        self.interval = heartbeat_interval
        self.max_restarts = max_restarts
        self.run_dir = run_dir or tempfile.mkdtemp(prefix="minips_run_")
        self.log_dir = log_dir
        self.startup_grace = startup_grace
        self.recovery = recovery
        self.progress_timeout = progress_timeout if progress_timeout is not None else 3 * heartbeat_interval
        self.ckpt_timeout = float(os.environ.get("MINIPS_CKPT_TIMEOUT", "3600"))
        self.restarts = 0
        self.generation = 0
        self.procs: list[subprocess.Popen | None] = [None] * nproc
        self.failed_rank = -1
        self.port = 0
        self.retired: set[int] = set()  # ranks >= the world of a scale-in (they exit by themselves)
        self._last_state: dict[int, str] = {}
        self.scales = 0

    # ------------------------------------------------------------------------------ spawning
    def _env(self, r: int) -> dict:
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(self.nproc),
                   LOCAL_WORLD_SIZE=str(self.nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.port),
                   MINIPS_RESTART_COUNT=str(self.restarts), MINIPS_FAILED_RANK=str(self.failed_rank),
                   MINIPS_GENERATION=str(self.generation))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return env

    def _spawn_rank(self, r: int, resume: bool):
        # the previous process's stamp -- and its recovery capabilities, possibly left by an earlier
        # run in the same directory -- must not count for this one
        for name in (f"hb_{r}", f"hb_{r}.quit", f"caps_{r}.json"):
            try:
                os.remove(os.path.join(self.hb_dir, name))
            except FileNotFoundError:
                pass
        self.t_spawn[r] = time.time()
        extra = [f"--heartbeat_dir={self.hb_dir}", f"--heartbeat_interval={self.interval}",
                 f"--recovery={self.recovery}"]
        if resume:
            extra.append("--use_weight_file=1")
        out = None
        if self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            out = open(os.path.join(self.log_dir, f"rank{r}_attempt{self.restarts}.log"), "a")
        self.procs[r] = subprocess.Popen(self.cmd + extra, env=self._env(r), stdout=out,
                                         stderr=subprocess.STDOUT if out else None, start_new_session=True)
        self._reset_progress(r)

    def _spawn_all(self, resume: bool):
        self.port = _free_port()
        self.hb_dir = os.path.join(self.run_dir, f"attempt{self.restarts}")
        os.makedirs(self.hb_dir, exist_ok=True)
        self.t_start = time.time()
        self.progress = {}
        self.t_spawn = {}
        for r in range(self.nproc):
            self._spawn_rank(r, resume)

    def _reset_progress(self, r: int):
        self.progress[r] = (None, time.time())  # (last seen step, time it last changed)

    @staticmethod
    def _kill(p: subprocess.Popen | None, sig=signal.SIGTERM):
        if p is not None and p.poll() is None:
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                pass

    def _stop(self, ranks):
        for r in ranks:
            self._kill(self.procs[r])
        deadline = time.time() + 10
        for r in ranks:
            p = self.procs[r]
            if p is None:
                continue
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                self._kill(p, signal.SIGKILL)
                p.wait()

    # ------------------------------------------------------------------------------ detection
    def _check(self):
        """-> (state, rank, reason, clear): state "running" | "done" | "failed"; ``clear`` tells
        whether the failed rank is unambiguously the culprit."""
        now = time.time()
        all_done, stalled = True, []
        for r, p in enumerate(self.procs):
            if r in self.retired:
                continue
            rc = p.poll()
            if rc is not None:
                if rc != 0:
                    return "failed", r, f"exit status {rc}", True
                continue
            all_done = False
            if self.interval <= 0:
                continue
            path = os.path.join(self.hb_dir, f"hb_{r}")
            hb = read_heartbeat(path)
            if hb is None:
                if now - self.t_spawn.get(r, self.t_start) > self.startup_grace:
                    return "failed", r, "no heartbeat", True
                continue
            t, step, state = hb
            if now - t > 3 * self.interval and not os.path.exists(path + ".quit"):
                return "failed", r, f"heartbeat silent for {now - t:.1f} s", True
            last, since = self.progress.get(r, (None, now))
            if step != last or state == "recover":
                self.progress[r] = (step, now)
                self._last_state[r] = state
                continue
            if self._last_state.get(r) == "ckpt" and state != "ckpt":
                # a checkpoint phase just ended: its (long-limit) time does not count against the
                # step that follows it
                self.progress[r] = (step, now)
                since = now
            self._last_state[r] = state
            # a checkpoint write / commit advances no step: it gets its own, longer limit
            limit = self.startup_grace if step < 0 else (self.ckpt_timeout if state == "ckpt"
                                                         else self.progress_timeout)
            if now - since > limit:
                stalled.append((r, state, step))
        if all_done:
            return "done", -1, "", True
        if stalled:
            computing = [r for r, st, _ in stalled if st != "comm"]
            if computing:
                r = computing[0]
                return "failed", r, f"no progress past step {self.progress[r][0]} for " \
                                    f"{now - self.progress[r][1]:.1f} s (stuck inside a step)", len(computing) == 1
            # everyone that stalled waits on peers: wait until every live rank has stalled
            live = [r for r, p in enumerate(self.procs) if p.poll() is None and r not in self.retired]
            if len(stalled) == len(live):
                r = min(s[0] for s in stalled)
                return "failed", r, "every rank waits on its peers (culprit ambiguous)", False
        return "running", -1, "", True

    # ------------------------------------------------------------------------------ recovery
    def _inplace_capable(self) -> bool:
        """Every rank said it can roll back in its own process (caps_<r>.json, written after its
        tables exist). A rank of the one-sided transport cannot: its peers hold IPC mappings of its
        shards and inboxes and a shared progress board, so only a whole-set restart is valid."""
        for r in range(self.nproc):
            try:
                caps = json.loads(open(os.path.join(self.hb_dir, f"caps_{r}.json")).read())
            except (OSError, ValueError):
                continue  # not written yet (start-up): the exit-status / heartbeat rules decide
            if not caps.get("inplace", True):
                return False
        return True

    def _recover_inplace(self, rank: int) -> bool:
        """Relaunch only ``rank``; the survivors roll back in place. False: not possible."""
        survivors = [r for r, p in enumerate(self.procs[:self.nproc]) if r != rank and p.poll() is None]
        if not survivors or len(survivors) != self.nproc - 1:
            return False
        if not self._inplace_capable():
            fault_tolerance_phase(3, "a rank cannot roll back in place (one-sided tables): whole-set restart")
            return False
        self._stop([rank])
        self.restarts += 1
        self.generation += 1
        self.failed_rank = rank
        self.port = _free_port()
        fault_tolerance_phase(3, f"relaunch rank {rank} (generation {self.generation}); "
                                 f"{len(survivors)} survivors roll back in place")
        tmp = os.path.join(self.hb_dir, "rollback.json.tmp")
        with open(tmp, "w") as f:
            json.dump(dict(generation=self.generation, port=self.port, failed_rank=rank, world=self.nproc), f)
        os.replace(tmp, os.path.join(self.hb_dir, "rollback.json"))
        self._spawn_rank(rank, resume=True)
        for r in survivors:
            self._reset_progress(r)
        return True

    # ------------------------------------------------------------------------------ scaling
    def _poll_scale(self):
        """A pending ``scale`` request (<run_dir>/scale.json, written by ``elastic scale``)."""
        path = os.path.join(self.run_dir, "scale.json")
        try:
            req = json.loads(open(path).read())
        except (OSError, ValueError):
            return
        os.replace(path, os.path.join(self.run_dir, f"scale.{self.scales}.done.json"))
        new = int(req.get("world", self.nproc))
        if new < 1 or new == self.nproc:
            return
        old = self.nproc
        self.scales += 1
        self.generation += 1
        self.port = _free_port()
        self.failed_rank = -1
        fault_tolerance_phase(3, f"scale {old} -> {new} ranks (generation {self.generation}): the running ranks "
                                 f"checkpoint, re-form the group in place and reshard")
        tmp = os.path.join(self.hb_dir, "rollback.json.tmp")
        with open(tmp, "w") as f:
            json.dump(dict(generation=self.generation, port=self.port, world=new, kind="scale", failed_rank=-1), f)
        os.replace(tmp, os.path.join(self.hb_dir, "rollback.json"))
        self.nproc = new
        for r in range(min(old, new)):
            self._reset_progress(r)
        if new > old:
            self.procs.extend([None] * (new - len(self.procs)))
            for r in range(old, new):
                self.retired.discard(r)
                self._spawn_rank(r, resume=True)
        else:
            self.retired.update(range(new, old))

    def run(self) -> int:
        self._spawn_all(resume=False)
        while True:
            time.sleep(min(0.2, self.interval / 4) if self.interval > 0 else 0.2)
            self._poll_scale()
            state, rank, reason, clear = self._check()
            if state == "done":
                return 0
            if state == "running":
                continue
            fault_tolerance_phase(2, f"rank {rank} failed (attempt {self.restarts}): {reason}")
            if self.restarts >= self.max_restarts:
                self._stop(range(len(self.procs)))
                print(f"[elastic] giving up after {self.restarts} restarts", file=sys.stderr, flush=True)
                return 1
            if self.recovery == "inplace" and clear and self._recover_inplace(rank):
                continue
            self._stop(range(len(self.procs)))
            self.restarts += 1
            self.generation += 1
            self.failed_rank = rank
            self.procs = self.procs[:self.nproc]
            self.retired.clear()
            fault_tolerance_phase(3, f"relaunch {self.nproc} ranks from the last checkpoint")
            self._spawn_all(resume=True)


def request_scale(run_dir: str, world: int):
    """Ask the supervisor of the job under ``run_dir`` to change the rank count to ``world``."""
    tmp = os.path.join(run_dir, "scale.json.tmp")
    with open(tmp, "w") as f:
        json.dump(dict(world=int(world), t=time.time()), f)
    os.replace(tmp, os.path.join(run_dir, "scale.json"))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "scale":
        ap = argparse.ArgumentParser(prog="python -m minips_amd.elastic scale")
        ap.add_argument("--run_dir", required=True)
        ap.add_argument("--world", type=int, required=True)
        a = ap.parse_args(argv[1:])
        request_scale(a.run_dir, a.world)
        return 0
    if "--" not in argv:
        raise SystemExit("usage: python -m minips_amd.elastic [options] -- <rank command>")
    i = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--heartbeat_interval", type=float, default=1.0)
    ap.add_argument("--progress_timeout", type=float, default=None,
                    help="seconds without a completed step before a rank counts as hung (default 3 x interval)")
    ap.add_argument("--max_restarts", type=int, default=3)
    ap.add_argument("--recovery", default="inplace", choices=["inplace", "restart"])
    ap.add_argument("--run_dir", default=None)
    ap.add_argument("--log_dir", default=None)
    a = ap.parse_args(argv[:i])
    sup = Supervisor(argv[i + 1:], a.nproc, a.heartbeat_interval, a.max_restarts, a.run_dir, a.log_dir,
                     recovery=a.recovery, progress_timeout=a.progress_timeout)
    return sup.run()


if __name__ == "__main__":
    sys.exit(main())
