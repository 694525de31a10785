"""Supervisor of a PS job: one process per rank, heartbeat failure detection, restart from the
last checkpoint (reference master/heartbeat_check_thread.cpp + the launcher's
relaunch verb).

    python -m minips_amd.elastic --nproc 8 --heartbeat_interval 2 --max_restarts 3 -- \
        python -m minips_amd.train --model widedeep --checkpoint_toggle=1 --checkpoint_every 50

Policy (the reference's, adapted to RCCL):
  * every rank stamps <run_dir>/hb_<rank> each `heartbeat_interval` s (minips_amd.ps.fault);
  * a rank whose process exited non-zero, or whose stamp is older than 3 x interval, is failed
    -> "[Fault Tolerance][Phase2]" (detect);
  * an RCCL communicator cannot outlive a member, so the survivors are stopped too (their
    process groups are signalled -- this supervisor's own children only) and the whole rank
    set is relaunched with --use_weight_file=1 on the SAME GPUs (LOCAL_RANK = rank) and a fresh
    rendezvous port -> "[Phase3]" (restart); each rank restores its shards from the checkpoint
    and logs "[Phase4]" (the failed rank) or "[Phase5]" (the others).
  * at most one recovery at a time; after `max_restarts` recoveries the job fails.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

from .utils.metrics import fault_tolerance_phase


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Supervisor:
    def __init__(self, cmd: list[str], nproc: int, heartbeat_interval: float = 1.0, max_restarts: int = 3,
                 run_dir: str | None = None, log_dir: str | None = None, startup_grace: float = 120.0):
        self.cmd = cmd
        self.nproc = nproc
        self.interval = heartbeat_interval
        self.max_restarts = max_restarts
        self.run_dir = run_dir or tempfile.mkdtemp(prefix="minips_run_")
        self.log_dir = log_dir
        self.startup_grace = startup_grace
        self.restarts = 0
        self.procs: list[subprocess.Popen] = []
        self.failed_rank = -1

    def _spawn(self, resume: bool):
        port = _free_port()
        hb = os.path.join(self.run_dir, f"attempt{self.restarts}")
        os.makedirs(hb, exist_ok=True)
        self.hb_dir = hb
        self.procs = []
        for r in range(self.nproc):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(self.nproc),
                       LOCAL_WORLD_SIZE=str(self.nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       MINIPS_RESTART_COUNT=str(self.restarts), MINIPS_FAILED_RANK=str(self.failed_rank))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            extra = [f"--heartbeat_dir={hb}", f"--heartbeat_interval={self.interval}"]
            if resume:
                extra.append("--use_weight_file=1")
            out = None
            if self.log_dir:
                os.makedirs(self.log_dir, exist_ok=True)
                out = open(os.path.join(self.log_dir, f"rank{r}_attempt{self.restarts}.log"), "w")
            self.procs.append(subprocess.Popen(self.cmd + extra, env=env, stdout=out, stderr=subprocess.STDOUT
                                               if out else None, start_new_session=True))
        self.t_start = time.time()

    def _stop_all(self):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in self.procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def _check(self):
        """-> ("running" | "done" | "failed", rank)."""
        all_done = True
        for r, p in enumerate(self.procs):
            rc = p.poll()
            if rc is None:
                all_done = False
                path = os.path.join(self.hb_dir, f"hb_{r}")
                if self.interval > 0 and os.path.exists(path):
                    age = time.time() - os.path.getmtime(path)
                    if age > 3 * self.interval and not os.path.exists(path + ".quit"):
                        return "failed", r
                elif self.interval > 0 and time.time() - self.t_start > self.startup_grace:
                    return "failed", r
            elif rc != 0:
                return "failed", r
        return ("done", -1) if all_done else ("running", -1)

    def run(self) -> int:
        self._spawn(resume=False)
        while True:
            time.sleep(min(0.2, self.interval / 4) if self.interval > 0 else 0.2)
            state, rank = self._check()
            if state == "done":
                return 0
            if state == "running":
                continue
            fault_tolerance_phase(2, f"rank {rank} failed (attempt {self.restarts})")
            self._stop_all()
            if self.restarts >= self.max_restarts:
                print(f"[elastic] giving up after {self.restarts} restarts", file=sys.stderr, flush=True)
                return 1
            self.restarts += 1
            self.failed_rank = rank
            fault_tolerance_phase(3, f"relaunch {self.nproc} ranks from the last checkpoint")
            self._spawn(resume=True)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        raise SystemExit("usage: python -m minips_amd.elastic [options] -- <rank command>")
    i = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--heartbeat_interval", type=float, default=1.0)
    ap.add_argument("--max_restarts", type=int, default=3)
    ap.add_argument("--run_dir", default=None)
    ap.add_argument("--log_dir", default=None)
    a = ap.parse_args(argv[:i])
    sup = Supervisor(argv[i + 1:], a.nproc, a.heartbeat_interval, a.max_restarts, a.run_dir, a.log_dir)
    return sup.run()


if __name__ == "__main__":
    sys.exit(main())
