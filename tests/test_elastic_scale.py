"""Live scale-out / scale-in of a running job under the elastic supervisor (the reference's
kScaleRollback, comm/mailbox.cpp:197-219; Engine::UpdateAndRestart, driver/engine.cpp:96-112):
gloo ranks on CPU. The running ranks checkpoint at the agreed iteration, re-form the group in their
own processes at the new world size and reshard; new ranks restore the same checkpoint; ranks past
the new world retire."""
import json
import os
import subprocess
import sys
import time

import pytest

from minips_amd.ps.fault import read_heartbeat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HB = 0.5


def _start(tmp, name, nproc, steps, train_extra=()):
    run_dir = tmp / f"run_{name}"
    cmd = [sys.executable, "-m", "minips_amd.elastic", "--nproc", str(nproc), "--heartbeat_interval", str(HB),
           "--max_restarts", "1", "--run_dir", str(run_dir), "--log_dir", str(tmp / f"log_{name}"), "--",
           sys.executable, "-m", "minips_amd.train", "--model=widedeep", "--small=1", "--steps", str(steps),
           "--scale_check_every", "5", f"--checkpoint_file_prefix={tmp}/ck_{name}/", *train_extra]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True), run_dir


def _wait_step(run_dir, rank, step, timeout=240):
    t0 = time.time()
    while time.time() - t0 < timeout:
        for d in sorted(run_dir.glob("attempt*")):
            hb = read_heartbeat(str(d / f"hb_{rank}"))
            if hb is not None and hb[1] >= step:
                return
        time.sleep(0.1)
    raise TimeoutError(f"rank {rank} never reached step {step}")


def _logs(tmp, name):
    d = tmp / f"log_{name}"
    return {f: open(d / f).read() for f in sorted(os.listdir(d))}


def _summary(logs):
    last = [l for k in sorted(logs) if k.startswith("rank0_") for l in logs[k].splitlines() if l.startswith("{")]
    return json.loads(last[-1])


ONESIDED = ("--transport=onesided", "--consistency=ssp", "--staleness=1")


@pytest.mark.parametrize("n0,n1,extra", [(2, 3, ()), (3, 2, ()), (2, 3, ONESIDED)],
                         ids=["2to3", "3to2", "2to3-onesided"])
def test_live_rescale(tmp_path, n0, n1, extra):
    """(the one-sided case: the old AsyncPS -- server thread, board, IPC maps -- is closed before
    the group is left, and the re-formed group, new rank included, builds a fresh one)"""
    steps = 400
    p, run_dir = _start(tmp_path, f"s{n0}{n1}", n0, steps, extra)
    try:
        _wait_step(run_dir, 0, 12)
        subprocess.run([sys.executable, "-m", "minips_amd.elastic", "scale", "--run_dir", str(run_dir),
                        "--world", str(n1)], cwd=ROOT, check=True, env=dict(os.environ, PYTHONPATH=ROOT))
        out, err = p.communicate(timeout=600)
    finally:
        if p.poll() is None:
            p.kill()
    logs = _logs(tmp_path, f"s{n0}{n1}")
    assert p.returncode == 0, (err[-3000:], {k: v[-2000:] for k, v in logs.items()})
    s = _summary(logs)
    assert s["world"] == n1 and s["generation"] == 1 and s["steps"] == steps, s
    assert s["start"] == 0  # rank 0 never left its process
    assert all(l == l and l < 10 for _, l in s["losses"]), s["losses"]
    # one process per rank for the whole run: the survivors were not relaunched
    assert sorted(k for k in logs if k.startswith("rank")) == [f"rank{r}_attempt0.log" for r in range(max(n0, n1))]
    text = "\n".join(logs.values()) + err
    assert text.count("rescaled in place") == min(n0, n1), text[-3000:]
    if n1 < n0:
        assert "retired by the scale" in text
    # the scale checkpoint was committed and the new ranks restored it (they resume mid-run)
    for r in range(n0, n1):
        assert f"rank {r} restored iteration" in text, text[-3000:]
