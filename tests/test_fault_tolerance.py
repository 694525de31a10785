"""Fault injection end to end: 2 gloo ranks train under the elastic
supervisor with periodic checkpoints; rank 1 is killed mid-run (--fail_rank/--fail_step), the
supervisor detects it (Phase2), relaunches the rank set from the last committed checkpoint (Phase3),
the ranks restore (Phase4/5) and finish; the final parameters equal an uninterrupted run's."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp, extra, name):
    cmd = [sys.executable, "-m", "minips_amd.elastic", "--nproc", "2", "--heartbeat_interval", "0.5",
           "--max_restarts", "2", "--run_dir", str(tmp / f"run_{name}"), "--log_dir", str(tmp / f"log_{name}"), "--",
           sys.executable, "-m", "minips_amd.train", "--small=1", "--steps", "12", "--checkpoint_toggle=1",
           "--checkpoint_every", "4", f"--checkpoint_file_prefix={tmp}/ck_{name}/", *extra]
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    logs = {}
    for f in sorted(os.listdir(tmp / f"log_{name}")):
        logs[f] = open(tmp / f"log_{name}" / f).read()
    return p, logs


def _summary(logs):
    last = [l for l in logs[max(k for k in logs if k.startswith("rank0_"))].splitlines() if l.startswith("{")]
    return json.loads(last[-1])


@pytest.mark.parametrize("model", ["widedeep", "lr"])
def test_kill_rank_restart_restore(tmp_path, model):
    ref, ref_logs = _run(tmp_path, [f"--model={model}"], "ref")
    assert ref.returncode == 0, ref.stderr[-3000:]
    got, logs = _run(tmp_path, [f"--model={model}", "--fail_rank=1", "--fail_step=9"], "ft")
    assert got.returncode == 0, (got.stderr[-3000:], logs)
    err = got.stderr
    assert "[Fault Tolerance][Phase2]" in err and "rank 1 failed" in err
    assert "[Fault Tolerance][Phase3]" in err
    rank_logs = "".join(v for k, v in logs.items() if "attempt1" in k)
    assert "[Fault Tolerance][Phase4]" in rank_logs and "[Fault Tolerance][Phase5]" in rank_logs
    a, b = _summary(ref_logs), _summary(logs)
    assert b["start"] == 8  # resumed from the checkpoint committed after iteration 8
    assert a["checksum"] == b["checksum"], (a, b)
    assert a["losses"][-1] == b["losses"][-1]
