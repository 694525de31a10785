"""Native apps end to end on the CPU runtime (BASELINE config 1: LR over TCP, 2 worker
threads per node) plus the basic and K-Means apps, launched through minips_amd.launch."""
import json
import os

import pytest

from _util import ensure_built, write_hostfile
from minips_amd import launch


@pytest.fixture(scope="module", autouse=True)
def _build():
    ensure_built("runtime", "apps")


def _run(app, tmp_path, nodes, flags, timeout=120):
    hf = write_hostfile(str(tmp_path / "hosts"), nodes)
    logs = str(tmp_path / "logs")
    rcs = launch.launch_nodes(app, hf, flags, log_dir=logs, timeout=timeout)
    assert all(rc == 0 for rc in rcs), rcs
    out = []
    for i in range(nodes):
        with open(os.path.join(logs, f"node_{i}.log")) as f:
            js = [l for l in f if l.startswith("{")]
        out.append(json.loads(js[-1]))
    return out


@pytest.mark.parametrize("model", ["BSP", "SSP", "ASP"])
def test_lr_two_nodes(tmp_path, model):
    res = _run("lr", tmp_path, 2, ["--num_workers_per_node=2", "--num_iters=200", "--batch_size=20",
                                   "--num_dims=5000", f"--kModelType={model}", "--kStaleness=2", "--alpha=0.5"])
    assert all(r["accuracy"] > 0.8 for r in res), res


def test_lr_single_node_two_workers_one_server(tmp_path):
    res = _run("lr", tmp_path, 1, ["--num_workers_per_node=2", "--num_servers_per_node=1", "--num_iters=200",
                                   "--batch_size=20", "--num_dims=3000", "--kModelType=BSP", "--alpha=0.5",
                                   "--kStorageType=Map"])
    assert res[0]["accuracy"] > 0.8


def test_basic_example_exact(tmp_path):
    res = _run("basic", tmp_path, 2, ["--num_workers_per_node=3", "--num_iters=30"])
    assert res[0]["got"] == res[0]["expected"] == 0.5 * 3 * 2 * 30


def test_kmeans(tmp_path):
    res = _run("kmeans", tmp_path, 2, ["--num_workers_per_node=2", "--num_iters=30", "--batch_size=40",
                                       "--num_dims=32", "--K=4", "--report_interval=10", "--kModelType=SSP"])
    assert res[0]["sampled_sse"] > 0  # the report worker (worker 0) lives on node 0


def test_lr_checkpoint_files(tmp_path):
    ck = str(tmp_path / "ckpt") + "/"
    _run("lr", tmp_path, 1, ["--num_workers_per_node=2", "--num_iters=201", "--batch_size=10", "--num_dims=2000",
                             "--kModelType=SSP", "--checkpoint_toggle=true", f"--checkpoint_file_prefix={ck}"])
    params = open(ck + "server_params_0").read().split()
    assert params and all(":" in p for p in params)
    prog = open(ck + "server_progress_0").read()
    assert prog.startswith("min_clock:")
    assert open(ck + "worker_config_0").read().strip()


def test_cluster_layout_parsing():
    from minips_amd.launch import cluster_layout, expand_nodelist, expand_tasks_per_node

    assert expand_nodelist("gpu[01-03,07],login1") == ["gpu01", "gpu02", "gpu03", "gpu07", "login1"]
    assert expand_tasks_per_node("2(x3),1", 4) == [2, 2, 2, 1]
    me, nodes = cluster_layout({"SLURM_PROCID": "3", "SLURM_JOB_NODELIST": "n[1-2]", "SLURM_TASKS_PER_NODE": "2(x2)"},
                               100)
    assert me == 3 and nodes == [(0, "n1", 100), (1, "n1", 101), (2, "n2", 100), (3, "n2", 101)]
    me, nodes = cluster_layout({"JOB_COMPLETION_INDEX": "2", "MINIPS_HOSTS": "p-0.svc,p-1.svc,p-2.svc"}, 7)
    assert me == 2 and nodes[2] == (2, "p-2.svc", 7)


def test_lr_via_simulated_slurm_steps(tmp_path):
    """The cluster verb (YARN-client/AM analogue) inside two simulated Slurm tasks on this host:
    each task derives its id and the same hostfile from SLURM_* and runs its node of the LR app."""
    import subprocess
    import sys

    from _util import ROOT, free_ports

    port = free_ports(1)[0]
    procs = []
    for rank in range(2):
        env = dict(os.environ, SLURM_PROCID=str(rank), SLURM_JOB_NODELIST="localhost", SLURM_TASKS_PER_NODE="2",
                   SLURM_JOB_ID="t1")
        cmd = [sys.executable, "-m", "minips_amd.launch", "--app", "lr", "--start-port", str(port),
               "--hostfile-out", str(tmp_path / f"hosts_{rank}"), "--log-dir", str(tmp_path / "logs"), "cluster",
               "--num_workers_per_node=2", "--num_iters=150", "--batch_size=20", "--num_dims=3000",
               "--kModelType=BSP", "--alpha=0.5"]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env))
    rcs = [p.wait(timeout=180) for p in procs]
    assert rcs == [0, 0]
    assert open(tmp_path / "hosts_0").read() == open(tmp_path / "hosts_1").read() == \
        f"0:localhost:{port}\n1:localhost:{port + 1}\n"
    for i in range(2):
        with open(tmp_path / "logs" / f"node_{i}.log") as f:
            assert json.loads([l for l in f if l.startswith("{")][-1])["accuracy"] > 0.8
