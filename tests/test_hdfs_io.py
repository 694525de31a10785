"""HDFS data plane of the runtime (reference io/ + base/third_party/{general_fstream,hdfs}):
webhdfs:// reads and writes through the native REST client, the locality-aware block
assigner service, and the apps loading input / dumping checkpoints over it. A Python WebHDFS
stand-in (tests/_webhdfs.py) plays namenode + datanode; the reference's own HDFS test
(test/test_hdfs_read.cpp) needs a live cluster and has no fixture, so parity is against local
files holding the same bytes."""
import json
import os
import random
import threading

import numpy as np
import pytest

from _util import ensure_built, write_hostfile
from _webhdfs import MockWebHdfs
from minips_amd import launch
from minips_amd._native import runtime


@pytest.fixture(scope="module", autouse=True)
def _build():
    ensure_built("runtime", "rt_py", "apps")


def _libsvm(path, rows=600, seed=0):
    rng = random.Random(seed)
    with open(path, "w") as f:
        for i in range(rows):
            feats = sorted(rng.sample(range(1, 400), 1 + i % 9))
            f.write(("+1" if i % 3 else "-1") + "".join(f" {k}:{rng.random():.6g}" for k in feats) + "\n")


def _load(url, **kw):
    return [np.asarray(a) for a in runtime().load_libsvm(url, **kw)]


def test_webhdfs_read_matches_local(tmp_path):
    root = tmp_path / "hdfs"
    (root / "data").mkdir(parents=True)
    for k in range(3):
        _libsvm(str(root / "data" / f"part-{k}"), rows=400 + 50 * k, seed=k)
    local = _load(str(root / "data"), threads=3)
    with MockWebHdfs(str(root), block_size=2048) as fs:
        before = runtime().remote_bytes_read()
        remote = _load(fs.url("/data"), threads=3)
        assert runtime().remote_bytes_read() - before >= sum(os.path.getsize(root / "data" / f) for f in
                                                             os.listdir(root / "data"))
        # blocks of the HDFS block size, each read with one ranged OPEN (+ the straddling tail)
        assert sum(1 for s, m, op in fs.ops if s == "dn" and op == "OPEN") >= 3
        # two static shards cover the data exactly once
        parts = [_load(fs.url("/data"), shard=r, num_shards=2, threads=2) for r in range(2)]
    for a, b in zip(local, remote):
        np.testing.assert_array_equal(a, b)
    assert sum(len(p[3]) for p in parts) == len(local[3])
    assert sorted(np.concatenate([p[3] for p in parts]).tolist()) == sorted(local[3].tolist())


def test_webhdfs_legacy_block_locations_and_listing(tmp_path):
    root = tmp_path / "hdfs"
    root.mkdir()
    _libsvm(str(root / "one.svm"), rows=300)
    with MockWebHdfs(str(root), block_size=1000, hosts_of=lambda k: [f"dn{k % 2}", "dn9"],
                     legacy_locations=True) as fs:
        files = runtime().fs_list(fs.url("/"))
        assert [f[0] for f in files] == [fs.url("/one.svm")]
        assert files[0][1] == os.path.getsize(root / "one.svm") and files[0][2] == 1000
        locs = runtime().fs_locations(fs.url("/one.svm"))
        assert len(locs) == (files[0][1] + 999) // 1000
        assert locs[1][2] == ["dn1", "dn9"]


def test_webhdfs_write_roundtrip(tmp_path):
    root = tmp_path / "hdfs"
    root.mkdir()
    with MockWebHdfs(str(root)) as fs:
        payload = os.urandom(100_000)
        runtime().fs_write(fs.url("/ck/deep/blob"), payload)
        assert (root / "ck" / "deep" / "blob").read_bytes() == payload
        assert runtime().fs_read(fs.url("/ck/deep/blob")) == payload
        assert runtime().fs_exists(fs.url("/ck/deep/blob"))
        assert not runtime().fs_exists(fs.url("/ck/missing"))


def test_locality_assigner_serves_local_blocks(tmp_path):
    """Two loader nodes on datanodes dn0 / dn1; block k lives on dn(k % 2) only. With the
    assigner service every block goes to the node that stores it (io/hdfs_assigner.cpp:160-222),
    each block exactly once, and the service halts after every loader thread's kExit."""
    root = tmp_path / "hdfs"
    (root / "in").mkdir(parents=True)
    for k in range(2):
        _libsvm(str(root / "in" / f"p{k}"), rows=500, seed=10 + k)
    local = _load(str(root / "in"))
    with MockWebHdfs(str(root), block_size=1500, hosts_of=lambda k: [f"dn{k % 2}"]) as fs:
        srv = runtime().BlockAssignerServer(0)
        srv.start()
        out = [None, None]

        def node(r):
            out[r] = _load(fs.url("/in"), shard=r, num_shards=2, threads=2, assigner=f"127.0.0.1:{srv.port}",
                           host=f"dn{r}")

        th = [threading.Thread(target=node, args=(r,)) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert srv.wait_done(10)
        n_blocks = sum(len(runtime().fs_locations(f[0])) for f in runtime().fs_list(fs.url("/in")))
        local_served, remote_served = srv.local_served, srv.remote_served
        srv.stop()
    assert local_served + remote_served == n_blocks
    assert remote_served <= 2  # only a node that ran out of its own blocks reads a remote one
    labels = np.concatenate([o[3] for o in out])
    assert len(labels) == len(local[3])
    assert sorted(labels.tolist()) == sorted(local[3].tolist())


def test_hdfs_scheme_without_libhdfs3(tmp_path, monkeypatch):
    ok, why = runtime().libhdfs3_available()
    if ok:
        pytest.skip("libhdfs3 is installed here")
    with pytest.raises(Exception, match="webhdfs://"):
        runtime().fs_list("hdfs://127.0.0.1:9/x")


def test_lr_app_webhdfs_input_assigner_and_checkpoints(tmp_path):
    """The LR app reads its libsvm input from (mock) HDFS through node 0's block assigner and
    dumps its checkpoint files to an hdfs prefix (reference: --hdfs_namenode/--input/
    --assigner_master_port, checkpoint_file_prefix=hdfs://...)."""
    root = tmp_path / "hdfs"
    (root / "train").mkdir(parents=True)
    rng = random.Random(3)
    teacher = [rng.gauss(0, 1) for _ in range(200)]
    with open(root / "train" / "part-0", "w") as f:
        for _ in range(1500):
            feats = sorted(rng.sample(range(200), 8))
            z = sum(teacher[k] for k in feats)
            f.write(("1" if z > 0 else "-1") + "".join(f" {k + 1}:1" for k in feats) + "\n")
    with MockWebHdfs(str(root), block_size=8192) as fs:
        hf = write_hostfile(str(tmp_path / "hosts"), 2)
        from _util import free_ports

        port = free_ports(1)[0]
        flags = ["--num_workers_per_node=2", "--num_iters=150", "--batch_size=20", "--num_dims=200",
                 "--kModelType=BSP", "--alpha=0.5", "--hdfs_namenode=127.0.0.1", f"--hdfs_http_port={fs.port}",
                 "--input=/train", f"--assigner_master_port={port}", "--checkpoint_toggle=true",
                 f"--checkpoint_file_prefix={fs.url('/ck/')}"]
        logs = str(tmp_path / "logs")
        rcs = launch.launch_nodes("lr", hf, flags, log_dir=logs, timeout=180)
        assert all(rc == 0 for rc in rcs), [open(os.path.join(logs, f)).read()[-2000:] for f in os.listdir(logs)]
        res = []
        for i in range(2):
            with open(os.path.join(logs, f"node_{i}.log")) as f:
                res.append(json.loads([l for l in f if l.startswith("{")][-1]))
        assert all(r["accuracy"] > 0.75 for r in res), res
        assert any(s == "dn" and op == "OPEN" for s, _, op in fs.ops)
        assert any(op == "CREATE" for _, _, op in fs.ops)
    params = (root / "ck" / "server_params_0").read_text().split()
    assert params and all(":" in p for p in params)
    assert (root / "ck" / "server_progress_0").read_text().startswith("min_clock:")


def test_train_driver_two_ranks_webhdfs_assigner(tmp_path):
    """python -m minips_amd.train (2 gloo ranks) --model lr with the input on (mock) HDFS and rank 0
    serving block assignment: every sample lands on exactly one rank and training converges."""
    import subprocess
    import sys

    from _util import free_ports

    root = tmp_path / "hdfs"
    (root / "d").mkdir(parents=True)
    rng = random.Random(5)
    teacher = [rng.gauss(0, 1) for _ in range(300)]
    with open(root / "d" / "part-0", "w") as f:
        for _ in range(4000):
            feats = sorted(rng.sample(range(300), 10))
            f.write(("1" if sum(teacher[k] for k in feats) > 0 else "0") + "".join(f" {k + 1}:1" for k in feats) + "\n")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mport, aport = free_ports(2)
    with MockWebHdfs(str(root), block_size=16384) as fs:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(mport), "-m", "minips_amd.train", "--model", "lr",
               "--input", "/d", "--hdfs_namenode", "127.0.0.1", "--hdfs_http_port", str(fs.port),
               "--assigner_master_port", str(aport), "--num_dims", "300", "--batch", "100", "--steps", "120",
               "--alpha", "0.1"]
        r = subprocess.run(cmd, cwd=repo, capture_output=True, text=True, timeout=300,
                           env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
        assert r.returncode == 0, r.stderr[-3000:]
    assert "block assigner:" in r.stdout
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    accs = [-v for _, v in out["losses"]]
    assert sum(accs[-5:]) / 5 > 0.8, accs
