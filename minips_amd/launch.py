"""Launcher (parity with the reference scripts/launch_utils.py + scripts/<app>.py verbs).

    python -m minips_amd.launch --app lr --hostfile config/localnodes local [--flag=value ...]
    python -m minips_amd.launch --app lr --hostfile config/localnodes relaunch <node_id>
    python -m minips_amd.launch --app lr --hostfile config/localnodes relocal <node_id>
    python -m minips_amd.launch --app lr --hostfile config/localnodes scale <id> <host> <port>
    python -m minips_amd.launch --app lr --hostfile config/localnodes kill

    srun python -m minips_amd.launch --app lr cluster --start-port 19000 [--flag=value ...]

`local` starts one process per hostfile line (locally, or over ssh for remote hosts) with
`--my_id=<id> --config_file=<hostfile>` plus the pass-through flags. `relaunch` restarts one
node with --use_weight_file (resume from the checkpoint) -- it is what the master's
--relaunch_cmd calls. `kill` stops every process this launcher started (tracked by PID files,
never by name pattern). Apps: lr, kmeans, basic (native C++ binaries in build/bin) or any
executable path. For the GPU data plane use torchrun / bench.py (one process per GPU).

`cluster` is the cluster-scheduler entry (the reference's YARN client + ApplicationMaster,
yarn/src/main/java/.../{Client,ApplicationMaster}.java, which allocate containers, write the
`i:ip:start_port` hostfile and run the launch script in every container): it runs INSIDE each
task a scheduler started -- a Slurm step (`srun`), a Kubernetes indexed Job, or anything that
sets MINIPS_NODE_ID + MINIPS_HOSTS -- derives this task's node id and the whole hostfile from
the scheduler's environment (every task computes the same file, so no shared file system is
needed), writes it, and runs its node of the app.
"""
from __future__ import annotations

import argparse
import os
import shlex
import signal
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = {"lr": "build/bin/lr_example", "kmeans": "build/bin/kmeans", "basic": "build/bin/basic_example"}
PID_DIR = os.environ.get("MINIPS_PID_DIR", "/tmp/minips_pids")


def parse_hostfile(path: str):
    nodes = []
    with open(path) as f:
        for line in f:
            line = line.split("#")[0].strip()
            if not line:
                continue
            parts = line.split(":")
            nodes.append({"id": int(parts[0]), "host": parts[1], "port": int(parts[2]),
                          "gpu": int(parts[3]) if len(parts) > 3 else -1})
    return nodes


def _is_local(host: str) -> bool:
    return host in ("localhost", "127.0.0.1", socket.gethostname())


def _binary(app: str) -> str:
    p = APPS.get(app, app)
    # MINIPS_BIN_DIR swaps the build (e.g. build/san_thread/bin for sanitizer runs of the apps)
    bdir = os.environ.get("MINIPS_BIN_DIR")
    if bdir and app in APPS:
        p = os.path.join(bdir, os.path.basename(p))
    return p if os.path.isabs(p) else os.path.join(ROOT, p)


def _pidfile(app: str, node_id: int) -> str:
    return os.path.join(PID_DIR, f"{os.path.basename(app)}_{node_id}.pid")


def launch_node(app: str, hostfile: str, node: dict, flags: list[str], extra: list[str] = (), log_dir=None,
                wait=False):
    cmd = [_binary(app), f"--config_file={os.path.abspath(hostfile)}", f"--my_id={node['id']}", *flags, *extra]
    env = dict(os.environ)
    if node.get("gpu", -1) >= 0:
        env["HIP_VISIBLE_DEVICES"] = str(node["gpu"])
    os.makedirs(PID_DIR, exist_ok=True)
    log = None
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        log = open(os.path.join(log_dir, f"node_{node['id']}.log"), "w")
    if _is_local(node["host"]):
        p = subprocess.Popen(cmd, env=env, stdout=log or None, stderr=subprocess.STDOUT if log else None,
                             start_new_session=True)
    else:
        remote = " ".join(shlex.quote(c) for c in cmd)
        p = subprocess.Popen(["ssh", "-o", "StrictHostKeyChecking=no", node["host"], remote],
                             stdout=log or None, stderr=subprocess.STDOUT if log else None, start_new_session=True)
    with open(_pidfile(app, node["id"]), "w") as f:
        f.write(str(p.pid))
    if wait:
        return p.wait()
    return p


def launch_nodes(app: str, hostfile: str, flags: list[str], log_dir=None, wait=True, timeout=None):
    procs = [launch_node(app, hostfile, n, flags, log_dir=log_dir) for n in parse_hostfile(hostfile)]
    if not wait:
        return procs
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            rcs.append(-9)
    return rcs


def relaunch(app: str, hostfile: str, node_id: int, flags: list[str], log_dir=None):
    node = next(n for n in parse_hostfile(hostfile) if n["id"] == node_id)
    return launch_node(app, hostfile, node, flags, extra=["--use_weight_file=true"], log_dir=log_dir)


def kill_nodes(app: str, hostfile: str):
    for n in parse_hostfile(hostfile):
        pf = _pidfile(app, n["id"])
        if not os.path.exists(pf):
            continue
        with open(pf) as f:
            pid = int(f.read().strip())
        try:
            os.killpg(pid, signal.SIGKILL)  # the process group this launcher created
        except ProcessLookupError:
            pass
        os.remove(pf)


# ------------------------------------------------------------------------------ cluster schedulers
def expand_nodelist(spec: str) -> list[str]:
    """Slurm hostlist syntax: "gpu[01-03,07],login1" -> gpu01 gpu02 gpu03 gpu07 login1."""
    out, i, n = [], 0, len(spec)
    while i < n:
        j = i
        while j < n and spec[j] not in ",[":
            j += 1
        prefix = spec[i:j]
        if j < n and spec[j] == "[":
            k = spec.index("]", j)
            suffix_end = k + 1
            while suffix_end < n and spec[suffix_end] != ",":
                suffix_end += 1
            suffix = spec[k + 1: suffix_end]
            for part in spec[j + 1: k].split(","):
                if "-" in part:
                    a, b = part.split("-")
                    for v in range(int(a), int(b) + 1):
                        out.append(f"{prefix}{str(v).zfill(len(a))}{suffix}")
                else:
                    out.append(prefix + part + suffix)
            i = suffix_end + 1
        else:
            if prefix:
                out.append(prefix)
            i = j + 1
    return out


def expand_tasks_per_node(spec: str, nodes: int) -> list[int]:
    """SLURM_TASKS_PER_NODE: "2(x3),1" -> [2, 2, 2, 1]."""
    out = []
    for part in spec.split(","):
        if "(x" in part:
            c, rep = part.rstrip(")").split("(x")
            out += [int(c)] * int(rep)
        elif part:
            out.append(int(part))
    return out if out else [1] * nodes


def cluster_layout(env=None, start_port: int = 19000):
    """(my node id, [(id, host, port)]) from the scheduler's environment."""
    env = os.environ if env is None else env
    if "SLURM_PROCID" in env:  # block task distribution (Slurm's default)
        hosts = expand_nodelist(env.get("SLURM_STEP_NODELIST") or env["SLURM_JOB_NODELIST"])
        per = expand_tasks_per_node(env.get("SLURM_STEP_TASKS_PER_NODE") or env.get("SLURM_TASKS_PER_NODE", ""),
                                    len(hosts))
        nodes = []
        for h, count in zip(hosts, per):
            for local in range(count):  # the tasks of one host get consecutive ports
                nodes.append((len(nodes), h, start_port + local))
        me = int(env["SLURM_PROCID"])
    elif "MINIPS_HOSTS" in env or "JOB_COMPLETION_INDEX" in env:  # generic / Kubernetes indexed Job
        hosts = [h for h in env["MINIPS_HOSTS"].split(",") if h]
        me = int(env.get("MINIPS_NODE_ID", env.get("JOB_COMPLETION_INDEX", "0")))
        seen: dict = {}
        nodes = []
        for i, h in enumerate(hosts):  # several tasks on one host get consecutive ports
            nodes.append((i, h, start_port + seen.get(h, 0)))
            seen[h] = seen.get(h, 0) + 1
    else:
        raise RuntimeError("cluster: no scheduler environment (SLURM_PROCID, or MINIPS_NODE_ID + MINIPS_HOSTS)")
    if not 0 <= me < len(nodes):
        raise RuntimeError(f"cluster: node id {me} outside the {len(nodes)}-node layout")
    return me, nodes


def run_cluster_task(app: str, flags: list[str], start_port: int, hostfile_out=None, log_dir=None, env=None):
    me, nodes = cluster_layout(env, start_port)
    tag = (env or os.environ).get("SLURM_JOB_ID") or (env or os.environ).get("MINIPS_JOB_ID", "job")
    path = hostfile_out or os.path.join("/tmp", f"minips_cluster_{tag}_{me}.hosts")
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path + ".tmp", "w") as f:
        f.writelines(f"{i}:{h}:{p}\n" for i, h, p in nodes)
    os.replace(path + ".tmp", path)
    node = {"id": me, "host": "localhost", "port": nodes[me][2], "gpu": -1}  # this task runs its own node
    return launch_node(app, path, node, flags, log_dir=log_dir, wait=True)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--app", default="lr")
    ap.add_argument("--hostfile", default=os.path.join(ROOT, "config/localnodes"))
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--start-port", type=int, default=19000, help="cluster: first port of every host")
    ap.add_argument("--hostfile-out", default=None, help="cluster: where this task writes the hostfile")
    ap.add_argument("verb", choices=["local", "relaunch", "relocal", "scale", "kill", "cluster"])
    ap.add_argument("args", nargs="*")
    ns, flags = ap.parse_known_args(argv)
    if ns.verb == "cluster":
        return abs(run_cluster_task(ns.app, flags, ns.start_port, ns.hostfile_out, log_dir=ns.log_dir))
    if ns.verb == "local":
        rcs = launch_nodes(ns.app, ns.hostfile, flags, log_dir=ns.log_dir)
        return max(abs(r) for r in rcs) if rcs else 0
    if ns.verb in ("relaunch", "relocal"):
        relaunch(ns.app, ns.hostfile, int(ns.args[0]), flags, log_dir=ns.log_dir)
        return 0
    if ns.verb == "scale":
        nid, host, port = int(ns.args[0]), ns.args[1], int(ns.args[2])
        node = {"id": nid, "host": host, "port": port, "gpu": -1}
        launch_node(ns.app, ns.hostfile, node, flags, extra=["--scale=true", f"--scale_node_id={nid}"],
                    log_dir=ns.log_dir)
        return 0
    kill_nodes(ns.app, ns.hostfile)
    return 0


if __name__ == "__main__":
    sys.exit(main())
