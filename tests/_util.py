import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ensure_built(*targets):
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py"), *targets], check=True, cwd=ROOT,
                   capture_output=True)


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def write_hostfile(path, n, gpu=False):
    ports = free_ports(n)
    with open(path, "w") as f:
        for i, p in enumerate(ports):
            f.write(f"{i}:localhost:{p}" + (f":{i}" if gpu else "") + "\n")
    return path
