"""In-process WebHDFS stand-in for the HDFS tests (no Hadoop in this image, no network).

A namenode and a datanode HTTP server over one local directory, speaking the subset of the
WebHDFS REST API the native client uses (csrc/runtime/fs.cc): GETFILESTATUS, LISTSTATUS,
GETFILEBLOCKLOCATIONS (or only the older GET_BLOCK_LOCATIONS), OPEN / CREATE / APPEND via a 307
redirect to the datanode, MKDIRS, RENAME, DELETE. Block k of every file is reported on
``hosts_of(k)`` so the locality-aware assigner can be exercised with made-up datanode names.
"""
from __future__ import annotations

import json
import os
import shutil
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, unquote, urlparse


class MockWebHdfs:
    def __init__(self, root: str, block_size: int = 4096, hosts_of=None, legacy_locations: bool = False):
        self.root = root
        self.block_size = block_size
        self.hosts_of = hosts_of or (lambda k: ["dn0"])
        self.legacy = legacy_locations
        self.ops = []  # (server, method, op) log
        self._nn = ThreadingHTTPServer(("127.0.0.1", 0), self._handler(namenode=True))
        self._dn = ThreadingHTTPServer(("127.0.0.1", 0), self._handler(namenode=False))
        self.port = self._nn.server_address[1]
        self.dn_port = self._dn.server_address[1]
        self._threads = [threading.Thread(target=s.serve_forever, daemon=True) for s in (self._nn, self._dn)]
        for t in self._threads:
            t.start()

    def url(self, path: str = "/") -> str:
        return f"webhdfs://127.0.0.1:{self.port}{path}"

    def close(self):
        for s in (self._nn, self._dn):
            s.shutdown()
            s.server_close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ handler
    def _status(self, path):
        st = os.stat(path)
        is_dir = os.path.isdir(path)
        return {"type": "DIRECTORY" if is_dir else "FILE", "length": 0 if is_dir else st.st_size,
                "blockSize": self.block_size, "pathSuffix": "", "replication": 3}

    def _handler(self, namenode: bool):
        fs = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _reply(self, code, body=b"", ctype="application/json", headers=()):
                if isinstance(body, (dict, list)):
                    body = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                for k, v in headers:
                    self.send_header(k, v)
                self.end_headers()
                if body:
                    self.wfile.write(body)

            def _err(self, code, msg):
                self._reply(code, {"RemoteException": {"exception": "FileNotFoundException", "message": msg}})

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return self.rfile.read(n) if n else b""

            def _handle(self, method):
                u = urlparse(self.path)
                assert u.path.startswith("/webhdfs/v1"), u.path
                hpath = unquote(u.path[len("/webhdfs/v1"):]) or "/"
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                op = q.get("op", "")
                fs.ops.append(("nn" if namenode else "dn", method, op))
                local = os.path.join(fs.root, hpath.lstrip("/"))
                if namenode and op in ("OPEN", "CREATE", "APPEND"):
                    self._body()
                    loc = f"http://127.0.0.1:{fs.dn_port}{self.path}&datanode=true"
                    return self._reply(307, b"", headers=[("Location", loc)])
                if op == "OPEN":
                    if not os.path.isfile(local):
                        return self._err(404, f"File {hpath} does not exist.")
                    off = int(q.get("offset", 0))
                    with open(local, "rb") as f:
                        f.seek(off)
                        data = f.read(int(q["length"])) if "length" in q else f.read()
                    return self._reply(200, data, "application/octet-stream")
                if op == "CREATE":
                    os.makedirs(os.path.dirname(local), exist_ok=True)
                    with open(local, "wb") as f:
                        f.write(self._body())
                    return self._reply(201)
                if op == "APPEND":
                    with open(local, "ab") as f:
                        f.write(self._body())
                    return self._reply(200)
                if op == "GETFILESTATUS":
                    if not os.path.exists(local):
                        return self._err(404, f"File does not exist: {hpath}")
                    return self._reply(200, {"FileStatus": fs._status(local)})
                if op == "LISTSTATUS":
                    if not os.path.exists(local):
                        return self._err(404, f"File does not exist: {hpath}")
                    names = sorted(os.listdir(local)) if os.path.isdir(local) else [""]
                    sts = []
                    for n in names:
                        s = fs._status(os.path.join(local, n) if n else local)
                        s["pathSuffix"] = n
                        sts.append(s)
                    return self._reply(200, {"FileStatuses": {"FileStatus": sts}})
                if op in ("GETFILEBLOCKLOCATIONS", "GET_BLOCK_LOCATIONS"):
                    if op == "GETFILEBLOCKLOCATIONS" and fs.legacy:
                        return self._reply(400, {"RemoteException": {"message": "Invalid value for webhdfs "
                                                                                "parameter \"op\""}})
                    size = os.path.getsize(local)
                    blocks = [(k, off, min(fs.block_size, size - off))
                              for k, off in enumerate(range(0, size, fs.block_size))]
                    if op == "GETFILEBLOCKLOCATIONS":
                        return self._reply(200, {"BlockLocations": {"BlockLocation": [
                            {"offset": off, "length": ln, "hosts": fs.hosts_of(k), "names": [], "topologyPaths": []}
                            for k, off, ln in blocks]}})
                    return self._reply(200, {"LocatedBlocks": {"fileLength": size, "locatedBlocks": [
                        {"startOffset": off, "block": {"numBytes": ln, "blockId": k},
                         "locations": [{"hostName": h, "ipAddr": "127.0.0.1"} for h in fs.hosts_of(k)]}
                        for k, off, ln in blocks]}})
                if op == "MKDIRS":
                    os.makedirs(local, exist_ok=True)
                    return self._reply(200, {"boolean": True})
                if op == "RENAME":
                    dst = os.path.join(fs.root, unquote(q["destination"]).lstrip("/"))
                    os.replace(local, dst)
                    return self._reply(200, {"boolean": True})
                if op == "DELETE":
                    if os.path.isdir(local):
                        shutil.rmtree(local)
                    elif os.path.exists(local):
                        os.unlink(local)
                    return self._reply(200, {"boolean": True})
                return self._reply(400, {"RemoteException": {"message": f"unsupported op {op}"}})

            def do_GET(self):
                self._handle("GET")

            def do_PUT(self):
                self._handle("PUT")

            def do_POST(self):
                self._handle("POST")

            def do_DELETE(self):
                self._handle("DELETE")

        return H
