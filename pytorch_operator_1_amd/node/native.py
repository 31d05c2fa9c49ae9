"""Build and drive the native C++ node agent (``csrc/node/node_agent.cpp``).

The agent is a plain executable (``_lib/pto-node-agent``) built with g++
(optionally under ``-fsanitize=address,undefined`` for the sanitizer CI
target).  :class:`AgentClient` talks to it over its
line-delimited JSON protocol, either as a child process on stdin/stdout
(the default: the agent dies with its parent) or over a Unix socket to a
long-running daemon.
"""
from __future__ import annotations

import fcntl
import json
import os
import shutil
import socket
import subprocess
import sys
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(PKG_DIR, "csrc", "node", "node_agent.cpp")
BIN = os.path.join(PKG_DIR, "_lib", "pto-node-agent")


def build(force: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    out = BIN + ("-san" if sanitize else "")
    deps = [SRC, os.path.join(os.path.dirname(SRC), "json.hpp")]
    def fresh() -> bool:
        return os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)

    if not force and fresh():
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # Concurrent builders (pytest-xdist workers) serialise on a lock file and
    # each writes its own temp name, so nobody execs a half-written binary
    # ("Text file busy") or renames another builder's output.
    with open(out + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and fresh():
            return out
        tmp = f"{out}.tmp{os.getpid()}"
        cxx = os.environ.get("CXX") or shutil.which("g++") or "c++"
        cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-o", tmp, SRC]
        if sanitize:
            cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, out)
    return out


class AgentError(RuntimeError):
    pass


class AgentClient:
    def __init__(self, gpus: int | None = None, socket_path: str | None = None, hbm_per_gpu: float | None = None,
                 backoff_base: float = 0.2, backoff_max: float = 10.0, binary: str | None = None,
                 zygote: bool = False):
        """``zygote``: warm starts -- the agent keeps a pre-imported
        interpreter (``node/zygote.py``) and forks ``python -m``/``python
        x.py`` containers from it instead of fork/exec."""
        self._lock = threading.Lock()
        self._proc = None
        self._sock = None
        self._rfile = None
        if socket_path and os.path.exists(socket_path):
            self._sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            self._sock.connect(socket_path)
            self._rfile = self._sock.makefile("r")
        else:
            exe = binary or build()
            cmd = [exe, "--stdio", "--backoff-base", str(backoff_base), "--backoff-max", str(backoff_max)]
            if gpus is not None:
                cmd += ["--gpus", str(gpus)]
            if hbm_per_gpu:
                cmd += ["--hbm-per-gpu", str(hbm_per_gpu)]
            if zygote:
                cmd += ["--zygote", sys.executable, "--zygote-pythonpath", os.path.dirname(PKG_DIR)]
            self._proc = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)

    def call(self, op: str, **kw) -> dict:
        req = dict(op=op, **kw)
        line = json.dumps(req) + "\n"
        with self._lock:
            if self._proc is not None:
                if self._proc.poll() is not None:
                    raise AgentError("node agent exited")
                self._proc.stdin.write(line)
                self._proc.stdin.flush()
                resp = self._proc.stdout.readline()
            else:
                self._sock.sendall(line.encode())
                resp = self._rfile.readline()
        if not resp:
            raise AgentError("node agent closed the connection")
        out = json.loads(resp)
        return out

    def ok(self, op: str, **kw) -> dict:
        r = self.call(op, **kw)
        if not r.get("ok"):
            raise AgentError(r.get("error", f"{op} failed"))
        return r

    # convenience wrappers
    def spawn(self, id, argv, env=None, cwd=None, log=None, restart_policy="Never", cpus=None, launcher="auto",
              group=""):
        """``launcher``: "auto" (zygote when eligible) or "exec" (always
        fork/exec a fresh interpreter).  ``group``: restart group -- a failed
        member that is restarted takes every other member down with it and
        the whole group restarts together (node_agent.cpp, restart groups)."""
        return self.ok("spawn", id=id, argv=list(argv), env=dict(env or {}), cwd=cwd or "", log=log or "",
                       restart_policy=restart_policy, cpus=list(cpus or []), launcher=launcher, group=group or "")

    def kill(self, id, signal=15, grace=10.0, restartable=False):
        return self.call("kill", id=id, signal=signal, grace=grace, restartable=restartable)

    def status(self, id=None):
        r = self.ok("status", **({"id": id} if id else {}))
        return {p["id"]: p for p in r["procs"]}

    def remove(self, id):
        return self.call("remove", id=id)

    def gpus(self):
        return self.ok("gpus")

    def alloc(self, requests):
        return self.call("alloc", requests=list(requests))

    def free(self, owner):
        return self.call("free", owner=owner)

    def ping(self) -> dict:
        return self.ok("ping")

    def wait_warm(self, timeout: float = 60.0) -> bool:
        """Block until the agent's zygote (if enabled) has finished its
        imports; False if it is disabled, died, or is not ready in time."""
        import time

        end = time.time() + timeout
        while time.time() < end:
            z = self.ping().get("zygote", {})
            if not z.get("enabled") or (z.get("pid", -1) < 0):
                return False
            if z.get("ready"):
                return True
            time.sleep(0.05)
        return False

    def probe(self, host, port, timeout=0.5) -> bool:
        return bool(self.ok("probe", host=host, port=int(port), timeout=timeout).get("open"))

    def close(self):
        try:
            if self._proc is not None and self._proc.poll() is None:
                self.call("shutdown")
                self._proc.wait(10)
        except Exception:
            if self._proc is not None:
                self._proc.kill()
        if self._sock is not None:
            self._sock.close()
