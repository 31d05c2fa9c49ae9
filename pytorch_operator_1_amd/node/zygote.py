"""Warm interpreter pool for the node agent (``pto-node-agent --zygote``).

A container that runs ``python -m <module> ...`` or ``python <script>.py
...`` normally pays the interpreter start and ``import torch`` (≈1.5–2 s on
this image) on the submit -> first-step critical path, and again on every
restart.  The reference pays it inside its container runtime too (image
pull + interpreter start, SURVEY §6: 121 s / 334 s submit -> Running).

The zygote is started ONCE by the agent, imports torch and this package's
runtimes (never touching the GPU: no HIP call, no kernel library load), and
then forks a ready interpreter per container:

  agent --{"argv","env","cwd","log","cpus"}--> zygote
  zygote: fork -> child forks the container process and exits at once, so
          the container is re-parented to the agent (a child subreaper)
          and the agent reaps it exactly like a fork/exec'ed container
          (exit codes, signals, restart policy, process-group kill).
  zygote --{"ok": true, "pid": N}--> agent

The container process: new session (own process group), log file on
stdout/stderr, /dev/null stdin, working directory, CPU affinity, the pod's
environment as ``os.environ`` (GPU pinning via ``HIP_VISIBLE_DEVICES`` is
read at HIP init, which has not happened yet), then ``runpy`` runs the
module/script as ``__main__``.  Nothing is exec'ed.

Protocol: JSON lines on the inherited socket ``--fd``; the first line the
zygote writes is ``{"ready": true, "pid": ...}``.

``--spare``: the same warm interpreter, but it runs the FIRST container it
is asked for itself, without forking (the agent keeps one ready for the
containers that must not start in a forked interpreter: the rendezvous
store host of a multi-rank job, node/kubelet.py), and is then replaced.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import signal
import sys
import traceback

# modules every supported container imports (torch dominates the cost)
PRELOAD = (
    "torch",
    "torch.distributed",
    "torch.nn.functional",
    "torch.optim",  # its first optimizer constructs import torch._dynamo (~1.5 s)
    "torch._dynamo",
    "numpy",
    "pytorch_operator_1_amd.train.mnist",
    "pytorch_operator_1_amd.train.fused_step",
    "pytorch_operator_1_amd.train.sendrecv",
)

# interpreter flags a forked container can honour (anything else: exec path)
_ELIGIBLE_FLAGS = {"-u"}


def eligible(argv: list[str], python: str) -> bool:
    """True if ``argv`` is ``python [-u] (-m MODULE | SCRIPT.py) ARGS...``
    for the zygote's own interpreter."""
    if len(argv) < 2 or os.path.realpath(argv[0]) != os.path.realpath(python):
        return False
    i = 1
    while i < len(argv) and argv[i] in _ELIGIBLE_FLAGS:
        i += 1
    if i >= len(argv):
        return False
    if argv[i] == "-m":
        return i + 1 < len(argv)
    return argv[i].endswith(".py") and not argv[i].startswith("-")


def _preload():
    import importlib
    import threading

    for m in PRELOAD:
        try:
            importlib.import_module(m)
        except Exception as e:  # noqa: BLE001 - a missing optional runtime only loses warmth
            print(f"[zygote] preload {m} failed: {e}", file=sys.stderr, flush=True)
    if threading.active_count() != 1:  # fork() copies only the calling thread
        print(f"[zygote] warning: {threading.active_count()} threads after preload", file=sys.stderr, flush=True)


def _run_container(req: dict) -> int:
    """Body of the container process; returns its exit code."""
    import time

    t_enter = time.time()
    os.setsid()
    for s in (signal.SIGTERM, signal.SIGCHLD, signal.SIGPIPE, signal.SIGHUP):
        signal.signal(s, signal.SIG_DFL)
    signal.signal(signal.SIGINT, signal.default_int_handler)
    signal.pthread_sigmask(signal.SIG_SETMASK, [])
    log = req.get("log") or ""
    if log:
        fd = os.open(log, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(fd, 1)
        os.dup2(fd, 2)
        if fd > 2:
            os.close(fd)
    nul = os.open(os.devnull, os.O_RDONLY)
    os.dup2(nul, 0)
    if nul > 0:
        os.close(nul)
    cwd = req.get("cwd") or ""
    if cwd:
        try:
            os.chdir(cwd)
        except OSError as e:
            print(f"pto-zygote: chdir({cwd}): {e}", file=sys.stderr)
    cpus = [int(c) for c in req.get("cpus") or []]
    if cpus:
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            pass
    env = {str(k): str(v) for k, v in (req.get("env") or {}).items()}
    # c10d's libuv TCPStore server does not survive being started in a
    # forked interpreter: measured on this image, 3 of 4 two-rank gloo
    # rendezvous hung with rank 0 inside TCPStore() while the peer had
    # connected; the classic store backend passed every run.  A pod that
    # sets USE_LIBUV itself keeps its choice.
    env.setdefault("USE_LIBUV", "0")
    os.environ.clear()
    os.environ.update(env)
    if env.get("PTO_FAULTHANDLER"):  # debugging: SIGUSR2 dumps every thread's Python stack to the log
        import faulthandler

        faulthandler.register(signal.SIGUSR2, all_threads=True)
    # the intra-op pool was sized when the zygote imported torch; honour the
    # container's OMP_NUM_THREADS as a fresh interpreter would
    nthreads = env.get("OMP_NUM_THREADS", "")
    if nthreads.isdigit() and int(nthreads) > 0 and "torch" in sys.modules:
        sys.modules["torch"].set_num_threads(int(nthreads))
    argv = list(req["argv"])
    i = 1
    unbuffered = bool(env.get("PYTHONUNBUFFERED"))
    while argv[i] in _ELIGIBLE_FLAGS:
        unbuffered = unbuffered or argv[i] == "-u"
        i += 1
    # fresh stdio objects on the new fds, buffered as the interpreter would
    # have set them up from PYTHONUNBUFFERED / -u
    sys.stdin = io.TextIOWrapper(io.FileIO(0, "r", closefd=False), encoding="utf-8")
    for n, fd in (("stdout", 1), ("stderr", 2)):
        raw = io.FileIO(fd, "w", closefd=False)
        stream = io.TextIOWrapper(raw if unbuffered else io.BufferedWriter(raw), encoding="utf-8",
                                  errors="backslashreplace", line_buffering=(not unbuffered) or n == "stderr",
                                  write_through=unbuffered)
        setattr(sys, n, stream)
        setattr(sys, f"__{n}__", stream)
    extra_path = [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p]
    import runpy

    # startup evidence for the trainer's own breakdown (train/mnist.py)
    os.environ["PTO_ZYGOTE_T"] = f"{t_enter:.6f},{time.time():.6f}"

    code = 0
    try:
        if argv[i] == "-m":
            sys.argv = [argv[i + 1]] + argv[i + 2:]
            sys.path[0:0] = [os.getcwd()] + extra_path
            runpy.run_module(argv[i + 1], run_name="__main__", alter_sys=True)
        else:
            script = argv[i]
            sys.argv = argv[i:]
            sys.path[0:0] = [os.path.dirname(os.path.abspath(script))] + extra_path
            runpy.run_path(script, run_name="__main__")
    except SystemExit as e:
        if e.code is None:
            code = 0
        elif isinstance(e.code, int):
            code = e.code
        else:
            print(e.code, file=sys.stderr)
            code = 1
    except KeyboardInterrupt:
        code = 128 + signal.SIGINT
    except BaseException:  # noqa: BLE001 - what the interpreter's top level does
        traceback.print_exc()
        code = 1
    try:
        import atexit

        atexit._run_exitfuncs()
    except Exception:  # noqa: BLE001
        pass
    for s in (sys.stdout, sys.stderr):
        try:
            s.flush()
        except Exception:  # noqa: BLE001
            pass
    return code & 0xFF


def _spawn(req: dict, sock_fd: int) -> int:
    """Double fork; returns the container's pid (re-parented to the agent)."""
    r, w = os.pipe()
    mid = os.fork()
    if mid == 0:
        try:
            os.close(r)
            pid = os.fork()
            if pid == 0:
                code = 1
                try:
                    os.close(w)
                    os.close(sock_fd)
                    code = _run_container(req)
                except BaseException:  # noqa: BLE001 - setup failed before the program ran
                    traceback.print_exc()
                finally:
                    os._exit(code)
            os.write(w, str(pid).encode())
        finally:
            os._exit(0)
    os.close(w)
    data = b""
    while True:
        chunk = os.read(r, 64)
        if not chunk:
            break
        data += chunk
    os.close(r)
    os.waitpid(mid, 0)
    if not data:
        raise RuntimeError("zygote: container fork failed")
    return int(data)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="pto warm interpreter (started by pto-node-agent)")
    ap.add_argument("--fd", type=int, required=True, help="inherited socket to the agent")
    ap.add_argument("--spare", action="store_true",
                    help="warm SPARE: run the first requested container in this very process (no fork), for "
                         "containers that must not start in a forked interpreter (the agent starts the next one)")
    args = ap.parse_args(argv)
    # interactive signals go to the agent; the zygote ends when its socket does
    signal.signal(signal.SIGINT, signal.SIG_IGN)
    _preload()
    rf = os.fdopen(args.fd, "rb", buffering=0)

    def reply(obj):
        os.write(args.fd, (json.dumps(obj) + "\n").encode())

    reply({"ready": True, "pid": os.getpid(), "python": sys.executable})
    buf = b""
    while True:
        chunk = rf.read(65536)
        if not chunk:
            return 0
        buf += chunk
        while b"\n" in buf:
            line, buf = buf.split(b"\n", 1)
            if not line.strip():
                continue
            try:
                req = json.loads(line)
                if args.spare:
                    # this process becomes the container: it is the agent's
                    # own child, so it is reaped, killed and restarted like
                    # an exec'ed one
                    reply({"ok": True, "pid": os.getpid(), "seq": req.get("seq")})
                    rf.close()
                    try:
                        os.close(args.fd)
                    except OSError:
                        pass
                    os._exit(_run_container(req))
                reply({"ok": True, "pid": _spawn(req, args.fd), "seq": req.get("seq")})
            except Exception as e:  # noqa: BLE001 - reported; the agent falls back to fork/exec
                reply({"ok": False, "error": f"{type(e).__name__}: {e}"})


if __name__ == "__main__":
    sys.exit(main())
