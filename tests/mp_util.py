"""Collect results from spawned worker processes without outliving them: a
worker that dies (abort, segfault, uncaught exception) fails the test at
once with its exit code, instead of the parent blocking on the queue until
the pytest timeout hides what happened."""
import queue
import time


def collect(q, procs, n, timeout=100.0):
    out, deadline = [], time.monotonic() + timeout
    while len(out) < n:
        try:
            out.append(q.get(timeout=0.5))
            continue
        except queue.Empty:
            pass
        dead = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode not in (None, 0)]
        if dead:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise AssertionError(f"worker(s) died before reporting: (index, exit code) {dead}")
        if time.monotonic() > deadline:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise AssertionError(f"no result from {n - len(out)} worker(s) within {timeout:.0f} s "
                                 f"(alive: {[p.is_alive() for p in procs]})")
    return out
