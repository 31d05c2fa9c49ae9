"""Rate-limited work queue with client-go semantics.

Reference: vendored ``k8s.io/client-go/util/workqueue`` as configured by
``DefaultControllerRateLimiter`` (``default_rate_limiters.go:39-45``):
per-item exponential backoff 5 ms -> 1000 s, MAX'd with a global token
bucket (10 qps, burst 100).  Queue guarantees: an item is never processed
by two workers at once (dirty/processing sets), re-adds while processing
are deferred until ``done``; ``num_requeues`` is the retry counter the
controller uses for ``backoffLimit`` (``controller.go:392``).
"""
from __future__ import annotations

import heapq
import threading
import time


class ItemExponentialFailureRateLimiter:
    def __init__(self, base_delay=0.005, max_delay=1000.0):
        self.base, self.max = base_delay, max_delay
        self.failures: dict = {}
        self._lock = threading.Lock()

    def when(self, item) -> float:
        with self._lock:
            n = self.failures.get(item, 0)
            self.failures[item] = n + 1
        d = self.base * (2 ** n)
        return min(d, self.max)

    def num_requeues(self, item) -> int:
        with self._lock:
            return self.failures.get(item, 0)

    def forget(self, item):
        with self._lock:
            self.failures.pop(item, None)


class BucketRateLimiter:
    """Token bucket (golang.org/x/time/rate semantics: reservation delay)."""

    def __init__(self, qps=10.0, burst=100):
        self.qps, self.burst = float(qps), float(burst)
        self.tokens = float(burst)
        self.last = time.monotonic()
        self._lock = threading.Lock()

    def when(self, item) -> float:
        with self._lock:
            now = time.monotonic()
            self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
            self.last = now
            self.tokens -= 1.0
            if self.tokens >= 0:
                return 0.0
            return -self.tokens / self.qps

    def num_requeues(self, item) -> int:
        return 0

    def forget(self, item):
        pass


class MaxOfRateLimiter:
    def __init__(self, *limiters):
        self.limiters = limiters

    def when(self, item) -> float:
        return max(l.when(item) for l in self.limiters)

    def num_requeues(self, item) -> int:
        return max(l.num_requeues(item) for l in self.limiters)

    def forget(self, item):
        for l in self.limiters:
            l.forget(item)


def default_controller_rate_limiter():
    return MaxOfRateLimiter(ItemExponentialFailureRateLimiter(0.005, 1000.0), BucketRateLimiter(10, 100))


class RateLimitingQueue:
    def __init__(self, name: str = "", rate_limiter=None):
        self.name = name
        self.rl = rate_limiter or default_controller_rate_limiter()
        self._cond = threading.Condition()
        self._queue: list = []
        self._dirty: set = set()
        self._processing: set = set()
        self._delayed: list = []  # heap of (ready_at, seq, item)
        self._seq = 0
        self._shutdown = False
        self._timer = threading.Thread(target=self._delay_loop, name=f"wq-{name}-delay", daemon=True)
        self._timer.start()

    # ---- basic queue
    def add(self, item):
        with self._cond:
            if self._shutdown or item in self._dirty:
                return
            self._dirty.add(item)
            if item in self._processing:
                return
            self._queue.append(item)
            self._cond.notify_all()  # the delay thread waits on the same condition

    def __len__(self):
        with self._cond:
            return len(self._queue)

    def get(self, timeout: float | None = None):
        """Block for the next item. Returns (item, shutdown)."""
        with self._cond:
            end = None if timeout is None else time.monotonic() + timeout
            while not self._queue and not self._shutdown:
                rem = None if end is None else end - time.monotonic()
                if rem is not None and rem <= 0:
                    return None, False
                self._cond.wait(rem)
            if not self._queue:
                return None, True
            item = self._queue.pop(0)
            self._processing.add(item)
            self._dirty.discard(item)
            return item, False

    def done(self, item):
        with self._cond:
            self._processing.discard(item)
            if item in self._dirty:
                self._queue.append(item)
                self._cond.notify_all()  # the delay thread waits on the same condition

    def shutdown(self):
        with self._cond:
            self._shutdown = True
            self._cond.notify_all()

    @property
    def shutting_down(self):
        return self._shutdown

    # ---- delaying
    def add_after(self, item, delay: float):
        if delay <= 0:
            self.add(item)
            return
        with self._cond:
            if self._shutdown:
                return
            self._seq += 1
            heapq.heappush(self._delayed, (time.monotonic() + delay, self._seq, item))
            self._cond.notify_all()

    def _delay_loop(self):
        while True:
            with self._cond:
                if self._shutdown:
                    return
                now = time.monotonic()
                ready = []
                while self._delayed and self._delayed[0][0] <= now:
                    ready.append(heapq.heappop(self._delayed)[2])
                wait = (self._delayed[0][0] - now) if self._delayed else 0.5
            for it in ready:
                self.add(it)
            with self._cond:
                if not self._shutdown:
                    self._cond.wait(min(max(wait, 0.001), 0.5))

    # ---- rate limiting
    def add_rate_limited(self, item):
        self.add_after(item, self.rl.when(item))

    def forget(self, item):
        self.rl.forget(item)

    def num_requeues(self, item) -> int:
        return self.rl.num_requeues(item)
