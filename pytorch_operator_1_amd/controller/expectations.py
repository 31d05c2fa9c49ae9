"""Controller expectations (vendored ``k8s.io/kubernetes/pkg/controller/
controller_utils.go:68-284``).

A sync is skipped until the informer has observed the pod/service
creations and deletions the previous sync issued, or until the
expectation is older than 5 minutes.  Note the reference semantics kept
here: ``expect_creations`` *sets* the pending add count (it does not
increment), and ``satisfied`` is True for unknown keys.
"""
from __future__ import annotations

import threading
import time

from ..api.constants import EXPECTATIONS_TIMEOUT_S


class _Exp:
    __slots__ = ("add", "dele", "ts")

    def __init__(self, add, dele):
        self.add, self.dele, self.ts = add, dele, time.monotonic()

    def fulfilled(self):
        return self.add <= 0 and self.dele <= 0

    def expired(self, ttl):
        return time.monotonic() - self.ts > ttl


class ControllerExpectations:
    def __init__(self, ttl: float = EXPECTATIONS_TIMEOUT_S):
        self.ttl = ttl
        self._m: dict[str, _Exp] = {}
        self._lock = threading.Lock()

    def get(self, key):
        with self._lock:
            e = self._m.get(key)
            return None if e is None else (e.add, e.dele)

    def satisfied(self, key) -> bool:
        with self._lock:
            e = self._m.get(key)
            if e is None:
                return True  # no expectations recorded: sync
            return e.fulfilled() or e.expired(self.ttl)

    def set_expectations(self, key, add, dele):
        with self._lock:
            self._m[key] = _Exp(add, dele)

    def expect_creations(self, key, adds):
        self.set_expectations(key, adds, 0)

    def expect_deletions(self, key, dels):
        self.set_expectations(key, 0, dels)

    def _lower(self, key, add, dele):
        with self._lock:
            e = self._m.get(key)
            if e is not None:
                e.add -= add
                e.dele -= dele

    def raise_expectations(self, key, add, dele):
        with self._lock:
            e = self._m.get(key)
            if e is not None:
                e.add += add
                e.dele += dele

    def creation_observed(self, key):
        self._lower(key, 1, 0)

    def deletion_observed(self, key):
        self._lower(key, 0, 1)

    def delete_expectations(self, key):
        with self._lock:
            self._m.pop(key, None)
