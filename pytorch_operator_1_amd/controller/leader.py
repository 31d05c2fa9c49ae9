"""Leader election on a ``coordination.k8s.io/v1`` Lease.

Reference: ``cmd/pytorch-operator.v1/app/server.go:146-171`` — lock name
``pytorch-operator`` in ``$KUBEFLOW_NAMESPACE``, lease 15 s / renew 5 s /
retry 3 s; on becoming leader the ``pytorch_operator_is_leader`` gauge is
set and the controller runs; losing the lease is fatal (the process exits
and its supervisor restarts it).  The reference uses an Endpoints lock; a
Lease object carries the same holder/expiry information.
"""
from __future__ import annotations

import logging
import os
import socket
import threading
import time
import uuid

from ..api import constants as C
from ..api.types import now_rfc3339, parse_rfc3339
from ..apiserver.store import ApiError

log = logging.getLogger("pytorch-operator")


class LeaderElector:
    def __init__(self, client, name: str = "pytorch-operator", namespace: str | None = None,
                 identity: str | None = None, lease_s: float = C.LEADER_LEASE_S, renew_s: float = C.LEADER_RENEW_S,
                 retry_s: float = C.LEADER_RETRY_S):
        self.client = client
        self.name = name
        self.namespace = namespace or os.environ.get(C.ENV_KUBEFLOW_NAMESPACE, "default")
        self.identity = identity or f"{socket.gethostname()}_{uuid.uuid4().hex[:8]}"
        self.lease_s, self.renew_s, self.retry_s = lease_s, renew_s, retry_s
        self._stop = threading.Event()
        self.is_leader = False

    def _try_acquire_or_renew(self) -> bool:
        now = time.time()
        try:
            lease = self.client.get("leases", self.namespace, self.name)
        except ApiError as e:
            if e.code != 404:
                return False
            obj = {"metadata": {"name": self.name, "namespace": self.namespace},
                   "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": self.lease_s,
                            "acquireTime": now_rfc3339(), "renewTime": now_rfc3339(), "renewTimeUnix": now,
                            "leaseTransitions": 0}}
            try:
                self.client.create("leases", obj, self.namespace)
                return True
            except ApiError:
                return False
        spec = lease.get("spec", {})
        holder = spec.get("holderIdentity")
        renewed = spec.get("renewTimeUnix") or parse_rfc3339(spec.get("renewTime")) or 0
        expired = now > float(renewed) + float(spec.get("leaseDurationSeconds", self.lease_s))
        if holder != self.identity and not expired:
            return False
        if holder != self.identity:
            spec["leaseTransitions"] = int(spec.get("leaseTransitions", 0)) + 1
            spec["acquireTime"] = now_rfc3339()
        spec.update(holderIdentity=self.identity, renewTime=now_rfc3339(), renewTimeUnix=now,
                    leaseDurationSeconds=self.lease_s)
        lease["spec"] = spec
        try:
            self.client.update("leases", lease, self.namespace)  # optimistic concurrency on resourceVersion
            return True
        except ApiError:
            return False

    def run(self, on_started_leading, on_stopped_leading=None, block: bool = True):
        """Block until leadership is acquired, call ``on_started_leading``,
        keep renewing; on loss call ``on_stopped_leading`` (default: exit)."""

        def loop():
            while not self._stop.is_set():
                if self._try_acquire_or_renew():
                    break
                self._stop.wait(self.retry_s)
            if self._stop.is_set():
                return
            self.is_leader = True
            log.info("became leader: %s", self.identity)
            threading.Thread(target=on_started_leading, daemon=True).start()
            last_ok = time.time()
            while not self._stop.is_set():
                self._stop.wait(self.renew_s)
                if self._try_acquire_or_renew():
                    last_ok = time.time()
                elif time.time() - last_ok > self.lease_s:
                    self.is_leader = False
                    log.error("leader election lost")
                    if on_stopped_leading:
                        on_stopped_leading()
                    else:
                        os._exit(1)  # reference: log.Fatalf
                    return

        if block:
            loop()
        else:
            t = threading.Thread(target=loop, name="leader-election", daemon=True)
            t.start()
            return t

    def stop(self):
        self._stop.set()
