"""List+watch informer with an indexed cache.

Equivalent of client-go's SharedIndexInformer as used by the reference
(pod/service informers from the kube informer factory, 12 h resync, and
the unstructured PyTorchJob informer with a 30 s resync,
``pkg/controller.v1/pytorch/informer.go:24-55``).  Handlers are called on
the informer thread in event order: ``on_add(obj)``,
``on_update(old, new)``, ``on_delete(obj)``; a periodic resync replays
``on_update(obj, obj)`` for every cached object.
"""
from __future__ import annotations

import logging
import threading
import time

from ..api.types import key_of

log = logging.getLogger(__name__)


class Informer:
    def __init__(self, client, resource: str, namespace: str | None = None, resync_period: float = 0.0,
                 label_selector=None):
        self.client, self.resource, self.namespace = client, resource, namespace
        self.resync_period = resync_period
        self.label_selector = label_selector
        self._cache: dict[str, dict] = {}
        self._lock = threading.RLock()
        self._handlers = []
        self._synced = threading.Event()
        self._stop = threading.Event()
        self._thread = None
        self._watch = None

    # ---- cache (lister) API
    def add_event_handler(self, on_add=None, on_update=None, on_delete=None):
        self._handlers.append((on_add, on_update, on_delete))

    def get_by_key(self, key: str):
        with self._lock:
            return self._cache.get(key)

    def list(self, namespace: str | None = None):
        with self._lock:
            return [o for o in self._cache.values()
                    if namespace is None or o.get("metadata", {}).get("namespace") == namespace]

    def has_synced(self) -> bool:
        return self._synced.is_set()

    def wait_for_sync(self, timeout: float = 30.0) -> bool:
        return self._synced.wait(timeout)

    def replace_in_cache(self, obj):
        """Write-through into the cache (mirrors the reference mutating the
        cached unstructured object in addPyTorchJob, job.go:104)."""
        with self._lock:
            self._cache[key_of(obj)] = obj

    # ---- run loop
    def start(self):
        self._thread = threading.Thread(target=self._run, name=f"informer-{self.resource}", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._watch is not None:
            try:
                self._watch.stop()
            except Exception:
                pass

    def _dispatch(self, kind, *args):
        for h in self._handlers:
            fn = h[{"add": 0, "update": 1, "delete": 2}[kind]]
            if fn is None:
                continue
            try:
                fn(*args)
            except Exception:  # a handler error must not kill the informer
                log.exception("informer %s handler %s failed", self.resource, kind)

    def _relist(self) -> str:
        lst = self.client.list(self.resource, self.namespace, self.label_selector)
        fresh = {key_of(o): o for o in lst.get("items", [])}
        with self._lock:
            old = self._cache
            self._cache = dict(fresh)
        for k, o in fresh.items():
            if k in old:
                if old[k].get("metadata", {}).get("resourceVersion") != o["metadata"].get("resourceVersion"):
                    self._dispatch("update", old[k], o)
            else:
                self._dispatch("add", o)
        for k, o in old.items():
            if k not in fresh:
                self._dispatch("delete", o)
        self._synced.set()
        return lst.get("metadata", {}).get("resourceVersion", "0")

    def _run(self):
        rv = None
        last_resync = time.monotonic()
        while not self._stop.is_set():
            try:
                if rv is None:
                    rv = self._relist()
                self._watch = self.client.watch(self.resource, self.namespace, self.label_selector,
                                                resource_version=rv, timeout_seconds=max(self.resync_period, 5)
                                                if self.resync_period else 60)
                for etype, obj in self._watch:
                    if self._stop.is_set():
                        break
                    if etype == "ERROR":
                        rv = None  # 410 Gone -> relist
                        break
                    rv = obj.get("metadata", {}).get("resourceVersion", rv)
                    k = key_of(obj)
                    if etype == "ADDED":
                        with self._lock:
                            old = self._cache.get(k)
                            self._cache[k] = obj
                        if old is None:
                            self._dispatch("add", obj)
                        else:
                            self._dispatch("update", old, obj)
                    elif etype == "MODIFIED":
                        with self._lock:
                            old = self._cache.get(k)
                            self._cache[k] = obj
                        self._dispatch("update", old if old is not None else obj, obj)
                    elif etype == "DELETED":
                        with self._lock:
                            self._cache.pop(k, None)
                        self._dispatch("delete", obj)
                    if self.resync_period and time.monotonic() - last_resync > self.resync_period:
                        break
                if self.resync_period and time.monotonic() - last_resync > self.resync_period:
                    last_resync = time.monotonic()
                    with self._lock:
                        objs = list(self._cache.values())
                    for o in objs:
                        self._dispatch("update", o, o)
            except Exception as e:  # connection errors: back off and relist
                if self._stop.is_set():
                    break
                log.warning("informer %s: watch error %s; relisting", self.resource, e)
                rv = None
                time.sleep(0.5)
