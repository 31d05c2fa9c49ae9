"""In-memory, watchable object store with Kubernetes API semantics.

This replaces kube-apiserver + etcd for a single MI355X node.
Semantics reproduced (what the controller and SDK rely on):

* objects are JSON dicts addressed by (resource, namespace, name);
* every write bumps a global ``resourceVersion``; ``metadata.uid``,
  ``creationTimestamp`` and ``generation`` are server-assigned;
* optimistic concurrency: an update carrying a stale ``resourceVersion``
  fails with 409 Conflict;
* status subresource isolation: ``update`` ignores ``.status`` for
  resources with a status subresource, ``update_status`` touches only it;
* ``delete`` with background propagation: dependents whose
  ``ownerReferences`` name the deleted uid are garbage-collected (the
  cascade the reference gets from the kube GC);
* ``watch(resourceVersion=rv)`` replays buffered events after ``rv`` then
  streams ADDED/MODIFIED/DELETED, like a kube watch;
* label selectors (``a=b,c!=d,e``) on list/watch;
* optional append-only JSONL write-ahead log for restart durability.
"""
from __future__ import annotations

import copy
import json
import os
import queue
import threading
import time
import uuid
from collections import deque
from dataclasses import dataclass

from ..api.types import now_rfc3339

# response header carrying an object's sub-second creation time
# (creationTimestamp has 1 s resolution); read by the node manager for the
# submit -> first-step metric
CREATED_UNIX_HEADER = "X-Pto-Created-Unix"


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str):
        super().__init__(message)
        self.code, self.reason, self.message = code, reason, message

    def status(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": self.message,
                "reason": self.reason, "code": self.code}


def NotFound(resource, name):
    return ApiError(404, "NotFound", f'{resource} "{name}" not found')


def AlreadyExists(resource, name):
    return ApiError(409, "AlreadyExists", f'{resource} "{name}" already exists')


def Conflict(resource, name):
    return ApiError(409, "Conflict", f'Operation cannot be fulfilled on {resource} "{name}": the object has been '
                                     f'modified; please apply your changes to the latest version and try again')


def Invalid(resource, name, msg):
    return ApiError(422, "Invalid", f'{resource} "{name}" is invalid: {msg}')


# resource -> (apiVersion, kind, namespaced, has_status_subresource)
RESOURCES = {
    "pytorchjobs": ("kubeflow.org/v1", "PyTorchJob", True, True),
    "pods": ("v1", "Pod", True, True),
    "services": ("v1", "Service", True, True),
    "events": ("v1", "Event", True, False),
    "endpoints": ("v1", "Endpoints", True, False),
    "configmaps": ("v1", "ConfigMap", True, False),
    "leases": ("coordination.k8s.io/v1", "Lease", True, False),
    "podgroups": ("scheduling.incubator.k8s.io/v1alpha1", "PodGroup", True, True),
    "customresourcedefinitions": ("apiextensions.k8s.io/v1beta1", "CustomResourceDefinition", False, True),
    "nodes": ("v1", "Node", False, True),
}


def parse_selector(sel: str | dict | None):
    """Label selector -> list of (key, op, value) with op in {=, !=, exists}."""
    if not sel:
        return []
    if isinstance(sel, dict):
        return [(k, "=", str(v)) for k, v in sel.items()]
    out = []
    for term in sel.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in term:
            k, v = term.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in term:
            k, v = term.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        else:
            out.append((term, "exists", None))
    return out


def match_selector(labels: dict | None, terms) -> bool:
    labels = labels or {}
    for k, op, v in terms:
        if op == "=" and labels.get(k) != v:
            return False
        if op == "!=" and labels.get(k) == v:
            return False
        if op == "exists" and k not in labels:
            return False
    return True


def match_fields(obj: dict, fields: str | None) -> bool:
    if not fields:
        return True
    for term in fields.split(","):
        if "=" not in term:
            continue
        k, v = term.split("=", 1)
        cur = obj
        for part in k.strip().split("."):
            cur = cur.get(part, {}) if isinstance(cur, dict) else {}
        if str(cur) != v.strip():
            return False
    return True


@dataclass
class WatchEvent:
    type: str  # ADDED | MODIFIED | DELETED | BOOKMARK | ERROR
    resource: str
    object: dict
    rv: int


class Watch:
    """A live watch: iterate (blocking) or ``get(timeout)``; ``stop()``."""

    def __init__(self, store, resource, namespace, selector, fields):
        self.store, self.resource, self.namespace = store, resource, namespace
        self.terms = parse_selector(selector)
        self.fields = fields
        self.q: queue.Queue = queue.Queue()
        self.closed = False

    def _offer(self, ev: WatchEvent):
        if self.closed or ev.resource != self.resource:
            return
        md = ev.object.get("metadata", {})
        if self.namespace and md.get("namespace") != self.namespace:
            return
        if not match_selector(md.get("labels"), self.terms) or not match_fields(ev.object, self.fields):
            return
        self.q.put(ev)

    def get(self, timeout: float | None = None) -> WatchEvent | None:
        try:
            return self.q.get(timeout=timeout)
        except queue.Empty:
            return None

    def __iter__(self):
        while not self.closed:
            ev = self.get(timeout=0.5)
            if ev is not None:
                yield ev

    def stop(self):
        self.closed = True
        self.store._remove_watch(self)


class Store:
    HISTORY = 10000

    def __init__(self, wal_path: str | None = None):
        self._lock = threading.RLock()
        self._objs: dict[tuple[str, str, str], dict] = {}
        self._created_unix: dict[str, float] = {}  # uid -> creation time (s, sub-second)
        self._rv = 0
        self._history: deque[WatchEvent] = deque(maxlen=self.HISTORY)
        self._watches: list[Watch] = []
        self._wal = None
        self._wal_path = wal_path
        if wal_path:
            self._replay_wal(wal_path)
            self._wal = open(wal_path, "a", buffering=1)

    # ------------------------------------------------------------------ WAL
    def _replay_wal(self, path):
        if not os.path.exists(path):
            return
        with open(path) as f:
            for line in f:
                try:
                    rec = json.loads(line)
                except json.JSONDecodeError:
                    continue  # torn tail write
                key = (rec["r"], rec["ns"], rec["n"])
                if rec["op"] == "put":
                    self._objs[key] = rec["o"]
                else:
                    self._objs.pop(key, None)
                self._rv = max(self._rv, int(rec["rv"]))

    def _log(self, op, key, obj, rv):
        if self._wal:
            self._wal.write(json.dumps({"op": op, "r": key[0], "ns": key[1], "n": key[2], "o": obj, "rv": rv}) + "\n")

    # --------------------------------------------------------------- helpers
    @staticmethod
    def _check_resource(resource):
        if resource not in RESOURCES:
            raise ApiError(404, "NotFound", f"the server could not find the requested resource ({resource})")
        return RESOURCES[resource]

    def _key(self, resource, namespace, name):
        namespaced = self._check_resource(resource)[2]
        return resource, (namespace or "default") if namespaced else "", name

    def _emit(self, etype, resource, obj):
        ev = WatchEvent(etype, resource, copy.deepcopy(obj), int(obj["metadata"]["resourceVersion"]))
        self._history.append(ev)
        for w in list(self._watches):
            w._offer(ev)

    def _bump(self, obj):
        self._rv += 1
        obj["metadata"]["resourceVersion"] = str(self._rv)
        return self._rv

    @property
    def resource_version(self) -> int:
        return self._rv

    # ------------------------------------------------------------------ CRUD
    def create(self, resource: str, obj: dict, namespace: str | None = None) -> dict:
        api_version, kind, namespaced, _ = self._check_resource(resource)
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise Invalid(resource, "", "metadata.name: Required value")
        if namespaced:
            md["namespace"] = namespace or md.get("namespace") or "default"
        else:
            md.pop("namespace", None)
        obj.setdefault("apiVersion", api_version)
        obj.setdefault("kind", kind)
        with self._lock:
            key = self._key(resource, md.get("namespace"), md["name"])
            if key in self._objs:
                raise AlreadyExists(resource, md["name"])
            md["uid"] = str(uuid.uuid4())
            md["creationTimestamp"] = now_rfc3339()
            # sub-second creation time for the submit -> first-step metric,
            # kept next to the object (never written into it: the user's
            # object comes back as submitted); served as a response header
            self._created_unix[md["uid"]] = time.time()
            md["generation"] = 1
            md.pop("deletionTimestamp", None)
            rv = self._bump(obj)
            self._objs[key] = obj
            self._log("put", key, obj, rv)
            self._emit("ADDED", resource, obj)
            return copy.deepcopy(obj)

    def created_unix(self, uid: str | None) -> float | None:
        """Sub-second creation time of the object with this uid (objects
        created by this process only; None otherwise)."""
        return self._created_unix.get(uid) if uid else None

    def get(self, resource: str, namespace: str | None, name: str) -> dict:
        with self._lock:
            o = self._objs.get(self._key(resource, namespace, name))
            if o is None:
                raise NotFound(resource, name)
            return copy.deepcopy(o)

    def list(self, resource: str, namespace: str | None = None, label_selector=None, field_selector=None) -> dict:
        api_version, kind, namespaced, _ = self._check_resource(resource)
        terms = parse_selector(label_selector)
        with self._lock:
            items = [copy.deepcopy(o) for (r, ns, _), o in sorted(self._objs.items())
                     if r == resource and (not namespace or not namespaced or ns == namespace)
                     and match_selector(o.get("metadata", {}).get("labels"), terms) and match_fields(o, field_selector)]
            return {"apiVersion": api_version, "kind": kind + "List", "metadata": {"resourceVersion": str(self._rv)},
                    "items": items}

    def _write(self, resource, obj, namespace, status_only: bool):
        api_version, kind, namespaced, has_status = self._check_resource(resource)
        md = obj.get("metadata", {})
        name = md.get("name")
        with self._lock:
            key = self._key(resource, namespace or md.get("namespace"), name)
            cur = self._objs.get(key)
            if cur is None:
                raise NotFound(resource, name)
            rv = md.get("resourceVersion")
            if rv and str(rv) != cur["metadata"]["resourceVersion"]:
                raise Conflict(resource, name)
            new = copy.deepcopy(cur)
            if status_only:
                new["status"] = copy.deepcopy(obj.get("status", {}))
            else:
                for k, v in obj.items():
                    if k in ("metadata", "status") or (k == "status" and has_status):
                        continue
                    new[k] = copy.deepcopy(v)
                for k in [k for k in new if k not in obj and k not in ("metadata", "status", "apiVersion", "kind")]:
                    new.pop(k)
                if not has_status and "status" in obj:
                    new["status"] = copy.deepcopy(obj["status"])
                # mutable metadata
                for mk in ("labels", "annotations", "ownerReferences", "finalizers"):
                    if mk in md:
                        new["metadata"][mk] = copy.deepcopy(md[mk])
                    else:
                        new["metadata"].pop(mk, None)
                if new.get("spec") != cur.get("spec"):
                    new["metadata"]["generation"] = int(cur["metadata"].get("generation", 1)) + 1
            if new == cur:
                return copy.deepcopy(cur)
            rv = self._bump(new)
            self._objs[key] = new
            self._log("put", key, new, rv)
            self._emit("MODIFIED", resource, new)
            return copy.deepcopy(new)

    def update(self, resource: str, obj: dict, namespace: str | None = None) -> dict:
        return self._write(resource, obj, namespace, status_only=False)

    def update_status(self, resource: str, obj: dict, namespace: str | None = None) -> dict:
        return self._write(resource, obj, namespace, status_only=True)

    def patch(self, resource: str, namespace: str | None, name: str, patch: dict, subresource: str | None = None):
        """JSON merge patch (RFC 7386)."""
        with self._lock:
            cur = self.get(resource, namespace, name)
            merged = _merge_patch(cur, patch)
            merged["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            if subresource == "status":
                return self.update_status(resource, merged, namespace)
            out = self.update(resource, merged, namespace)
            if "status" in patch and RESOURCES[resource][3]:
                out = self.update_status(resource, _merge_patch(out, {"status": patch["status"]}), namespace)
            return out

    def delete(self, resource: str, namespace: str | None, name: str, propagation: str = "Background") -> dict:
        with self._lock:
            key = self._key(resource, namespace, name)
            cur = self._objs.pop(key, None)
            if cur is None:
                raise NotFound(resource, name)
            self._created_unix.pop(cur["metadata"].get("uid"), None)
            cur["metadata"]["deletionTimestamp"] = now_rfc3339()
            rv = self._bump(cur)
            self._log("del", key, None, rv)
            self._emit("DELETED", resource, cur)
            if propagation != "Orphan":
                self._gc(cur["metadata"].get("uid"))
            return copy.deepcopy(cur)

    def _gc(self, owner_uid):
        """Cascade-delete dependents (ownerReferences.uid == owner_uid)."""
        if not owner_uid:
            return
        victims = [k for k, o in self._objs.items()
                   if any(r.get("uid") == owner_uid for r in o.get("metadata", {}).get("ownerReferences") or [])]
        for r, ns, n in victims:
            if (r, ns, n) in self._objs:
                self.delete(r, ns or None, n)

    # ----------------------------------------------------------------- watch
    def watch(self, resource: str, namespace: str | None = None, label_selector=None, field_selector=None,
              resource_version: str | int | None = None) -> Watch:
        self._check_resource(resource)
        w = Watch(self, resource, namespace, label_selector, field_selector)
        with self._lock:
            if resource_version not in (None, "", "0", 0):
                since = int(resource_version)
                if self._history and since < self._history[0].rv - 1:
                    w.q.put(WatchEvent("ERROR", resource, {"kind": "Status", "code": 410, "reason": "Expired",
                                                           "message": "too old resource version"}, since))
                else:
                    for ev in self._history:
                        if ev.rv > since:
                            w._offer(ev)
            self._watches.append(w)
        return w

    def _remove_watch(self, w):
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    # ---------------------------------------------------------------- events
    def record_event(self, involved: dict, etype: str, reason: str, message: str, component="pytorch-operator"):
        """Create a core/v1 Event (aggregating repeats like kube's recorder)."""
        md = involved.get("metadata", {})
        ns = md.get("namespace", "default")
        base = f"{md.get('name', 'unknown')}.{reason}".lower()
        with self._lock:
            for (r, n, nm), o in self._objs.items():
                if r == "events" and n == ns and nm.startswith(base) and o.get("message") == message and \
                        o.get("involvedObject", {}).get("uid") == md.get("uid"):
                    o = copy.deepcopy(o)
                    o["count"] = int(o.get("count", 1)) + 1
                    o["lastTimestamp"] = now_rfc3339()
                    return self.update("events", o, ns)
            ev = {
                "metadata": {"name": f"{base}.{uuid.uuid4().hex[:10]}", "namespace": ns},
                "involvedObject": {"kind": involved.get("kind"), "name": md.get("name"), "namespace": ns,
                                   "uid": md.get("uid"), "apiVersion": involved.get("apiVersion")},
                "type": etype, "reason": reason, "message": message, "count": 1,
                "source": {"component": component},
                "firstTimestamp": now_rfc3339(), "lastTimestamp": now_rfc3339(),
            }
            return self.create("events", ev, ns)

    def close(self):
        if self._wal:
            self._wal.close()
            self._wal = None


def _merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = _merge_patch(out.get(k), v)
    return out


def wait_for(predicate, timeout: float = 10.0, interval: float = 0.02) -> bool:
    end = time.time() + timeout
    while time.time() < end:
        if predicate():
            return True
        time.sleep(interval)
    return predicate()
