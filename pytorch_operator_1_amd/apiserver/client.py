"""API clients used by the controller, node agent shim, SDK and CLI.

Two interchangeable transports with one interface:

* :class:`LocalClient` — direct calls into an in-process
  :class:`~.store.Store` (tests, the all-in-one daemon);
* :class:`RestClient` — HTTP against :class:`~.server.ApiServer` (or any
  server speaking the same paths), with streaming watches.

This is the equivalent of the reference's generated clientset
(``pkg/client/clientset/versioned/typed/pytorch/v1/pytorchjob.go:37-189``:
Get/List/Watch/Create/Update/UpdateStatus/Delete/DeleteCollection/Patch)
plus the core/v1 pieces the controller uses through client-go.
"""
from __future__ import annotations

import json
import threading
from typing import Iterator

from .store import RESOURCES, ApiError, Store


class Client:
    """Abstract interface (documentation only)."""

    def create(self, resource, obj, namespace=None): ...
    def get(self, resource, namespace, name): ...
    def list(self, resource, namespace=None, label_selector=None, field_selector=None): ...
    def update(self, resource, obj, namespace=None): ...
    def update_status(self, resource, obj, namespace=None): ...
    def patch(self, resource, namespace, name, patch, subresource=None): ...
    def delete(self, resource, namespace, name, propagation="Background"): ...
    def watch(self, resource, namespace=None, label_selector=None, resource_version=None,
              timeout_seconds=None): ...
    def record_event(self, involved, etype, reason, message): ...


class LocalClient(Client):
    def __init__(self, store: Store):
        self.store = store

    def create(self, resource, obj, namespace=None):
        return self.store.create(resource, obj, namespace)

    def get(self, resource, namespace, name):
        return self.store.get(resource, namespace, name)

    def list(self, resource, namespace=None, label_selector=None, field_selector=None):
        return self.store.list(resource, namespace, label_selector, field_selector)

    def update(self, resource, obj, namespace=None):
        return self.store.update(resource, obj, namespace)

    def update_status(self, resource, obj, namespace=None):
        return self.store.update_status(resource, obj, namespace)

    def patch(self, resource, namespace, name, patch, subresource=None):
        return self.store.patch(resource, namespace, name, patch, subresource)

    def delete(self, resource, namespace, name, propagation="Background"):
        return self.store.delete(resource, namespace, name, propagation)

    def watch(self, resource, namespace=None, label_selector=None, resource_version=None, timeout_seconds=None):
        w = self.store.watch(resource, namespace, label_selector, None, resource_version)
        return _LocalWatch(w, timeout_seconds)

    def record_event(self, involved, etype, reason, message):
        return self.store.record_event(involved, etype, reason, message)

    def created_unix(self, resource, namespace, name) -> float | None:
        """Sub-second creation time of an object (None if unknown)."""
        return self.store.created_unix(self.store.get(resource, namespace, name)["metadata"].get("uid"))


class _LocalWatch:
    def __init__(self, w, timeout):
        self.w, self.timeout = w, timeout

    def __iter__(self) -> Iterator[tuple[str, dict]]:
        import time

        end = time.time() + self.timeout if self.timeout else None
        while not self.w.closed:
            if end and time.time() > end:
                break
            ev = self.w.get(timeout=0.2)
            if ev is not None:
                yield ev.type, ev.object

    def stop(self):
        self.w.stop()


def _paths():
    out = {}
    for r, (api_version, _, namespaced, _) in RESOURCES.items():
        prefix = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        out[r] = (prefix, namespaced)
    return out


class RestClient(Client):
    def __init__(self, base_url: str = "http://127.0.0.1:8080", token: str | None = None, timeout: float = 30.0,
                 qps: float | None = None):
        import requests

        self.base = base_url.rstrip("/")
        self.session = requests.Session()
        self.timeout = timeout
        if token:
            self.session.headers["Authorization"] = f"Bearer {token}"
        self._paths = _paths()
        self._lock = threading.Lock()

    def _url(self, resource, namespace=None, name=None, sub=None):
        prefix, namespaced = self._paths[resource]
        u = self.base + prefix
        if namespaced and namespace:
            u += f"/namespaces/{namespace}"
        u += f"/{resource}"
        if name:
            u += f"/{name}"
        if sub:
            u += f"/{sub}"
        return u

    def _do(self, method, url, body=None, params=None):
        r = self.session.request(method, url, json=body, params=params, timeout=self.timeout)
        if r.status_code >= 400:
            try:
                st = r.json()
            except ValueError:
                st = {"code": r.status_code, "reason": "Unknown", "message": r.text}
            raise ApiError(st.get("code", r.status_code), st.get("reason", ""), st.get("message", r.text))
        return r.json() if r.content else {}

    def create(self, resource, obj, namespace=None):
        ns = namespace or obj.get("metadata", {}).get("namespace") or "default"
        return self._do("POST", self._url(resource, ns), obj)

    def get(self, resource, namespace, name):
        return self._do("GET", self._url(resource, namespace or "default", name))

    def created_unix(self, resource, namespace, name) -> float | None:
        """Sub-second creation time of an object, from the API server's
        ``X-Pto-Created-Unix`` response header (None if it has none)."""
        from .store import CREATED_UNIX_HEADER

        r = self.session.get(self._url(resource, namespace or "default", name), timeout=self.timeout)
        if r.status_code >= 400:
            return None
        v = r.headers.get(CREATED_UNIX_HEADER)
        return float(v) if v else None

    def list(self, resource, namespace=None, label_selector=None, field_selector=None):
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector if isinstance(label_selector, str) else \
                ",".join(f"{k}={v}" for k, v in label_selector.items())
        if field_selector:
            params["fieldSelector"] = field_selector
        return self._do("GET", self._url(resource, namespace), params=params)

    def update(self, resource, obj, namespace=None):
        md = obj["metadata"]
        return self._do("PUT", self._url(resource, namespace or md.get("namespace") or "default", md["name"]), obj)

    def update_status(self, resource, obj, namespace=None):
        md = obj["metadata"]
        return self._do("PUT", self._url(resource, namespace or md.get("namespace") or "default", md["name"],
                                         "status"), obj)

    def patch(self, resource, namespace, name, patch, subresource=None):
        return self._do("PATCH", self._url(resource, namespace or "default", name, subresource), patch)

    def delete(self, resource, namespace, name, propagation="Background"):
        return self._do("DELETE", self._url(resource, namespace or "default", name),
                        params={"propagationPolicy": propagation})

    def watch(self, resource, namespace=None, label_selector=None, resource_version=None, timeout_seconds=None):
        params = {"watch": "true"}
        if label_selector:
            params["labelSelector"] = label_selector
        if resource_version:
            params["resourceVersion"] = str(resource_version)
        if timeout_seconds:
            params["timeoutSeconds"] = str(int(timeout_seconds))
        return _RestWatch(self.session, self._url(resource, namespace), params)

    def record_event(self, involved, etype, reason, message):
        from ..api.types import now_rfc3339

        md = involved.get("metadata", {})
        ns = md.get("namespace", "default")
        import uuid

        ev = {"metadata": {"name": f"{md.get('name')}.{uuid.uuid4().hex[:10]}", "namespace": ns},
              "involvedObject": {"kind": involved.get("kind"), "name": md.get("name"), "namespace": ns,
                                 "uid": md.get("uid"), "apiVersion": involved.get("apiVersion")},
              "type": etype, "reason": reason, "message": message, "count": 1,
              "source": {"component": "pytorch-operator"}, "firstTimestamp": now_rfc3339(),
              "lastTimestamp": now_rfc3339()}
        return self.create("events", ev, ns)

    def pod_log(self, namespace, name, follow=False, tail_lines=None, container=None):
        params = {}
        if follow:
            params["follow"] = "true"
        if tail_lines:
            params["tailLines"] = str(tail_lines)
        if container:
            params["container"] = container
        r = self.session.get(self._url("pods", namespace, name, "log"), params=params, stream=follow,
                             timeout=None if follow else self.timeout)
        if follow:
            return (line.decode(errors="replace") for line in r.iter_lines())
        return r.text


class _RestWatch:
    def __init__(self, session, url, params):
        self.session, self.url, self.params = session, url, params
        self._resp = None
        self._stopped = False

    def __iter__(self):
        self._resp = self.session.get(self.url, params=self.params, stream=True, timeout=(10, None))
        try:
            for line in self._resp.iter_lines():
                if self._stopped:
                    break
                if not line:
                    continue
                ev = json.loads(line)
                yield ev["type"], ev["object"]
        except Exception:
            if not self._stopped:
                raise

    def stop(self):
        self._stopped = True
        if self._resp is not None:
            try:
                self._resp.close()
            except Exception:
                pass


def client_from_env(store: Store | None = None) -> Client:
    """PTO_APISERVER=http://host:port -> RestClient; else LocalClient(store)."""
    import os

    url = os.environ.get("PTO_APISERVER")
    if url:
        return RestClient(url, token=os.environ.get("PTO_TOKEN"))
    if store is None:
        raise RuntimeError("no PTO_APISERVER and no in-process store")
    return LocalClient(store)
