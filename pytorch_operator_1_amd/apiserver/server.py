"""Kubernetes-compatible REST front end for :class:`~.store.Store` (aiohttp).

Paths follow the Kubernetes API so the SDK and ``kubectl``-style tools
address objects exactly as on a cluster:

* ``/apis/kubeflow.org/v1/namespaces/{ns}/pytorchjobs[/{name}[/status]]``
  and ``/apis/kubeflow.org/v1/pytorchjobs`` (all namespaces)
* ``/api/v1/namespaces/{ns}/{pods,services,events,endpoints,configmaps}[/{name}[/status|/log]]``
* ``/apis/coordination.k8s.io/v1/namespaces/{ns}/leases[/{name}]``
* ``/apis/scheduling.incubator.k8s.io/v1alpha1/namespaces/{ns}/podgroups[/{name}]``
* ``/apis/apiextensions.k8s.io/v1beta1/customresourcedefinitions[/{name}]``

Verbs: GET (get/list, ``?labelSelector=``, ``?fieldSelector=``,
``?watch=true&resourceVersion=`` streaming newline-delimited watch events),
POST (create), PUT (update / status update), PATCH (JSON merge patch),
DELETE (``propagationPolicy``).  PyTorchJob creates/updates are checked
against the CRD's OpenAPI constraints (``manifests/base/crd.yaml:19-38``:
Master replicas in [1,1], Worker replicas >= 1) and rejected with 422.
"""
from __future__ import annotations

import asyncio
import json
import os
import threading

from aiohttp import web

from ..api import crd
from .store import CREATED_UNIX_HEADER, RESOURCES, ApiError, Store

GROUP_PATHS = {
    ("kubeflow.org", "v1"): {"pytorchjobs"},
    ("coordination.k8s.io", "v1"): {"leases"},
    ("scheduling.incubator.k8s.io", "v1alpha1"): {"podgroups"},
    ("apiextensions.k8s.io", "v1beta1"): {"customresourcedefinitions"},
    ("apiextensions.k8s.io", "v1"): {"customresourcedefinitions"},
}
CORE = {"pods", "services", "events", "endpoints", "configmaps", "nodes"}
LOG_ANNOTATION = "pto.amd.com/log-path"


def _parse(path: str):
    """-> (resource, namespace, name, subresource) or raise 404."""
    parts = [p for p in path.strip("/").split("/") if p]
    if parts[:2] == ["api", "v1"]:
        rest, allowed = parts[2:], CORE
    elif len(parts) >= 3 and parts[0] == "apis" and (parts[1], parts[2]) in GROUP_PATHS:
        rest, allowed = parts[3:], GROUP_PATHS[(parts[1], parts[2])]
    else:
        raise ApiError(404, "NotFound", f"no route for {path}")
    ns = None
    if len(rest) >= 2 and rest[0] == "namespaces":
        ns, rest = rest[1], rest[2:]
        if not rest:
            raise ApiError(404, "NotFound", "namespace objects are implicit")
    if not rest or rest[0] not in allowed:
        raise ApiError(404, "NotFound", f"the server could not find the requested resource ({path})")
    resource = rest[0]
    name = rest[1] if len(rest) > 1 else None
    sub = rest[2] if len(rest) > 2 else None
    return resource, ns, name, sub


def _json(obj, status=200):
    return web.json_response(obj, status=status, dumps=lambda o: json.dumps(o))


class ApiServer:
    def __init__(self, store: Store | None = None, host: str = "127.0.0.1", port: int = 8080, token: str | None = None):
        self.store = store or Store()
        self.host, self.port = host, port
        self.token = token
        self.app = web.Application(middlewares=[self._errors])
        self.app.router.add_get("/healthz", self._healthz)
        self.app.router.add_get("/version", self._version)
        self.app.router.add_route("*", "/{tail:.*}", self._dispatch)
        self._runner = None
        self._thread = None
        self._loop = None

    @web.middleware
    async def _errors(self, request, handler):
        if self.token and request.path not in ("/healthz", "/version"):
            if request.headers.get("Authorization") != f"Bearer {self.token}":
                return _json({"kind": "Status", "status": "Failure", "code": 401, "reason": "Unauthorized",
                              "message": "Unauthorized"}, 401)
        try:
            return await handler(request)
        except ApiError as e:
            return _json(e.status(), e.code)
        except json.JSONDecodeError as e:
            return _json(ApiError(400, "BadRequest", f"invalid JSON body: {e}").status(), 400)

    async def _healthz(self, request):
        return web.Response(text="ok")

    async def _version(self, request):
        from .. import __version__

        return _json({"major": "1", "minor": "16", "gitVersion": f"pto-{__version__}", "platform": "linux/amd64"})

    def _validate(self, resource, obj):
        if resource == "pytorchjobs":
            err = crd.openapi_check(obj)
            if err:
                raise ApiError(422, "Invalid", f'PyTorchJob.kubeflow.org "{obj.get("metadata", {}).get("name")}" '
                                               f"is invalid: {err}")

    async def _dispatch(self, request: web.Request):
        resource, ns, name, sub = _parse(request.path)
        st, q, m = self.store, request.query, request.method
        if m == "GET":
            if name is None:
                if q.get("watch") in ("1", "true", "True"):
                    return await self._watch(request, resource, ns)
                return _json(st.list(resource, ns, q.get("labelSelector"), q.get("fieldSelector")))
            if sub == "log":
                return await self._log(request, ns, name)
            obj = st.get(resource, ns, name)
            resp = _json(obj)
            t = st.created_unix(obj.get("metadata", {}).get("uid"))
            if t is not None:
                resp.headers[CREATED_UNIX_HEADER] = f"{t:.6f}"
            return resp
        body = await request.json() if m in ("POST", "PUT", "PATCH") and request.can_read_body else None
        if m == "POST":
            if name is not None:
                raise ApiError(405, "MethodNotAllowed", "POST to a named object")
            self._validate(resource, body)
            return _json(st.create(resource, body, ns), 201)
        if name is None:
            if m == "DELETE":  # deletecollection
                items = st.list(resource, ns, q.get("labelSelector"))["items"]
                for it in items:
                    st.delete(resource, ns, it["metadata"]["name"])
                return _json({"kind": "Status", "status": "Success"})
            raise ApiError(405, "MethodNotAllowed", f"{m} needs an object name")
        if m == "PUT":
            body.setdefault("metadata", {}).setdefault("name", name)
            if sub == "status":
                return _json(st.update_status(resource, body, ns))
            self._validate(resource, body)
            return _json(st.update(resource, body, ns))
        if m == "PATCH":
            out = st.patch(resource, ns, name, body, subresource=sub)
            if sub is None:
                try:
                    self._validate(resource, out)
                except ApiError:
                    raise
            return _json(out)
        if m == "DELETE":
            prop = q.get("propagationPolicy") or (body or {}).get("propagationPolicy") or "Background"
            return _json(st.delete(resource, ns, name, propagation=prop))
        raise ApiError(405, "MethodNotAllowed", m)

    async def _watch(self, request, resource, ns):
        q = request.query
        w = self.store.watch(resource, ns, q.get("labelSelector"), q.get("fieldSelector"),
                             q.get("resourceVersion"))
        timeout = float(q.get("timeoutSeconds", "0") or 0)
        resp = web.StreamResponse(headers={"Content-Type": "application/json", "Transfer-Encoding": "chunked"})
        await resp.prepare(request)
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout if timeout > 0 else None
        try:
            while True:
                if deadline and loop.time() > deadline:
                    break
                ev = await loop.run_in_executor(None, w.get, 0.5)
                if ev is None:
                    continue
                await resp.write((json.dumps({"type": ev.type, "object": ev.object}) + "\n").encode())
                if ev.type == "ERROR":
                    break
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            w.stop()
        return resp

    async def _log(self, request, ns, name):
        pod = self.store.get("pods", ns, name)
        path = (pod.get("metadata", {}).get("annotations") or {}).get(LOG_ANNOTATION)
        container = request.query.get("container")
        if container and path:
            cpath = path.replace(".log", f".{container}.log")
            if os.path.exists(cpath):
                path = cpath
        if not path or not os.path.exists(path):
            return web.Response(text="")
        follow = request.query.get("follow") in ("1", "true", "True")
        tail = request.query.get("tailLines")
        if not follow:
            with open(path, errors="replace") as f:
                lines = f.readlines()
            if tail:
                lines = lines[-int(tail):]
            return web.Response(text="".join(lines))
        resp = web.StreamResponse(headers={"Content-Type": "text/plain"})
        await resp.prepare(request)
        with open(path, errors="replace") as f:
            while True:
                chunk = f.read()
                if chunk:
                    await resp.write(chunk.encode())
                    continue
                try:
                    phase = self.store.get("pods", ns, name).get("status", {}).get("phase")
                except ApiError:
                    break
                if phase in ("Succeeded", "Failed"):
                    rest = f.read()
                    if rest:
                        await resp.write(rest.encode())
                    break
                await asyncio.sleep(0.2)
        return resp

    # ------------------------------------------------------------ lifecycle
    async def start_async(self):
        self._runner = web.AppRunner(self.app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        if self.port == 0:
            self.port = site._server.sockets[0].getsockname()[1]

    def start_in_thread(self) -> "ApiServer":
        ready = threading.Event()

        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._loop.run_until_complete(self.start_async())
            ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, name="pto-apiserver", daemon=True)
        self._thread.start()
        ready.wait(10)
        return self

    def stop(self):
        if self._loop:
            async def _shutdown():
                await self._runner.cleanup()

            fut = asyncio.run_coroutine_threadsafe(_shutdown(), self._loop)
            try:
                fut.result(5)
            except Exception:
                pass
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(5)

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"


def resource_paths() -> dict:
    """resource -> URL path template (used by the REST client)."""
    out = {}
    for r, (api_version, _, namespaced, _) in RESOURCES.items():
        prefix = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        out[r] = (prefix, namespaced)
    return out
