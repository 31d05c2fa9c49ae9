"""``PyTorchJobClient`` — same class, methods and signatures as the
reference SDK (``sdk/python/kubeflow/pytorchjob/api/py_torch_job_client.py:
29-393``), talking to this stack's API server.

Connection: ``base_url=`` / ``$PTO_APISERVER`` / ``config_file`` (a JSON or
YAML file with ``server:`` and optional ``token:``; a kubeconfig's current
context ``cluster.server`` is also understood) / default
``http://127.0.0.1:8080``.  Objects are returned as dicts exactly like the
reference (which returns the CustomObjectsApi dicts).

Fixes vs the reference: ``get_job_status`` returns ""
for a job with no conditions instead of raising IndexError, and
``replica_index=0`` selects index 0 instead of being ignored.
"""
from __future__ import annotations

import logging
import os
import time

from ..apiserver.client import LocalClient, RestClient
from ..apiserver.store import ApiError
from . import constants, utils
from .models import sanitize_for_serialization
from .watch import watch as pytorchjob_watch


def _load_config(config_file: str | None, context: str | None):
    if not config_file:
        for cand in (os.environ.get("PTO_CONFIG"), os.path.expanduser("~/.pto/config")):
            if cand and os.path.exists(cand):
                config_file = cand
                break
    if not config_file or not os.path.exists(config_file):
        return None, None
    import yaml

    with open(config_file) as f:
        cfg = yaml.safe_load(f) or {}
    if "server" in cfg:
        return cfg["server"], cfg.get("token")
    # kubeconfig
    ctx_name = context or cfg.get("current-context")
    ctx = next((c["context"] for c in cfg.get("contexts", []) if c.get("name") == ctx_name), None)
    if ctx:
        cl = next((c["cluster"] for c in cfg.get("clusters", []) if c.get("name") == ctx.get("cluster")), {})
        user = next((u["user"] for u in cfg.get("users", []) if u.get("name") == ctx.get("user")), {})
        return cl.get("server"), user.get("token")
    return None, None


class PyTorchJobClient:
    def __init__(self, config_file=None, context=None, client_configuration=None, persist_config=True,
                 base_url: str | None = None, token: str | None = None, api=None):
        if api is not None:  # in-process (LocalClient) or custom transport
            self.api = api
        else:
            server, tok = _load_config(config_file, context)
            url = base_url or os.environ.get("PTO_APISERVER") or server or "http://127.0.0.1:8080"
            self.api = RestClient(url, token=token or tok or os.environ.get("PTO_TOKEN"),
                                  timeout=constants.APISERVER_TIMEOUT)

    # ------------------------------------------------------------ CRUD
    def create(self, pytorchjob, namespace=None):
        body = sanitize_for_serialization(pytorchjob)
        if namespace is None:
            namespace = utils.set_pytorchjob_namespace(body)
        try:
            return self.api.create(constants.PYTORCHJOB_PLURAL, body, namespace)
        except ApiError as e:
            raise RuntimeError(
                "Exception when calling CustomObjectsApi->create_namespaced_custom_object: %s\n" % e.message)

    def get(self, name=None, namespace=None, watch=False, timeout_seconds=600):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        if watch:
            pytorchjob_watch(self.api, name=name, namespace=namespace, timeout_seconds=timeout_seconds)
            return None
        try:
            if name:
                return self.api.get(constants.PYTORCHJOB_PLURAL, namespace, name)
            return self.api.list(constants.PYTORCHJOB_PLURAL, namespace)
        except ApiError as e:
            what = "get_namespaced_custom_object" if name else "list_namespaced_custom_object"
            raise RuntimeError(f"Exception when calling CustomObjectsApi->{what}: {e.message}\n")

    def patch(self, name, pytorchjob, namespace=None):
        body = sanitize_for_serialization(pytorchjob)
        if namespace is None:
            namespace = utils.set_pytorchjob_namespace(body)
        try:
            return self.api.patch(constants.PYTORCHJOB_PLURAL, namespace, name, body)
        except ApiError as e:
            raise RuntimeError(
                "Exception when calling CustomObjectsApi->patch_namespaced_custom_object: %s\n" % e.message)

    def delete(self, name, namespace=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        try:
            return self.api.delete(constants.PYTORCHJOB_PLURAL, namespace, name)
        except ApiError as e:
            raise RuntimeError(
                "Exception when calling CustomObjectsApi->delete_namespaced_custom_object: %s\n" % e.message)

    # ------------------------------------------------------------ waiting
    def wait_for_job(self, name, namespace=None, watch=False, timeout_seconds=600, polling_interval=30,
                     status_callback=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        if watch:
            pytorchjob_watch(self.api, name=name, namespace=namespace, timeout_seconds=timeout_seconds)
            return self.get(name, namespace=namespace)
        return self.wait_for_condition(name, ["Succeeded", "Failed"], namespace=namespace,
                                       timeout_seconds=timeout_seconds, polling_interval=polling_interval,
                                       status_callback=status_callback)

    def wait_for_condition(self, name, expected_condition, namespace=None, timeout_seconds=600,
                           polling_interval=30, status_callback=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        pytorchjob = None
        end = time.time() + timeout_seconds
        while True:
            pytorchjob = self.get(name, namespace=namespace)
            if pytorchjob:
                if status_callback:
                    status_callback(pytorchjob)
                for c in pytorchjob.get("status", {}).get("conditions", []) or []:
                    if c.get("type", "") in expected_condition:
                        return pytorchjob
            if time.time() + polling_interval > end:
                break
            time.sleep(polling_interval)
        raise RuntimeError(
            "Timeout waiting for PyTorchJob {0} in namespace {1} to enter one of the conditions {2}.".format(
                name, namespace, expected_condition), pytorchjob)

    def get_job_status(self, name, namespace=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        pytorchjob = self.get(name, namespace=namespace)
        conds = pytorchjob.get("status", {}).get("conditions", []) or []
        return conds[-1].get("type", "") if conds else ""

    def is_job_running(self, name, namespace=None):
        return self.get_job_status(name, namespace=namespace).lower() == "running"

    def is_job_succeeded(self, name, namespace=None):
        return self.get_job_status(name, namespace=namespace).lower() == "succeeded"

    # ------------------------------------------------------------ pods/logs
    def get_pod_names(self, name, namespace=None, master=False, replica_type=None, replica_index=None):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        labels = utils.get_labels(name, master=master, replica_type=replica_type, replica_index=replica_index)
        try:
            resp = self.api.list("pods", namespace, utils.to_selector(labels))
        except ApiError as e:
            raise RuntimeError("Exception when calling CoreV1Api->list_namespaced_pod: %s\n" % e.message)
        pod_names = [p["metadata"]["name"] for p in resp.get("items", []) if p.get("metadata", {}).get("name")]
        if not pod_names:
            logging.warning("Not found Pods of the PyTorchJob %s with the labels %s.", name, labels)
            return None
        return set(pod_names)

    def get_logs(self, name, namespace=None, master=True, replica_type=None, replica_index=None, follow=False):
        if namespace is None:
            namespace = utils.get_default_target_namespace()
        pod_names = self.get_pod_names(name, namespace=namespace, master=master, replica_type=replica_type,
                                       replica_index=replica_index)
        if not pod_names:
            raise RuntimeError("Not found Pods of the PyTorchJob {} in namespace {}".format(name, namespace))
        out = {}
        for pod in sorted(pod_names):
            logs = self._pod_log(namespace, pod, follow)
            logging.info("The logs of Pod %s:\n %s", pod, logs)
            out[pod] = logs
        return out

    def _pod_log(self, namespace, pod, follow):
        if isinstance(self.api, RestClient):
            r = self.api.pod_log(namespace, pod, follow=follow)
            return "".join(l + "\n" for l in r) if follow else r
        if isinstance(self.api, LocalClient):
            p = self.api.get("pods", namespace, pod)
            path = (p["metadata"].get("annotations") or {}).get("pto.amd.com/log-path")
            return open(path, errors="replace").read() if path and os.path.exists(path) else ""
        return ""
