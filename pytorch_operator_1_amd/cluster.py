"""All-in-one single-node cluster: object store + REST API server +
PyTorchJob controller + node manager (native agent), in one process.

This is what ``pto up`` runs on an 8xMI355X node (the reference needs a
Kubernetes cluster, kube-dns, a device plugin and the operator
Deployment; here one process hosts the control plane and the C++ agent
supervises the training processes).  Tests use it to run real
multi-process jobs end to end on CPU (gloo).
"""
from __future__ import annotations

import logging
import os
import time

from .api import constants as C
from .apiserver.client import LocalClient, RestClient
from .apiserver.server import ApiServer
from .apiserver.store import ApiError, Store
from .controller.metrics import OperatorMetrics
from .controller.pytorch import ControllerConfig, PyTorchController
from .node.kubelet import Kubelet

log = logging.getLogger("pto-cluster")


class LocalCluster:
    def __init__(self, gpus: int | None = None, port: int = 0, wal_path: str | None = None,
                 log_dir: str | None = None, enable_gang_scheduling: bool = False, serve_http: bool = True,
                 extra_env: dict | None = None, threadiness: int = 2, hbm_per_gpu: float | None = None,
                 gpu_visibility: str | None = None, gpu_share: int | None = None, restart_scope: str = "job"):
        self.store = Store(wal_path=wal_path)
        self.client = LocalClient(self.store)
        self.server = ApiServer(self.store, port=port) if serve_http else None
        self.metrics = OperatorMetrics()
        self.controller = PyTorchController(
            self.client, ControllerConfig(enable_gang_scheduling=enable_gang_scheduling, threadiness=threadiness,
                                          job_resync_period=5.0, restart_scope=restart_scope), metrics=self.metrics)
        kw = {"hbm_per_gpu": hbm_per_gpu} if hbm_per_gpu else {}
        if gpu_visibility:
            kw["gpu_visibility"] = gpu_visibility
        if gpu_share:
            kw["gpu_share"] = gpu_share
        self.kubelet = Kubelet(self.client, gpus=gpus, log_dir=log_dir, extra_env=extra_env, metrics=self.metrics,
                               **kw)

    def start(self):
        if self.server:
            self.server.start_in_thread()
        try:
            from .api.crd import crd_manifest

            self.store.create("customresourcedefinitions", crd_manifest())
        except ApiError:
            pass
        self.controller.run()
        self.kubelet.start()
        self.metrics.is_leader.set(1)
        return self

    def stop(self):
        self.kubelet.stop()
        self.controller.stop()
        if self.server:
            self.server.stop()
        self.store.close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    @property
    def url(self):
        return self.server.url if self.server else None

    def rest_client(self):
        return RestClient(self.url)

    # ---------------------------------------------------------- helpers
    def submit(self, job: dict) -> dict:
        return self.client.create("pytorchjobs", job, job.get("metadata", {}).get("namespace"))

    def wait_for_condition(self, name, types=(C.JOB_SUCCEEDED, C.JOB_FAILED), namespace="default",
                           timeout=120.0) -> dict:
        end = time.time() + timeout
        while time.time() < end:
            try:
                j = self.store.get("pytorchjobs", namespace, name)
            except ApiError:
                j = None
            if j:
                for c in j.get("status", {}).get("conditions") or []:
                    if c["type"] in types and c["status"] == "True":
                        return j
            time.sleep(0.05)
        raise TimeoutError(f"job {namespace}/{name} did not reach {types} in {timeout}s; last={j}")

    def pod_log(self, namespace, name) -> str:
        pod = self.store.get("pods", namespace, name)
        path = (pod["metadata"].get("annotations") or {}).get("pto.amd.com/log-path")
        if path and os.path.exists(path):
            return open(path, errors="replace").read()
        return ""
