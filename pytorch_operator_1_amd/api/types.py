"""PyTorchJob object model.

Objects travel as plain JSON dictionaries with the exact camelCase keys of
the Kubernetes API (so YAML manifests, the SDK and any real kube-apiserver
round-trip unchanged).  This module gives typed accessors, naming helpers
and the exit-code table used by the controller.

Reference: ``pkg/apis/pytorch/v1/types.go:27-97`` (PyTorchJob,
PyTorchJobSpec), vendored ``kubeflow/common/job_controller/api/v1/
types.go:23-191`` (JobStatus, ReplicaSpec, ReplicaStatus, JobCondition),
vendored ``tf-operator/pkg/util/train/train_util.go:18-53``
(IsRetryableExitCode), ``jobcontroller/util.go:24-57`` (names/keys).
"""
from __future__ import annotations

import copy
import datetime as _dt
from typing import Any

from . import constants as C

Obj = dict[str, Any]


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def parse_rfc3339(s: str | None) -> float | None:
    if not s:
        return None
    s = s.replace("Z", "+00:00")
    return _dt.datetime.fromisoformat(s).timestamp()


def deepcopy(o: Obj) -> Obj:
    return copy.deepcopy(o)


def meta(o: Obj) -> Obj:
    return o.setdefault("metadata", {})


def name_of(o: Obj) -> str:
    return o.get("metadata", {}).get("name", "")


def namespace_of(o: Obj) -> str:
    return o.get("metadata", {}).get("namespace", "default") or "default"


def key_of(o: Obj) -> str:
    """cache.MetaNamespaceKeyFunc: ``<namespace>/<name>``."""
    return f"{namespace_of(o)}/{name_of(o)}"


def split_key(key: str) -> tuple[str, str]:
    parts = key.split("/")
    if len(parts) == 1:
        return "", parts[0]
    if len(parts) == 2:
        return parts[0], parts[1]
    raise ValueError(f"unexpected key format: {key!r}")


def replica_specs(job: Obj) -> dict[str, Obj]:
    return job.get("spec", {}).get("pytorchReplicaSpecs") or {}


def total_replicas(job: Obj) -> int:
    """``getTotalReplicas`` (job.go:216-222) == WORLD_SIZE."""
    return sum(int(s.get("replicas", 1) if s is not None else 0) for s in replica_specs(job).values())


def gen_general_name(job_name: str, rtype: str, index) -> str:
    """``<job>-<rtype-lower>-<index>``, '/' replaced by '-'."""
    return f"{job_name}-{rtype.lower()}-{index}".replace("/", "-")


def gen_labels(job_name: str) -> dict[str, str]:
    n = job_name.replace("/", "-")
    return {
        C.LABEL_GROUP_NAME: C.GROUP_NAME,
        C.LABEL_JOB_NAME: n,
        C.LABEL_PYTORCH_JOB_NAME: n,
        C.LABEL_CONTROLLER_NAME: C.CONTROLLER_NAME,
    }


def gen_owner_reference(job: Obj) -> Obj:
    return {
        "apiVersion": C.API_VERSION,
        "kind": C.KIND,
        "name": name_of(job),
        "uid": job.get("metadata", {}).get("uid", ""),
        "blockOwnerDeletion": True,
        "controller": True,
    }


def gen_expectation_pods_key(job_key: str, rtype: str) -> str:
    return f"{job_key}/{rtype.lower()}/pods"


def gen_expectation_services_key(job_key: str, rtype: str) -> str:
    return f"{job_key}/{rtype.lower()}/services"


def gen_pod_group_name(job_name: str) -> str:
    return job_name


# Exit-code classifier (train_util.go:18-53).  1-127 user/permanent errors,
# 128+N signals: SIGINT(130), SIGKILL(137), SIGUSR1(138, user-requested
# retry), SIGTERM(143) are retryable; SIGSEGV(139) and everything else not.
_RETRYABLE = frozenset({130, 137, 138, 143})


def is_retryable_exit_code(code: int) -> bool:
    return int(code) in _RETRYABLE


def get_port_from_job(job: Obj, rtype: str = C.REPLICA_MASTER) -> int:
    """``GetPortFromPyTorchJob`` (util.go:34-47): the ``pytorchjob-port`` of
    the ``pytorch`` container of the given replica type."""
    spec = replica_specs(job).get(rtype)
    if spec is None:
        raise KeyError(f"replica type {rtype} not found")
    for c in spec.get("template", {}).get("spec", {}).get("containers", []):
        if c.get("name") == C.DEFAULT_CONTAINER_NAME:
            for p in c.get("ports", []) or []:
                if p.get("name") == C.DEFAULT_PORT_NAME:
                    return int(p.get("containerPort"))
    raise KeyError("failed to find the port")


def conditions(job: Obj) -> list[Obj]:
    return job.get("status", {}).get("conditions") or []


def has_condition(status: Obj, ctype: str) -> bool:
    return any(c.get("type") == ctype and c.get("status") == "True" for c in status.get("conditions") or [])


def is_succeeded(status: Obj) -> bool:
    return has_condition(status, C.JOB_SUCCEEDED)


def is_failed(status: Obj) -> bool:
    return has_condition(status, C.JOB_FAILED)


def last_condition_type(job: Obj) -> str | None:
    cs = conditions(job)
    return cs[-1].get("type") if cs else None


def new_job(name: str, namespace: str = "default", image: str = "pytorch-mnist:rocm", master_args=None,
            workers: int = 1, worker_args=None, restart_policy: str = "OnFailure", gpus: int = 0,
            command=None, env=None, clean_pod_policy: str | None = None, backoff_limit: int | None = None,
            active_deadline_seconds: int | None = None, ttl_seconds_after_finished: int | None = None) -> Obj:
    """Convenience builder (mirrors the reference testutil job builders,
    ``pkg/common/util/v1/testutil/job.go:28-145``)."""

    def tmpl(args):
        c = {"name": C.DEFAULT_CONTAINER_NAME, "image": image}
        if command:
            c["command"] = list(command)
        if args:
            c["args"] = list(args)
        if env:
            c["env"] = [{"name": k, "value": str(v)} for k, v in env.items()]
        if gpus:
            c["resources"] = {"limits": {C.GPU_RESOURCE: gpus}}
        return {"spec": {"containers": [c]}}

    specs = {C.REPLICA_MASTER: {"replicas": 1, "restartPolicy": restart_policy, "template": tmpl(master_args)}}
    if workers:
        specs[C.REPLICA_WORKER] = {"replicas": workers, "restartPolicy": restart_policy,
                                   "template": tmpl(worker_args if worker_args is not None else master_args)}
    spec: Obj = {"pytorchReplicaSpecs": specs}
    if clean_pod_policy is not None:
        spec["cleanPodPolicy"] = clean_pod_policy
    if backoff_limit is not None:
        spec["backoffLimit"] = backoff_limit
    if active_deadline_seconds is not None:
        spec["activeDeadlineSeconds"] = active_deadline_seconds
    if ttl_seconds_after_finished is not None:
        spec["ttlSecondsAfterFinished"] = ttl_seconds_after_finished
    return {"apiVersion": C.API_VERSION, "kind": C.KIND, "metadata": {"name": name, "namespace": namespace},
            "spec": spec}
