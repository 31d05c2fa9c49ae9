"""Typed PyTorchJob models with the reference SDK's class names and
snake_case <-> camelCase mapping (``sdk/python/kubeflow/pytorchjob/models/
v1_*.py``; spec fields ``v1_py_torch_job_spec.py:49-63``).

The reference depends on the ``kubernetes`` client for ``V1ObjectMeta`` /
``V1PodTemplateSpec``; that package is not part of this stack, so minimal
equivalents with the same constructor keywords are provided here.  Any
field may also be given as a plain dict.
"""
from __future__ import annotations

import datetime as _dt
import re
from typing import Any


def _camel(s: str) -> str:
    return re.sub(r"_([a-z0-9])", lambda m: m.group(1).upper(), s)


def sanitize_for_serialization(obj: Any):
    """Model/dict/list/datetime -> JSON-ready structure (camelCase keys)."""
    if obj is None:
        return None
    if isinstance(obj, (str, int, float, bool)):
        return obj
    if isinstance(obj, (_dt.datetime, _dt.date)):
        return obj.isoformat()
    if isinstance(obj, (list, tuple)):
        return [sanitize_for_serialization(o) for o in obj]
    if isinstance(obj, dict):
        return {k: sanitize_for_serialization(v) for k, v in obj.items()}
    if isinstance(obj, _Model):
        out = {}
        for attr, key in obj.attribute_map.items():
            v = getattr(obj, attr)
            if v is not None:
                out[key] = sanitize_for_serialization(v)
        return out
    if hasattr(obj, "to_dict"):
        return sanitize_for_serialization(obj.to_dict())
    raise TypeError(f"cannot serialize {type(obj)}")


class _Model:
    swagger_types: dict[str, str] = {}
    attribute_map: dict[str, str] = {}

    def __init__(self, **kw):
        for attr in self.attribute_map:
            setattr(self, attr, kw.pop(attr, None))
        if kw:
            raise TypeError(f"{type(self).__name__}: unexpected fields {sorted(kw)}")

    def to_dict(self):
        return sanitize_for_serialization(self)

    @classmethod
    def from_dict(cls, d: dict | None):
        if d is None:
            return None
        inv = {v: k for k, v in cls.attribute_map.items()}
        kw = {}
        for key, val in d.items():
            attr = inv.get(key)
            if attr is None:
                continue
            sub = _NESTED.get((cls.__name__, attr))
            if sub is not None and val is not None:
                kind, typ = sub
                if kind == "one":
                    val = typ.from_dict(val)
                elif kind == "list":
                    val = [typ.from_dict(x) for x in val]
                elif kind == "map":
                    val = {k: typ.from_dict(x) for k, x in val.items()}
            kw[attr] = val
        return cls(**kw)

    def __eq__(self, other):
        return isinstance(other, type(self)) and self.to_dict() == other.to_dict()

    def __repr__(self):
        return f"{type(self).__name__}({self.to_dict()!r})"


def _model(name, fields):
    attrs = {"attribute_map": {f: _camel(f) for f in fields}, "swagger_types": {f: "object" for f in fields}}
    return type(name, (_Model,), attrs)


V1ObjectMeta = _model("V1ObjectMeta", ["name", "namespace", "labels", "annotations", "uid", "resource_version",
                                       "creation_timestamp", "generate_name", "owner_references", "generation",
                                       "deletion_timestamp", "finalizers"])
V1Container = _model("V1Container", ["name", "image", "command", "args", "env", "ports", "resources",
                                     "working_dir", "image_pull_policy"])
V1PodSpec = _model("V1PodSpec", ["containers", "init_containers", "restart_policy", "scheduler_name",
                                 "node_selector", "volumes"])
V1PodTemplateSpec = _model("V1PodTemplateSpec", ["metadata", "spec"])


class V1Time(str):
    """RFC3339 timestamp (the reference models it as a string)."""


V1JobCondition = _model("V1JobCondition", ["last_transition_time", "last_update_time", "message", "reason",
                                           "status", "type"])
V1ReplicaStatus = _model("V1ReplicaStatus", ["active", "failed", "succeeded"])
V1JobStatus = _model("V1JobStatus", ["completion_time", "conditions", "last_reconcile_time", "replica_statuses",
                                     "start_time"])
V1ReplicaSpec = _model("V1ReplicaSpec", ["replicas", "restart_policy", "template"])
V1PyTorchJobSpec = _model("V1PyTorchJobSpec", ["active_deadline_seconds", "backoff_limit", "clean_pod_policy",
                                               "pytorch_replica_specs", "ttl_seconds_after_finished"])
V1PyTorchJob = _model("V1PyTorchJob", ["api_version", "kind", "metadata", "spec", "status"])
V1PyTorchJobList = _model("V1PyTorchJobList", ["api_version", "items", "kind", "metadata"])

_NESTED = {
    ("V1PyTorchJob", "metadata"): ("one", V1ObjectMeta),
    ("V1PyTorchJob", "spec"): ("one", V1PyTorchJobSpec),
    ("V1PyTorchJob", "status"): ("one", V1JobStatus),
    ("V1PyTorchJobList", "items"): ("list", V1PyTorchJob),
    ("V1PyTorchJobSpec", "pytorch_replica_specs"): ("map", V1ReplicaSpec),
    ("V1ReplicaSpec", "template"): ("one", V1PodTemplateSpec),
    ("V1PodTemplateSpec", "metadata"): ("one", V1ObjectMeta),
    ("V1PodTemplateSpec", "spec"): ("one", V1PodSpec),
    ("V1PodSpec", "containers"): ("list", V1Container),
    ("V1PodSpec", "init_containers"): ("list", V1Container),
    ("V1JobStatus", "conditions"): ("list", V1JobCondition),
    ("V1JobStatus", "replica_statuses"): ("map", V1ReplicaStatus),
}

__all__ = ["V1ObjectMeta", "V1Container", "V1PodSpec", "V1PodTemplateSpec", "V1Time", "V1JobCondition",
           "V1ReplicaStatus", "V1JobStatus", "V1ReplicaSpec", "V1PyTorchJobSpec", "V1PyTorchJob", "V1PyTorchJobList",
           "sanitize_for_serialization"]
