"""CustomResourceDefinition for ``pytorchjobs.kubeflow.org`` and the
OpenAPI-level checks the API server applies on create/update.

Reference: ``manifests/base/crd.yaml:1-42`` (namespaced, ``status``
subresource, printer columns State/Age, Master replicas in [1,1], Worker
replicas >= 1) and the generated OpenAPI in
``pkg/apis/pytorch/v1/openapi_generated.go:28-188``.  The JSON Schema
below is emitted from the same field list the SDK models use.
"""
from __future__ import annotations

from . import constants as C


def _replica_schema(minimum: int, maximum: int | None = None) -> dict:
    rep = {"type": "integer", "minimum": minimum}
    if maximum is not None:
        rep["maximum"] = maximum
    return {"type": "object", "properties": {
        "replicas": rep,
        "restartPolicy": {"type": "string", "enum": list(C.RESTART_POLICIES)},
        "template": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
    }}


def crd_manifest() -> dict:
    return {
        "apiVersion": "apiextensions.k8s.io/v1beta1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": C.CRD_NAME},
        "spec": {
            "group": C.GROUP_NAME,
            "version": C.VERSION,
            "scope": "Namespaced",
            "names": {"kind": C.KIND, "plural": C.PLURAL, "singular": C.SINGULAR},
            "subresources": {"status": {}},
            "additionalPrinterColumns": [
                {"name": "State", "type": "string", "JSONPath": ".status.conditions[-1:].type"},
                {"name": "Age", "type": "date", "JSONPath": ".metadata.creationTimestamp"},
            ],
            "validation": {"openAPIV3Schema": {"properties": {"spec": {"properties": {
                "activeDeadlineSeconds": {"type": "integer", "format": "int64"},
                "backoffLimit": {"type": "integer", "format": "int32"},
                "cleanPodPolicy": {"type": "string", "enum": ["", "All", "Running", "None"]},
                "ttlSecondsAfterFinished": {"type": "integer", "format": "int32"},
                "pytorchReplicaSpecs": {"properties": {
                    "Master": _replica_schema(1, 1),
                    "Worker": _replica_schema(1),
                }},
            }}}}},
        },
    }


def openapi_check(job: dict) -> str | None:
    """Return an error string (kube-apiserver wording) or None."""
    spec = (job or {}).get("spec") or {}
    specs = spec.get("pytorchReplicaSpecs") or {}
    for rtype, lo, hi in ((C.REPLICA_MASTER, 1, 1), (C.REPLICA_WORKER, 1, None)):
        rs = specs.get(rtype)
        if not isinstance(rs, dict) or rs.get("replicas") is None:
            continue
        try:
            n = int(rs["replicas"])
        except (TypeError, ValueError):
            return f"spec.pytorchReplicaSpecs.{rtype}.replicas in body must be of type integer"
        if n < lo:
            return f"spec.pytorchReplicaSpecs.{rtype}.replicas in body should be greater than or equal to {lo}"
        if hi is not None and n > hi:
            return f"spec.pytorchReplicaSpecs.{rtype}.replicas in body should be less than or equal to {hi}"
        rp = rs.get("restartPolicy")
        if rp and rp not in C.RESTART_POLICIES:
            return (f"spec.pytorchReplicaSpecs.{rtype}.restartPolicy in body should be one of "
                    f"{list(C.RESTART_POLICIES)}")
    cpp = spec.get("cleanPodPolicy")
    if cpp not in (None, "", "All", "Running", "None"):
        return 'spec.cleanPodPolicy in body should be one of ["" "All" "Running" "None"]'
    return None


def json_schema() -> dict:
    """Standalone JSON Schema of a PyTorchJob (for SDK/model generation)."""
    m = crd_manifest()["spec"]["validation"]["openAPIV3Schema"]
    return {"$schema": "http://json-schema.org/draft-07/schema#", "title": C.KIND, "type": "object",
            "properties": {"apiVersion": {"type": "string"}, "kind": {"type": "string"},
                           "metadata": {"type": "object"}, **m["properties"],
                           "status": {"type": "object", "properties": {
                               "conditions": {"type": "array"}, "replicaStatuses": {"type": "object"},
                               "startTime": {"type": "string"}, "completionTime": {"type": "string"},
                               "lastReconcileTime": {"type": "string"}}}}}
