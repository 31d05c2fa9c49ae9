"""Spec validation (``pkg/apis/pytorch/validation/validation.go:23-77``).

Same rules and the same error messages as the reference, plus MI355X
resource checks (``amd.com/gpu`` must be a non-negative integer and may not
exceed the node's GPU count) exposed separately in
:func:`validate_resources` so the base rules stay reference-exact.
"""
from __future__ import annotations

from . import constants as C
from .types import Obj


class ValidationError(ValueError):
    pass


def validate_spec(spec: Obj | None) -> None:
    """Raise :class:`ValidationError` if the PyTorchJobSpec is invalid."""
    if spec is None:
        raise ValidationError("PyTorchJobSpec is not valid")
    specs = spec.get("pytorchReplicaSpecs")
    if specs is None:
        raise ValidationError("PyTorchJobSpec is not valid")
    master_exists = False
    for rtype, value in specs.items():
        containers = (((value or {}).get("template") or {}).get("spec") or {}).get("containers") or []
        if value is None or len(containers) == 0:
            raise ValidationError(f"PyTorchJobSpec is not valid: containers definition expected in {rtype}")
        if rtype not in C.REPLICA_TYPES:
            raise ValidationError(f"PyTorchReplicaType is {rtype} but must be one of [Master Worker]")
        default_present = False
        for c in containers:
            if not c.get("image"):
                raise ValidationError(f"PyTorchJobSpec is not valid: Image is undefined in the container of {rtype}")
            if c.get("name") == C.DEFAULT_CONTAINER_NAME:
                default_present = True
        if not default_present:
            raise ValidationError(
                f"PyTorchJobSpec is not valid: There is no container named {C.DEFAULT_CONTAINER_NAME} in {rtype}")
        if rtype == C.REPLICA_MASTER:
            master_exists = True
            if value.get("replicas") is not None and int(value["replicas"]) != 1:
                raise ValidationError("PyTorchJobSpec is not valid: There must be only 1 master replica")
    if not master_exists:
        raise ValidationError("PyTorchJobSpec is not valid: Master ReplicaSpec must be present")


def gpus_requested(container: Obj) -> int:
    res = container.get("resources") or {}
    n = 0
    for section in ("limits", "requests"):
        sec = res.get(section) or {}
        for key in (C.GPU_RESOURCE,) + C.LEGACY_GPU_RESOURCES:
            if key in sec:
                n = max(n, int(sec[key]))
    return n


def validate_resources(job: Obj, gpus_per_node: int = 8) -> None:
    """MI355X extension: per-replica ``amd.com/gpu`` sanity."""
    for rtype, rspec in (job.get("spec", {}).get("pytorchReplicaSpecs") or {}).items():
        for c in rspec.get("template", {}).get("spec", {}).get("containers", []):
            try:
                g = gpus_requested(c)
            except (TypeError, ValueError):
                raise ValidationError(f"PyTorchJobSpec is not valid: {C.GPU_RESOURCE} must be an integer in {rtype}")
            if g < 0 or g > gpus_per_node:
                raise ValidationError(
                    f"PyTorchJobSpec is not valid: {rtype} requests {g} {C.GPU_RESOURCE}, node has {gpus_per_node}")
