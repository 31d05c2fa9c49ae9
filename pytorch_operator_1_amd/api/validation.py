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


_SUFFIX = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50,
           "k": 10 ** 3, "K": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15}


def parse_quantity(q) -> float:
    """Kubernetes resource quantity -> number ("288Gi", "200G", "1.5e11", 7)."""
    if isinstance(q, (int, float)):
        return float(q)
    s = str(q).strip()
    for suf in sorted(_SUFFIX, key=len, reverse=True):
        if s.endswith(suf):
            return float(s[: -len(suf)]) * _SUFFIX[suf]
    return float(s)


def hbm_requested(container: Obj) -> float:
    """Bytes of HBM per GPU requested via ``amd.com/hbm`` (0 = unspecified)."""
    res = container.get("resources") or {}
    n = 0.0
    for section in ("limits", "requests"):
        v = (res.get(section) or {}).get(C.HBM_RESOURCE)
        if v is not None:
            n = max(n, parse_quantity(v))
    return n


def validate_resources(job: Obj, gpus_per_node: int = 8, hbm_per_gpu: float = C.HBM_PER_GPU_BYTES) -> None:
    """MI355X extension: per-replica ``amd.com/gpu`` / ``amd.com/hbm`` sanity."""
    for rtype, rspec in (job.get("spec", {}).get("pytorchReplicaSpecs") or {}).items():
        for c in rspec.get("template", {}).get("spec", {}).get("containers", []):
            try:
                g = gpus_requested(c)
            except (TypeError, ValueError):
                raise ValidationError(f"PyTorchJobSpec is not valid: {C.GPU_RESOURCE} must be an integer in {rtype}")
            if g < 0 or g > gpus_per_node:
                raise ValidationError(
                    f"PyTorchJobSpec is not valid: {rtype} requests {g} {C.GPU_RESOURCE}, node has {gpus_per_node}")
            try:
                h = hbm_requested(c)
            except ValueError:
                raise ValidationError(f"PyTorchJobSpec is not valid: bad {C.HBM_RESOURCE} quantity in {rtype}")
            if h > hbm_per_gpu:
                raise ValidationError(f"PyTorchJobSpec is not valid: {rtype} requests {h / 1e9:.0f} GB "
                                      f"{C.HBM_RESOURCE} per GPU, an MI355X has {hbm_per_gpu / 1e9:.0f} GB")
