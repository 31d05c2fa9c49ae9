"""Defaulting (``pkg/apis/pytorch/v1/defaults.go:27-105``).

* ``cleanPodPolicy`` → ``None`` when unset;
* replica-type keys normalised case-insensitively to ``Master``/``Worker``;
* ``replicas`` → 1 and ``restartPolicy`` → ``OnFailure`` when unset;
* on the Master only: ``pytorchjob-port: 23456`` appended to the container
  named ``pytorch`` (container 0 if none is named so) unless present.
"""
from __future__ import annotations

from . import constants as C
from .types import Obj


def _set_default_port(pod_spec: Obj) -> None:
    containers = pod_spec.get("containers") or []
    if not containers:
        return
    index = 0
    for i, c in enumerate(containers):
        if c.get("name") == C.DEFAULT_CONTAINER_NAME:
            index = i
            break
    ports = containers[index].setdefault("ports", []) or []
    containers[index]["ports"] = ports
    if not any(p.get("name") == C.DEFAULT_PORT_NAME for p in ports):
        ports.append({"name": C.DEFAULT_PORT_NAME, "containerPort": C.DEFAULT_PORT})


def _set_default_replicas(spec: Obj) -> None:
    if spec.get("replicas") is None:
        spec["replicas"] = 1
    if not spec.get("restartPolicy"):
        spec["restartPolicy"] = C.DEFAULT_RESTART_POLICY


def _normalise_type_names(specs: dict) -> None:
    for typ in C.REPLICA_TYPES:
        for t in list(specs.keys()):
            if t.lower() == typ.lower() and t != typ:
                specs[typ] = specs.pop(t)
                break


def set_defaults(job: Obj) -> Obj:
    """Mutate and return ``job`` (``SetDefaults_PyTorchJob``)."""
    spec = job.setdefault("spec", {})
    if spec.get("cleanPodPolicy") is None:
        spec["cleanPodPolicy"] = C.CLEAN_POD_POLICY_NONE
    specs = spec.get("pytorchReplicaSpecs")
    if not specs:
        return job
    _normalise_type_names(specs)
    for rtype, rspec in specs.items():
        if rspec is None:
            continue
        _set_default_replicas(rspec)
        if rtype == C.REPLICA_MASTER:
            _set_default_port(rspec.setdefault("template", {}).setdefault("spec", {}))
    return job
