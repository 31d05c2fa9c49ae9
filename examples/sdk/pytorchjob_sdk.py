#!/usr/bin/env python3
"""The reference SDK walkthrough (``sdk/python/examples/kubeflow-pytorchjob-
sdk.ipynb``) as a script: build a ``pytorch-dist-mnist-gloo`` PyTorchJob
(Master 1 + Worker 1) with the SDK models, create it, read it back, wait for
it, check it succeeded, print the master's log and delete it.

Against a running stack (``pto up``)::

    python examples/sdk/pytorchjob_sdk.py --url http://127.0.0.1:8080

With no ``--url`` a throw-away single-node stack (API server + operator +
node agent) is started in-process first, so the example runs anywhere (CPU,
gloo).  ``--gpu`` runs the replicas on MI355X with RCCL instead
(``amd.com/gpu: 1`` each).

Differences from the notebook: ``V1Container`` / ``V1PodSpec`` /
``V1PodTemplateSpec`` / ``V1ObjectMeta`` come from ``kubeflow.pytorchjob``
(the ``kubernetes`` client package is not part of this stack; the classes
take the same keywords), and the trainer is told to run a bounded number of
synthetic-data steps so the walkthrough finishes in seconds.
"""
from __future__ import annotations

import argparse
import contextlib
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from kubeflow.pytorchjob import (PyTorchJobClient, V1Container, V1ObjectMeta, V1PodSpec,  # noqa: E402
                                 V1PodTemplateSpec, V1PyTorchJob, V1PyTorchJobSpec, V1ReplicaSpec, utils)


def build_job(name: str, namespace: str, gpu: bool, steps: int) -> V1PyTorchJob:
    args = ["--backend", "rccl" if gpu else "gloo", "--max-steps", str(steps), "--log-interval", "10", "--no-test"]
    if not gpu:
        args += ["--no-cuda", "--train-size", "2560"]
    container = V1Container(
        name="pytorch",
        image="gcr.io/kubeflow-ci/pytorch-dist-mnist-test:v1.0",  # mapped to this package's trainer
        args=args,
        resources={"limits": {"amd.com/gpu": 1}} if gpu else None,
    )

    def replica():
        return V1ReplicaSpec(replicas=1, restart_policy="OnFailure",
                             template=V1PodTemplateSpec(spec=V1PodSpec(containers=[container])))

    return V1PyTorchJob(
        api_version="kubeflow.org/v1",
        kind="PyTorchJob",
        metadata=V1ObjectMeta(name=name, namespace=namespace),
        spec=V1PyTorchJobSpec(clean_pod_policy="None",
                              pytorch_replica_specs={"Master": replica(), "Worker": replica()}),
    )


@contextlib.contextmanager
def local_stack(gpu: bool):
    from pytorch_operator_1_amd.cluster import LocalCluster

    with tempfile.TemporaryDirectory(prefix="pto-sdk-") as d, \
            LocalCluster(gpus=None if gpu else 0, log_dir=d) as c:
        yield c.url


def walkthrough(url: str, gpu: bool, steps: int, name: str = "pytorch-dist-mnist-gloo") -> bool:
    namespace = utils.get_default_target_namespace()
    client = PyTorchJobClient(base_url=url)
    client.create(build_job(name, namespace, gpu, steps))
    job = client.get(name, namespace=namespace)
    print("created:", job["metadata"]["name"], "uid", job["metadata"].get("uid"))
    print("status now:", client.get_job_status(name, namespace=namespace))
    client.wait_for_job(name, namespace=namespace, watch=True, timeout_seconds=600)
    ok = client.is_job_succeeded(name, namespace=namespace)
    print("succeeded:", ok)
    logs = client.get_logs(name, namespace=namespace)
    for pod, text in (logs.items() if isinstance(logs, dict) else [("master", logs)]):
        tail = "\n".join(str(text).splitlines()[-5:])
        print(f"--- {pod} (last lines)\n{tail}")
    client.delete(name, namespace=namespace)
    print("deleted")
    return bool(ok)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--url", help="API server of a running stack (default: start one in-process)")
    p.add_argument("--gpu", action="store_true", help="one MI355X per replica, RCCL")
    p.add_argument("--steps", type=int, default=40, help="training steps per replica")
    a = p.parse_args(argv)
    if a.url:
        return 0 if walkthrough(a.url, a.gpu, a.steps) else 1
    with local_stack(a.gpu) as url:
        return 0 if walkthrough(url, a.gpu, a.steps) else 1


if __name__ == "__main__":
    sys.exit(main())
