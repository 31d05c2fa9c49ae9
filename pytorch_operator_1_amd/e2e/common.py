"""Shared driver logic for the e2e programs (reference
``test/e2e/v1/default/defaults.go`` and
``test/e2e/v1/cleanpolicy/cleanpolicy_all.go``: create a Master 1 + Worker 3
job, poll every few seconds until Succeeded/Failed, assert, delete, wait for
the job to disappear; ``--num_jobs`` copies run concurrently)."""
from __future__ import annotations

import argparse
import logging
import sys
import time
from concurrent.futures import ThreadPoolExecutor

from ..api import constants as C
from ..api.types import gen_general_name, new_job
from ..apiserver.store import ApiError
from ..utils.misc import pformat, rand_string

log = logging.getLogger("e2e")


def parse(argv, prog):
    p = argparse.ArgumentParser(prog=prog)
    p.add_argument("--name", default="", help="job name (default example-job-<rand>)")
    p.add_argument("--namespace", default="kubeflow")
    p.add_argument("--num_jobs", type=int, default=1)
    p.add_argument("--timeout", type=float, default=600.0, help="seconds")
    p.add_argument("--image", default="pto/pytorch-sendrecv:rocm", help="test image (node-agent image map)")
    p.add_argument("--workers", type=int, default=3)
    p.add_argument("--poll", type=float, default=1.0, help="poll interval seconds (reference: 5)")
    p.add_argument("--server", default=None, help="API server URL; default: start a LocalCluster")
    p.add_argument("--gpus", type=int, default=0, help="LocalCluster GPUs (0 = CPU/gloo)")
    return p.parse_args(argv)


def has_condition(job, ctype) -> bool:
    return any(c.get("type") == ctype and c.get("status") == "True"
               for c in (job.get("status") or {}).get("conditions") or [])


def wait_finished(client, ns, name, timeout, poll):
    job, end = None, time.time() + timeout
    while time.time() < end:
        job = client.get(C.PLURAL, ns, name)
        if has_condition(job, C.JOB_SUCCEEDED) or has_condition(job, C.JOB_FAILED):
            log.info("job %s finished:\n%s", name, pformat(job.get("status")))
            return job
        time.sleep(poll)
    return job


def wait_gone(fn, timeout, poll) -> bool:
    end = time.time() + timeout
    while time.time() < end:
        if fn():
            return True
        time.sleep(poll)
    return False


def make_job(args, name, clean_pod_policy=None):
    job = new_job(name, image=args.image, workers=args.workers, namespace=args.namespace)
    if clean_pod_policy:
        job["spec"]["cleanPodPolicy"] = clean_pod_policy
    return job


def main(argv, prog, scenario):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    args = parse(argv, prog)
    cluster = None
    if args.server:
        from ..apiserver.client import RestClient

        client = RestClient(args.server)
    else:
        from ..cluster import LocalCluster

        cluster = LocalCluster(gpus=args.gpus).start()
        client = cluster.rest_client()
    try:
        def one(i):
            name = args.name or f"example-job-{rand_string(5)}"
            if args.num_jobs > 1 and args.name:
                name = f"{args.name}-{i}"
            try:
                scenario(client, args, name)
                log.info("Job %s ran successfully", name)
                return True
            except Exception as e:  # noqa: BLE001 - report every job
                log.error("Job %s didn't run successfully; %s", name, e)
                return False

        with ThreadPoolExecutor(max_workers=max(1, args.num_jobs)) as ex:
            results = list(ex.map(one, range(args.num_jobs)))
    finally:
        if cluster is not None:
            cluster.stop()
    ok = sum(results)
    log.info("%d jobs succeeded, %d failed", ok, len(results) - ok)
    return 0 if ok == len(results) else 1


def expect_deleted_job(client, ns, name, args):
    client.delete(C.PLURAL, ns, name)

    def gone():
        try:
            client.get(C.PLURAL, ns, name)
            return False
        except ApiError as e:
            return e.code == 404

    if not wait_gone(gone, args.timeout, args.poll):
        raise RuntimeError(f"Deletion of PyTorchJob {name} failed")


def expect_pods_exist(client, ns, job):
    for rtype, spec in job["spec"]["pytorchReplicaSpecs"].items():
        for i in range(int(spec.get("replicas", 1))):
            pod = gen_general_name(job["metadata"]["name"], rtype.lower(), i)
            try:
                client.get("pods", ns, pod)
            except ApiError:
                raise RuntimeError(f"PyTorchJob {job['metadata']['name']} did not create pod {pod} "
                                   f"for ReplicaType {rtype} Index {i}") from None


if __name__ == "__main__":  # pragma: no cover
    sys.exit(2)
