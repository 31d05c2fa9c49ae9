"""Whole stack on a real MI355X: PyTorchJob -> controller -> node agent
(GPU pinned with HIP_VISIBLE_DEVICES) -> fused HIP trainer; plus the
submit -> first optimizer step latency that BASELINE.json asks for."""
import os
import time

import pytest

from pytorch_operator_1_amd.api.types import new_job
from pytorch_operator_1_amd.cluster import LocalCluster

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    c = LocalCluster(gpus=None, log_dir=str(tmp_path_factory.mktemp("pods"))).start()
    yield c
    c.stop()


@pytest.mark.timeout(360)
def test_gpu_job_runs_fused_trainer(cluster):
    t0 = time.time()
    job = new_job("mnist-gpu", image="pto/pytorch-mnist:rocm",
                  master_args=["--backend", "rccl", "--impl", "fused", "--max-steps", "300", "--log-interval", "100"],
                  workers=0, gpus=1)
    cluster.submit(job)
    j = cluster.wait_for_condition("mnist-gpu", timeout=300)
    log = cluster.pod_log("default", "mnist-gpu-master-0")
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", log[-3000:]
    assert "Using CUDA (HIP)" in log and "accuracy=" in log
    pod = cluster.store.get("pods", "default", "mnist-gpu-master-0")
    assert pod["metadata"]["annotations"]["pto.amd.com/gpus"] == "0"
    first = float(pod["metadata"]["annotations"]["pto.amd.com/first-step-unix"])
    latency = first - t0
    print(f"submit -> first optimizer step: {latency:.2f} s")
    assert 0 < latency < 120


@pytest.mark.timeout(120)
def test_gang_admission_unschedulable_when_gpus_exhausted(cluster):
    n = cluster.kubelet.agent.gpus()["count"]
    job = new_job("too-big", image="pto/python:rocm", master_args=["-c", "print(1)"], workers=0, gpus=n + 1)
    cluster.submit(job)
    end = time.time() + 30
    while time.time() < end:
        try:
            pod = cluster.store.get("pods", "default", "too-big-master-0")
            conds = pod.get("status", {}).get("conditions") or []
            if any(c.get("reason") == "Unschedulable" for c in conds):
                break
        except Exception:
            pass
        time.sleep(0.1)
    assert pod["status"]["phase"] == "Pending"
    assert any(c.get("reason") == "Unschedulable" for c in pod["status"]["conditions"])
    cluster.store.delete("pytorchjobs", "default", "too-big")


@pytest.mark.timeout(360)
def test_gpu_kill_rejoin_resumes_fused_trainer(cluster, tmp_path):
    """Config 5 on the GPU: the fused HIP trainer is SIGKILLed mid-run
    (exit 137, retryable) -> ExitCode policy recreates the pod on the same
    GPU -> it resumes from the flat-buffer checkpoint and the job succeeds."""
    import os

    ck = str(tmp_path / "ckpt")
    job = new_job("mnist-gpu-kill", image="pto/pytorch-mnist:rocm",
                  master_args=["--backend", "rccl", "--impl", "fused", "--max-steps", "200", "--log-interval", "50",
                               "--checkpoint-dir", ck, "--checkpoint-interval", "50", "--fail-at-step", "120",
                               "--fail-rank", "0", "--no-test"],
                  workers=0, gpus=1, restart_policy="ExitCode")
    job["spec"]["backoffLimit"] = 3
    cluster.submit(job)
    j = cluster.wait_for_condition("mnist-gpu-kill", timeout=300)
    log = cluster.pod_log("default", "mnist-gpu-kill-master-0")
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", (j["status"], log[-2000:])
    assert "Resumed from" in log and "at step 100" in log
    assert any(f.startswith("ckpt-") for f in os.listdir(ck))


# ---------------------------------------------------------------------------
# BASELINE config 2 rehearsed through the operator on the one-GPU box: the
# node manager offers the GPU as 4 allocatable slots (test-only gpu_share),
# so Master=1 Worker=3 with amd.com/gpu:1 each lands on one device; ranks
# rendezvous with gloo and all-reduce gradients with the same-device xGMI
# kernel (RCCL refuses duplicate devices).  On the 8-GPU node the same spec
# runs with --backend rccl, one GPU per replica.

_SHARED_ARGS = ["--backend", "gloo", "--impl", "fused", "--comm", "xgmi", "--log-interval", "50", "--no-test",
                "--train-size", "16384"]
_SHARED_ENV = {"PTO_FAULTHANDLER": "1"}  # SIGUSR2 dumps every thread's stack (PTO_TEST_DUMP_AFTER)


@pytest.fixture(scope="module")
def shared_cluster(tmp_path_factory):
    c = LocalCluster(gpus=None, log_dir=str(tmp_path_factory.mktemp("pods-shared")), gpu_share=4,
                     gpu_visibility="node").start()
    yield c
    c.stop()


def _wait_verbose(c, name, timeout, dump_after=None):
    """wait_for_condition that prints the job state and each replica's last
    log line every 15 s (a silent multi-minute wait reads as a hang); after
    ``dump_after`` s the replicas are sent SIGUSR2 (stack dump)."""
    start = time.time()
    end = start + timeout
    dumped = False
    while True:
        try:
            return c.wait_for_condition(name, timeout=min(15.0, max(0.1, end - time.time())))
        except TimeoutError:
            if time.time() >= end:
                for n in _replicas(name):  # full logs (faulthandler stacks included) for the report
                    print(f"==== {n}\n" + "\n".join(c.pod_log("default", n).splitlines()[-80:]), flush=True)
                raise
            if dump_after and time.time() > start + dump_after and not dumped:
                dumped = True  # PTO_FAULTHANDLER pods dump every thread's stack on SIGUSR2
                for n in _replicas(name):
                    try:
                        c.kubelet.inject_fault("default", n, signal=12)
                    except Exception:  # noqa: BLE001
                        pass
            j = c.store.get("pytorchjobs", "default", name)
            conds = [x["type"] for x in j.get("status", {}).get("conditions") or []]
            print(f"[wait {name}] conditions={conds}", flush=True)
            for n in _replicas(name):
                try:
                    pod = c.store.get("pods", "default", n)
                    tail = (c.pod_log("default", n).strip().splitlines() or [""])[-1][-160:]
                    print(f"  {n} {pod.get('status', {}).get('phase')}: {tail}", flush=True)
                except Exception as e:  # noqa: BLE001
                    print(f"  {n}: {e}", flush=True)


def _replicas(job):
    return [f"{job}-master-0"] + [f"{job}-worker-{i}" for i in range(3)]


@pytest.mark.timeout(420)
def test_config2_master1_worker3_through_operator(shared_cluster):
    c = shared_cluster
    job = new_job("mnist-w3", image="pto/pytorch-mnist:rocm", master_args=_SHARED_ARGS + ["--max-steps", "200"],
                  workers=3, gpus=1, env=_SHARED_ENV)
    c.submit(job)
    j = _wait_verbose(c, "mnist-w3", timeout=360)
    logs = {n: c.pod_log("default", n) for n in _replicas("mnist-w3")}
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", (j["status"], logs["mnist-w3-master-0"][-3000:])
    for n, log in logs.items():
        assert "Train Epoch: 1 [6400/16384" in log, (n, log[-2000:])
    assert "'transport': 'xgmi'" in logs["mnist-w3-master-0"]
    assert "Using distributed PyTorch with gloo backend" in logs["mnist-w3-master-0"]


@pytest.mark.timeout(420)
@pytest.mark.parametrize("policy", ["ExitCode", "OnFailure"])
def test_config2_kill_rejoin_every_replica_resumes(shared_cluster, tmp_path, policy):
    """Worker 0 (rank 1) is SIGKILLed at step 120 (exit 137, retryable).
    ExitCode: the controller deletes all four pods (job-level restart) and
    the node manager starts the new ones only after every old process has
    exited.  OnFailure: the node agent's restart group stops the other three
    replicas and restarts all four in place.  Either way the new world
    rendezvouses under a new restart generation, agrees on the newest
    checkpoint (step 100) and finishes the job."""
    c = shared_cluster
    ck = str(tmp_path / "ckpt")
    name = f"mnist-w3-{policy.lower()}"
    args = _SHARED_ARGS + ["--max-steps", "200", "--checkpoint-dir", ck, "--checkpoint-interval", "50",
                           "--fail-at-step", "120", "--fail-rank", "1"]
    job = new_job(name, image="pto/pytorch-mnist:rocm", master_args=args, workers=3, gpus=1,
                  env=_SHARED_ENV, restart_policy=policy)
    job["spec"]["backoffLimit"] = 12
    c.submit(job)
    # well inside the test's own timeout, so a failure prints every replica's log
    j = _wait_verbose(c, name, timeout=int(os.environ.get("PTO_TEST_KILL_TIMEOUT", "300")),
                      dump_after=float(os.environ.get("PTO_TEST_DUMP_AFTER", "0")) or None)
    logs = {n: c.pod_log("default", n) for n in _replicas(name)}
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", (j["status"], logs)
    import re

    for n, log in logs.items():
        m = re.search(r"Resumed from \S+ at step (\d+)", log)
        assert m and int(m.group(1)) >= 100, (n, log[-2000:])
    if policy == "ExitCode":
        # Restarting is not in the final conditions (Running replaces it,
        # status.go filterOutCondition); the restart shows in the events
        msgs = [e.get("message", "") for e in c.store.list("events", "default")["items"]
                if e.get("involvedObject", {}).get("name") == name and e.get("reason") == "PyTorchJobRestarting"]
        assert any("restarting all 4 replicas" in m for m in msgs), msgs
    else:
        pod = c.store.get("pods", "default", f"{name}-worker-0")
        assert pod["status"]["containerStatuses"][0]["restartCount"] >= 1, pod["status"]
