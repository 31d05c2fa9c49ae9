"""Whole stack on a real MI355X: PyTorchJob -> controller -> node agent
(GPU pinned with HIP_VISIBLE_DEVICES) -> fused HIP trainer; plus the
submit -> first optimizer step latency that BASELINE.json asks for."""
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
