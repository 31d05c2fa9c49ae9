"""GPU pinning env of an 8-replica job (BASELINE config 2 shape: Master=1
Worker=7, amd.com/gpu:1 each) under both visibility models, and the
pytorchjob_* Prometheus series fed from a finished job."""
import json
import os
import socket
import urllib.request

import pytest

from pytorch_operator_1_amd.api.types import new_job
from pytorch_operator_1_amd.cluster import LocalCluster

pytestmark = pytest.mark.slow

KEYS = ["RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "HIP_VISIBLE_DEVICES",
        "PTO_GPU_IDS", "PTO_MASTER_SERVICE"]
PRINT_ENV = "import os,json; print('ENV ' + json.dumps({k: os.environ.get(k) for k in %r}))" % KEYS


def _wait_pods_done(c, names, timeout=120):
    """The job succeeds when its Master does; workers may still be running."""
    import time

    end = time.time() + timeout
    while time.time() < end:
        phases = [c.store.get("pods", "default", n).get("status", {}).get("phase") for n in names]
        if all(p == "Succeeded" for p in phases):
            return
        time.sleep(0.05)
    raise TimeoutError(f"pods not done: {dict(zip(names, phases))}")


def _envs(c, job, n):
    out = {}
    names = [f"{job}-master-0"] + [f"{job}-worker-{i}" for i in range(n - 1)]
    _wait_pods_done(c, names)
    for name in names:
        line = [x for x in c.pod_log("default", name).splitlines() if x.startswith("ENV ")]
        assert line, c.pod_log("default", name)
        out[name] = json.loads(line[0][4:])
        pod = c.store.get("pods", "default", name)
        eff = json.loads(pod["metadata"]["annotations"]["pto.amd.com/effective-env"])
        assert eff["MASTER_PORT"] == out[name]["MASTER_PORT"] and eff["LOCAL_RANK"] == out[name]["LOCAL_RANK"]
    return out


@pytest.mark.parametrize("mode", ["job", "node", "isolated"])
def test_master1_worker7_gpu_env(tmp_path, mode):
    # gang admission: all 8 GPUs are assigned at once (a replica that finished
    # early would otherwise hand its GPU to one admitted after it)
    with LocalCluster(gpus=8, log_dir=str(tmp_path), gpu_visibility=mode, enable_gang_scheduling=True) as c:
        job = f"pin-{mode}"
        c.submit(new_job(job, image="pto/python:rocm", master_args=["-c", PRINT_ENV], workers=7, gpus=1))
        j = c.wait_for_condition(job, timeout=120)
        assert j["status"]["conditions"][-1]["type"] == "Succeeded", j["status"]
        envs = _envs(c, job, 8)
    ranks = sorted(int(e["RANK"]) for e in envs.values())
    assert ranks == list(range(8))
    assert {e["WORLD_SIZE"] for e in envs.values()} == {"8"}
    assert {e["MASTER_ADDR"] for e in envs.values()} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs.values()}) == 1
    assert {e["PTO_MASTER_SERVICE"] for n, e in envs.items() if "worker" in n} == {f"pin-{mode}-master-0"}
    gpu_ids = sorted(int(e["PTO_GPU_IDS"]) for e in envs.values())
    assert gpu_ids == list(range(8))  # every GPU handed to exactly one replica
    if mode == "job":
        # own GPU first (cuda:0), then the job's 7 other GPUs: peers enumerable for RCCL P2P / xGMI IPC
        for e in envs.values():
            vis = e["HIP_VISIBLE_DEVICES"].split(",")
            assert vis[0] == e["PTO_GPU_IDS"] and sorted(map(int, vis)) == list(range(8)), e
        assert {e["LOCAL_RANK"] for e in envs.values()} == {"0"}
    elif mode == "node":
        assert {e["HIP_VISIBLE_DEVICES"] for e in envs.values()} == {"0,1,2,3,4,5,6,7"}
        assert all(e["LOCAL_RANK"] == e["PTO_GPU_IDS"] for e in envs.values())
        assert {e["LOCAL_WORLD_SIZE"] for e in envs.values()} == {"8"}
    else:
        assert all(e["HIP_VISIBLE_DEVICES"] == e["PTO_GPU_IDS"] for e in envs.values())
        assert {e["LOCAL_RANK"] for e in envs.values()} == {"0"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_training_gauges_scraped_for_finished_gloo_job(tmp_path):
    from pytorch_operator_1_amd.controller.metrics import serve_metrics

    sysfs = tmp_path / "sys"
    for card, used in (("card0", 1 << 30), ("card1", 2 << 30)):
        d = sysfs / "class" / "drm" / card / "device"
        d.mkdir(parents=True)
        (d / "mem_info_vram_used").write_text(f"{used}\n")
        (d / "mem_info_vram_total").write_text(f"{288 << 30}\n")
    with LocalCluster(gpus=0, log_dir=str(tmp_path / "pods"), extra_env={"OMP_NUM_THREADS": "2"}) as c:
        c.kubelet.sysfs_root = str(sysfs)
        c.kubelet.update_node_metrics()
        args = ["--backend", "gloo", "--no-cuda", "--max-steps", "30", "--log-interval", "10", "--train-size", "2560",
                "--no-test"]
        c.submit(new_job("gauges", image="pto/pytorch-mnist:rocm", master_args=args, workers=1))
        j = c.wait_for_condition("gauges", timeout=180)
        assert j["status"]["conditions"][-1]["type"] == "Succeeded", j["status"]
        port = _free_port()
        srv = serve_metrics(c.metrics, port, host="127.0.0.1")
        try:
            text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
        finally:
            if isinstance(srv, tuple):
                srv[0].shutdown()
    series = {}
    for line in text.splitlines():
        if line.startswith("pytorchjob_"):
            name, val = line.rsplit(" ", 1)
            series[name] = float(val)
    for rep in ("master-0", "worker-0"):
        k = f'pytorchjob_samples_per_second{{job="gauges",replica="{rep}"}}'
        assert series.get(k, 0) > 0, sorted(series)
        assert series.get(f'pytorchjob_step_seconds{{job="gauges",replica="{rep}"}}', 0) > 0
    s2f = series.get('pytorchjob_submit_to_first_step_seconds{job="gauges"}')
    assert s2f is not None and 0 < s2f < 120
    assert series['pytorchjob_gpu_hbm_used_bytes{gpu="card1"}'] == float(2 << 30)
    assert series['pytorchjob_gpu_hbm_total_bytes{gpu="card0"}'] == float(288 << 30)


def test_job_port_released_after_job_deleted(tmp_path):
    """A job's virtual master port (and its host-wide lock) is given back
    once the job's pods are gone, so a long-running node does not walk the
    port range one job at a time."""
    import time

    with LocalCluster(gpus=0, log_dir=str(tmp_path)) as c:
        k = c.kubelet
        c.submit(new_job("port-a", image="pto/python:rocm", master_args=["-c", "print('ok')"], workers=0, gpus=0))
        j = c.wait_for_condition("port-a", timeout=60)
        assert j["status"]["conditions"][-1]["type"] == "Succeeded", j["status"]
        assert "default/port-a" in k.job_ports
        port = k.job_ports["default/port-a"]
        assert port in k._port_locks
        c.store.delete("pytorchjobs", "default", "port-a")
        end = time.time() + 30
        while time.time() < end and "default/port-a" in k.job_ports:
            time.sleep(0.05)
        assert "default/port-a" not in k.job_ports and port not in k._port_locks
        c.submit(new_job("port-b", image="pto/python:rocm", master_args=["-c", "print('ok')"], workers=0, gpus=0))
        c.wait_for_condition("port-b", timeout=60)
        assert k.job_ports["default/port-b"] == port  # the same base port is free again
