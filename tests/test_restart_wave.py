"""Restart waves of multi-replica jobs (round-2
kill/rejoin stall, docs/multi_gpu.md "Restarts").

The race, reproduced deterministically by ``rdzv_probe.py``: a worker dies,
and the job's old master is still alive, serving the rendezvous store on the
job's port, when the worker is recreated.  A recreated replica that joins
that store is in the wrong world.

* ``restart_scope="pod"`` (the reference: delete only the failed pod) shows
  the race: the recreated worker reaches the old store, refuses it
  (``StaleRendezvous``, restart generations) and the job fails once the old
  master gives up.
* ``restart_scope="job"`` (default): every replica is deleted, the new pods
  are held until the last old process has exited, and the whole new world
  rendezvouses under the next generation.
* ``OnFailure``: the agent's restart group takes the survivors down and
  restarts all replicas together, in place (restartCount counts it).
"""
import os
import re
import sys
import time

import pytest

from pytorch_operator_1_amd.api.types import new_job
from pytorch_operator_1_amd.cluster import LocalCluster

pytestmark = pytest.mark.slow

PROBE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rdzv_probe.py")


def _probe_job(name, marker, workers, policy, hold=20.0, linger=3.0, backoff_limit=8):
    args = [PROBE, "--marker", marker, "--fail-rank", "1", "--hold", str(hold), "--linger", str(linger)]
    job = new_job(name, image="pto/python:rocm", master_args=args, workers=workers, restart_policy=policy)
    job["spec"]["backoffLimit"] = backoff_limit
    return job


def _logs(c, name, workers):
    names = [f"{name}-master-0"] + [f"{name}-worker-{i}" for i in range(workers)]
    return {n: c.pod_log("default", n) for n in names}


@pytest.fixture
def cluster(tmp_path, request):
    scope = getattr(request, "param", "job")
    c = LocalCluster(gpus=0, log_dir=str(tmp_path / "pods"), restart_scope=scope,
                     extra_env={"OMP_NUM_THREADS": "1"}).start()
    yield c
    c.stop()


@pytest.mark.timeout(240)
def test_exitcode_job_wave_waits_for_old_master(cluster, tmp_path):
    """Worker 0 dies (137); the old master lingers 3 s after SIGTERM while
    holding the store.  Every replica is recreated, none starts before the
    old master has exited, and the new world joins generation 1."""
    name = "wave"
    cluster.submit(_probe_job(name, str(tmp_path / "marker"), workers=2, policy="ExitCode"))
    j = cluster.wait_for_condition(name, timeout=180)
    logs = _logs(cluster, name, 2)
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", (j["status"], logs)
    for n, log in logs.items():
        assert "STALE" not in log, (n, log)
        m = re.search(r"DONE rank=\d+ gen=(\S+)", log)
        assert m and m.group(1) == "1", (n, log)
    reasons = [e["reason"] for e in cluster.store.list("events", "default")["items"]
               if e["involvedObject"]["name"] == name]
    assert "ExitedWithCode" in reasons and "PyTorchJobRestarting" in reasons, reasons
    msgs = [e["message"] for e in cluster.store.list("events", "default")["items"]
            if e["reason"] == "PyTorchJobRestarting" and e["involvedObject"]["name"] == name]
    assert any("restarting all 3 replicas" in m for m in msgs), msgs


@pytest.mark.timeout(240)
@pytest.mark.parametrize("cluster", ["pod"], indirect=True)
def test_exitcode_pod_scope_reproduces_stale_store(cluster, tmp_path):
    """Reference semantics (only the failed pod is recreated): the new
    worker starts while the old master still serves the port and reaches
    the old world's store.  Generations make that a clean refusal instead of
    a hang; the job fails when the old master gives up (exit 1)."""
    name = "perpod"
    cluster.submit(_probe_job(name, str(tmp_path / "marker"), workers=1, policy="ExitCode", hold=8.0))
    j = cluster.wait_for_condition(name, timeout=180)
    assert j["status"]["conditions"][-1]["type"] == "Failed", j["status"]
    ev = [e["message"] for e in cluster.store.list("events", "default")["items"]
          if e["reason"] == "ExitedWithCode" and e["involvedObject"]["name"] == name]
    assert any("exited with code 138" in m for m in ev), ev  # the STALE refusal's retryable exit


@pytest.mark.timeout(240)
def test_onfailure_group_restarts_in_place(cluster, tmp_path):
    """In-place restarts: the killed worker's group (its job) is stopped and
    restarted together under generation 0.1, and the job succeeds.  The
    wave counts as ONE restart (the failed replica's), so a 4-replica job
    with backoffLimit 2 survives one kill (per-member counting
    made every wave cost N restarts against pastBackoffLimit)."""
    name = "group"
    cluster.submit(_probe_job(name, str(tmp_path / "marker"), workers=3, policy="OnFailure", backoff_limit=2))
    j = cluster.wait_for_condition(name, timeout=180)
    logs = _logs(cluster, name, 3)
    assert j["status"]["conditions"][-1]["type"] == "Succeeded", (j["status"], logs)
    for n, log in logs.items():
        assert re.search(r"DONE rank=\d+ gen=0\.1\b", log), (n, log)
        assert "STALE" not in log and "GAVE-UP" not in log, (n, log)
    counts = {n: cluster.store.get("pods", "default", n)["status"]["containerStatuses"][0]["restartCount"]
              for n in [f"{name}-master-0"] + [f"{name}-worker-{i}" for i in range(3)]}
    assert counts[f"{name}-worker-0"] == 1 and sum(counts.values()) == 1, counts


def test_agent_restart_group_unit(tmp_path):
    """The agent alone: a failing member kills its group, all members are
    held until the last exits, then restart together with the wave's
    generation; a member of another group is untouched."""
    from pytorch_operator_1_amd.node.native import AgentClient

    a = AgentClient(gpus=0)
    try:
        py = sys.executable
        marker = tmp_path / "m"
        fail = (f"import os,sys,time; m={str(marker)!r}; first=not os.path.exists(m); "
                f"open(m,'a').close(); time.sleep(0.3 if first else 0.2); sys.exit(3 if first else 0)")
        env = {"PTO_RESTART_GENERATION": "4", "PATH": os.environ.get("PATH", "")}
        a.spawn("g/a", [py, "-c", fail], env=env, restart_policy="OnFailure", group="g",
                log=str(tmp_path / "a.log"))
        a.spawn("g/b", [py, "-c", "import time; time.sleep(60)"], env=env, restart_policy="OnFailure", group="g",
                log=str(tmp_path / "b.log"))
        a.spawn("h/c", [py, "-c", "import time; time.sleep(60)"], env=env, restart_policy="OnFailure", group="h")
        end = time.time() + 30
        st = {}
        while time.time() < end:
            st = a.status()
            if st["g/a"]["state"] == "terminated" and st["g/a"]["restart_count"] == 1:
                break
            time.sleep(0.05)
        assert st["g/a"]["exit_code"] == 0 and st["g/a"]["generation"] == "4.1", st
        # killed by the wave, restarted with it, but not charged a restart
        assert st["g/b"]["restart_count"] == 0 and st["g/b"]["generation"] == "4.1", st
        assert st["g/b"]["state"] == "running" and st["g/b"]["last_exit_code"] == 137, st
        assert st["h/c"]["restart_count"] == 0 and st["h/c"]["state"] == "running", st
    finally:
        for i in ("g/a", "g/b", "h/c"):
            a.kill(i, signal=9)
        a.close()


def test_agent_wave_never_revives_completed_member(tmp_path):
    """A member that already exited 0 (OnFailure: Completed -- e.g. the
    Master, whose success completes the job, reference status.go:99-106)
    when a peer fails stays terminated: a succeeded pod is terminal in
    Kubernetes.  The failed peer restarts alone under the next generation
    (ADVICE r4)."""
    from pytorch_operator_1_amd.node.native import AgentClient

    a = AgentClient(gpus=0)
    try:
        py = sys.executable
        marker = tmp_path / "m"
        fail = (f"import os,sys,time; m={str(marker)!r}; first=not os.path.exists(m); "
                f"open(m,'a').close(); time.sleep(1.0 if first else 0.2); sys.exit(3 if first else 0)")
        env = {"PTO_RESTART_GENERATION": "2", "PATH": os.environ.get("PATH", "")}
        a.spawn("g/done", [py, "-c", "import os; print('gen', os.environ['PTO_RESTART_GENERATION'])"], env=env,
                restart_policy="OnFailure", group="g", log=str(tmp_path / "done.log"))
        a.spawn("g/fail", [py, "-c", fail], env=env, restart_policy="OnFailure", group="g",
                log=str(tmp_path / "fail.log"))
        end = time.time() + 30
        st = {}
        while time.time() < end:
            st = a.status()
            if st["g/fail"]["state"] == "terminated" and st["g/fail"]["restart_count"] == 1:
                break
            time.sleep(0.05)
        assert st["g/fail"]["exit_code"] == 0 and st["g/fail"]["generation"] == "2.1", st
        assert st["g/done"]["state"] == "terminated" and st["g/done"]["exit_code"] == 0, st
        assert st["g/done"]["generation"] == "2" and st["g/done"]["restart_count"] == 0, st
        assert (tmp_path / "done.log").read_text().count("gen ") == 1
    finally:
        for i in ("g/done", "g/fail"):
            a.kill(i, signal=9)
        a.close()
