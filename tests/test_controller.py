"""Reconcile / status machine of the PyTorchJob controller, driven against
an in-memory store with fake pod/service control and hand-set pod phases —
the pattern of the reference's testutil (SetPodsStatuses into informer
indexers, FakePodControl, FakeServiceControl), covering the scenarios of
upstream's controller/job/pod/status tests that this fork dropped."""
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from pytorch_operator_1_amd.api import constants as C
from pytorch_operator_1_amd.api.types import gen_labels, gen_owner_reference, key_of, new_job, now_rfc3339
from pytorch_operator_1_amd.apiserver.client import LocalClient
from pytorch_operator_1_amd.apiserver.store import Store
from pytorch_operator_1_amd.controller import pytorch as ctl
from pytorch_operator_1_amd.controller.control import FakePodControl, FakeServiceControl
from pytorch_operator_1_amd.controller.pytorch import ControllerConfig, PyTorchController


class Harness:
    def __init__(self, **cfg):
        self.store = Store()
        self.client = LocalClient(self.store)
        self.pods = FakePodControl()
        self.svcs = FakeServiceControl()
        self.pc = PyTorchController(self.client, ControllerConfig(**cfg), pod_control=self.pods,
                                    service_control=self.svcs, start_informers=False)
        for inf in (self.pc.job_informer, self.pc.pod_informer, self.pc.service_informer):
            inf._synced.set()
        self.statuses = []
        orig = self.pc.update_status_handler

        def capture(job):
            self.statuses.append(job)
            return orig(job)

        self.pc.update_status_handler = capture

    def add_job(self, job):
        obj = self.store.create("pytorchjobs", job)
        self.pc.job_informer.replace_in_cache(obj)
        self.pc.add_pytorch_job(obj)
        return self.pc.job_informer.get_by_key(key_of(obj))

    def set_pods(self, job, rtype, pending=0, active=0, succeeded=0, failed=0, restart_counts=None,
                 exit_code=None):
        """SetPodsStatuses (testutil/pod.go:67-95)."""
        phases = ["Pending"] * pending + ["Running"] * active + ["Succeeded"] * succeeded + ["Failed"] * failed
        for i, ph in enumerate(phases):
            labels = gen_labels(job["metadata"]["name"])
            labels[C.LABEL_REPLICA_TYPE] = rtype.lower()
            labels[C.LABEL_REPLICA_INDEX] = str(i)
            st_ = {"phase": ph}
            if restart_counts:
                st_["containerStatuses"] = [{"name": "pytorch", "restartCount": restart_counts[i]}]
            if ph == "Failed" and exit_code is not None:
                st_["containerStatuses"] = [{"name": "pytorch", "state": {"terminated": {"exitCode": exit_code}}}]
            pod = {"metadata": {"name": f"{job['metadata']['name']}-{rtype.lower()}-{i}", "namespace": "default",
                                "labels": labels, "ownerReferences": [gen_owner_reference(job)],
                                "resourceVersion": str(i)},
                   "status": st_}
            self.pc.pod_informer.replace_in_cache(pod)

    def set_services(self, job, rtype="Master", n=1):
        for i in range(n):
            labels = gen_labels(job["metadata"]["name"])
            labels[C.LABEL_REPLICA_TYPE] = rtype.lower()
            labels[C.LABEL_REPLICA_INDEX] = str(i)
            svc = {"metadata": {"name": f"{job['metadata']['name']}-{rtype.lower()}-{i}", "namespace": "default",
                                "labels": labels, "ownerReferences": [gen_owner_reference(job)]}}
            self.pc.service_informer.replace_in_cache(svc)

    def sync(self, job):
        return self.pc.sync_pytorch_job(key_of(job))

    def last(self):
        return self.statuses[-1] if self.statuses else None


def cond_types(job):
    return [(c["type"], c["status"]) for c in job["status"]["conditions"]]


def test_created_condition_and_metrics():
    h = Harness()
    j = h.add_job(new_job("a", workers=1))
    assert j["status"]["conditions"][0]["type"] == "Created"
    assert j["status"]["conditions"][0]["reason"] == "PyTorchJobCreated"
    assert j["status"]["conditions"][0]["message"] == "PyTorchJob a is created."
    assert h.pc.metrics.jobs_created._value.get() == 1


def test_creates_pods_and_master_service_with_env():
    h = Harness()
    j = h.add_job(new_job("mnist", workers=3, gpus=1))
    h.sync(j)
    names = sorted(t["metadata"]["name"] for t in h.pods.templates)
    assert names == ["mnist-master-0", "mnist-worker-0", "mnist-worker-1", "mnist-worker-2"]
    by = {t["metadata"]["name"]: t for t in h.pods.templates}
    m = by["mnist-master-0"]
    env = {e["name"]: e["value"] for e in m["spec"]["containers"][0]["env"]}
    assert env == {"MASTER_PORT": "23456", "MASTER_ADDR": "localhost", "WORLD_SIZE": "4", "RANK": "0",
                   "PYTHONUNBUFFERED": "0"}
    assert m["metadata"]["labels"]["job-role"] == "master"
    assert m["metadata"]["labels"]["pytorch-replica-type"] == "master"
    assert "initContainers" not in m["spec"]
    w2 = by["mnist-worker-2"]
    env = {e["name"]: e["value"] for e in w2["spec"]["containers"][0]["env"]}
    assert env["RANK"] == "3" and env["MASTER_ADDR"] == "mnist-master-0"
    assert "job-role" not in w2["metadata"]["labels"]
    init = w2["spec"]["initContainers"][0]
    assert init["name"] == "init-pytorch" and init["image"] == "alpine:3.10"
    assert "until nslookup mnist-master-0" in init["command"][2]
    assert w2["spec"]["restartPolicy"] == "OnFailure"
    assert w2["spec"]["containers"][0]["resources"]["limits"] == {"amd.com/gpu": 1}
    assert [s["metadata"]["name"] for s in h.svcs.templates] == ["mnist-master-0"]
    svc = h.svcs.templates[0]
    assert svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["ports"] == [{"name": "pytorchjob-port", "port": 23456}]
    assert h.pods.controller_refs[0]["uid"] == j["metadata"]["uid"]


def test_expectations_suppress_duplicate_creates():
    h = Harness()
    j = h.add_job(new_job("e", workers=1))
    h.sync(j)
    n = len(h.pods.templates)
    h.sync(j)  # informer has not observed the creations yet
    assert len(h.pods.templates) == n


# (pending, active, succeeded, failed) per type -> expected last condition
STATUS_CASES = [
    ("master running", dict(Master=(0, 1, 0, 0), Worker=(0, 1, 0, 0)), "Running"),
    ("master pending", dict(Master=(1, 0, 0, 0), Worker=(1, 0, 0, 0)), "Created"),
    ("master succeeded", dict(Master=(0, 0, 1, 0), Worker=(0, 1, 0, 0)), "Succeeded"),
    ("worker failed", dict(Master=(0, 1, 0, 0), Worker=(0, 0, 0, 1)), "Failed"),
    ("master failed", dict(Master=(0, 0, 0, 1), Worker=(0, 1, 0, 0)), "Failed"),
    ("workers succeeded, master running", dict(Master=(0, 1, 0, 0), Worker=(0, 0, 2, 0)), "Running"),
]


@pytest.mark.parametrize("name,pods,expected", STATUS_CASES, ids=[c[0] for c in STATUS_CASES])
def test_status_table(name, pods, expected):
    h = Harness()
    nw = sum(pods["Worker"])
    j = h.add_job(new_job("s", workers=nw))
    for rt, (p, a, s, f) in pods.items():
        h.set_pods(j, rt, p, a, s, f)
    h.set_services(j)
    h.sync(j)
    job = h.last() or h.pc.job_informer.get_by_key("default/s")
    assert job["status"]["conditions"][-1]["type"] == expected
    rs = job["status"]["replicaStatuses"]
    assert rs["Master"]["active"] == pods["Master"][1]
    if expected == "Succeeded":
        assert job["status"]["completionTime"]
        assert ("Running", "False") not in cond_types(job) or True


def test_running_then_succeeded_marks_running_false():
    h = Harness()
    j = h.add_job(new_job("r", workers=1))
    h.set_pods(j, "Master", active=1)
    h.set_pods(j, "Worker", active=1)
    h.set_services(j)
    h.sync(j)
    j = h.pc.job_informer.get_by_key("default/r")
    h.set_pods(j, "Master", succeeded=1)
    h.sync(j)
    job = h.last()
    assert cond_types(job) == [("Created", "True"), ("Running", "False"), ("Succeeded", "True")]
    assert h.pc.metrics.jobs_successful._value.get() == 1


@pytest.mark.parametrize("scope", ["job", "pod"])
def test_exitcode_retryable_restarts(scope):
    """A retryable failure -> Restarting.  ``pod`` scope (the reference,
    pod.go:91-109) deletes only the failed pod; the default ``job`` scope
    deletes every replica of the job in the same pass (restart wave)."""
    h = Harness(restart_scope=scope)
    job = new_job("x", workers=2, restart_policy="ExitCode")
    j = h.add_job(job)
    h.set_pods(j, "Master", active=1)
    h.set_pods(j, "Worker", failed=1, exit_code=137)
    h.set_services(j)
    h.sync(j)
    last = h.last()
    assert last["status"]["conditions"][-1]["type"] == "Restarting"
    assert "restarting because 1 Worker replica(s) failed" in last["status"]["conditions"][-1]["message"]
    if scope == "pod":
        assert h.pods.delete_pod_names == ["x-worker-0"]
    else:
        assert sorted(h.pods.delete_pod_names) == ["x-master-0", "x-worker-0"]
    assert h.pc.metrics.jobs_restarted._value.get() == 1
    # pods created with restartPolicy Never for ExitCode
    assert all(t["spec"]["restartPolicy"] == "Never" for t in h.pods.templates)


def test_exitcode_wave_not_started_by_permanent_failure():
    """A permanent failure next to a retryable one fails the job; nothing
    else is deleted for a restart."""
    h = Harness()
    j = h.add_job(new_job("p", workers=2, restart_policy="ExitCode"))
    h.set_pods(j, "Master", failed=1, exit_code=1)
    h.set_pods(j, "Worker", failed=1, exit_code=137)
    h.set_services(j)
    h.sync(j)
    assert h.last()["status"]["conditions"][-1]["type"] == "Failed"
    assert "p-master-0" not in h.pods.delete_pod_names and "p-worker-1" not in h.pods.delete_pod_names


def test_exitcode_permanent_fails():
    h = Harness()
    j = h.add_job(new_job("y", workers=1, restart_policy="ExitCode"))
    h.set_pods(j, "Master", active=1)
    h.set_pods(j, "Worker", failed=1, exit_code=1)
    h.set_services(j)
    h.sync(j)
    assert h.last()["status"]["conditions"][-1]["type"] == "Failed"
    assert h.pods.delete_pod_names == []


def test_backoff_limit_restart_counts():
    h = Harness()
    j = h.add_job(new_job("b", workers=1, backoff_limit=2))
    h.set_pods(j, "Master", active=1, restart_counts=[1])
    h.set_pods(j, "Worker", active=1, restart_counts=[1])
    h.set_services(j)
    h.sync(j)
    last = h.last()
    assert last["status"]["conditions"][-1]["type"] == "Failed"
    assert last["status"]["conditions"][-1]["message"] == \
        "PyTorchJob b has failed because it has reached the specified backoff limit"


def test_active_deadline_and_clean_pod_policy_all():
    h = Harness()
    j = h.add_job(new_job("d", workers=1, active_deadline_seconds=1, clean_pod_policy="All"))
    h.set_pods(j, "Master", active=1)
    h.set_pods(j, "Worker", active=1)
    h.set_services(j)
    h.sync(j)
    j = h.pc.job_informer.get_by_key("default/d")
    # move startTime into the past
    j["status"]["startTime"] = "2000-01-01T00:00:00Z"
    h.pc.job_informer.replace_in_cache(j)
    h.sync(j)
    last = h.last()
    assert last["status"]["conditions"][-1]["type"] == "Failed"
    assert "active longer than specified deadline" in last["status"]["conditions"][-1]["message"]
    assert sorted(h.pods.delete_pod_names) == ["d-master-0", "d-worker-0"]
    assert h.svcs.delete_service_names == ["d-master-0"]


@pytest.mark.parametrize("policy,deleted", [("All", ["c-master-0", "c-worker-0"]), ("Running", ["c-worker-0"]),
                                            ("None", [])])
def test_clean_pod_policy_after_success(policy, deleted):
    h = Harness()
    j = h.add_job(new_job("c", workers=1, clean_pod_policy=policy))
    h.set_pods(j, "Master", succeeded=1)
    h.set_pods(j, "Worker", active=1)
    h.set_services(j)
    h.sync(j)
    assert h.last()["status"]["conditions"][-1]["type"] == "Succeeded"
    j = h.pc.job_informer.get_by_key("default/c")
    h.sync(j)  # terminal pass: cleanup
    assert sorted(h.pods.delete_pod_names) == deleted
    fin = h.last()
    assert fin["status"]["replicaStatuses"]["Worker"]["active"] == 0
    assert fin["status"]["replicaStatuses"]["Worker"]["succeeded"] == 1


def test_ttl_deletes_job():
    h = Harness()
    j = h.add_job(new_job("t", workers=1, ttl_seconds_after_finished=0))
    h.set_pods(j, "Master", succeeded=1)
    h.set_pods(j, "Worker", succeeded=1)
    h.set_services(j)
    h.sync(j)
    j = h.pc.job_informer.get_by_key("default/t")
    time.sleep(1.1)
    h.sync(j)
    assert h.store.list("pytorchjobs")["items"] == []


def test_invalid_spec_marks_failed():
    h = Harness()
    bad = new_job("bad", workers=1)
    bad["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]["name"] = "other"
    obj = h.store.create("pytorchjobs", bad)
    h.pc.add_pytorch_job(obj)
    got = h.store.get("pytorchjobs", "default", "bad")
    c = got["status"]["conditions"][-1]
    assert c["type"] == "Failed" and c["reason"] == "InvalidPyTorchJobSpec"
    evs = h.store.list("events")["items"]
    assert any(e["reason"] == "InvalidPyTorchJobSpec" for e in evs)


def test_gang_scheduling_podgroup_and_annotations():
    h = Harness(enable_gang_scheduling=True)
    j = h.add_job(new_job("g", workers=3))
    h.sync(j)
    pg = h.store.get("podgroups", "default", "g")
    assert pg["spec"]["minMember"] == 4
    for t in h.pods.templates:
        assert t["spec"]["schedulerName"] == "volcano"
        assert t["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == "g"


def test_deleted_job_counts():
    h = Harness()
    assert h.pc.sync_pytorch_job("default/nothere") is True
    assert h.pc.metrics.jobs_deleted._value.get() == 1


# ---- condition invariants (hypothesis) -------------------------------------
cond_strategy = st.sampled_from([(C.JOB_RUNNING, C.REASON_RUNNING), (C.JOB_RESTARTING, C.REASON_RESTARTING),
                                 (C.JOB_SUCCEEDED, C.REASON_SUCCEEDED), (C.JOB_FAILED, C.REASON_FAILED),
                                 (C.JOB_CREATED, C.REASON_CREATED)])


@settings(max_examples=300, deadline=None)
@given(st.lists(cond_strategy, min_size=1, max_size=12))
def test_condition_invariants(seq):
    status = {}
    terminal_at = None
    for i, (t, r) in enumerate(seq):
        before = [dict(c) for c in status.get("conditions", [])]
        ctl.set_condition(status, ctl.new_condition(t, r, f"{t} msg"))
        conds = status.get("conditions", [])
        types = [c["type"] for c in conds]
        # Running and Restarting are mutually exclusive
        assert not (C.JOB_RUNNING in types and C.JOB_RESTARTING in types)
        # each type at most once
        assert len(types) == len(set(types))
        if terminal_at is not None:
            assert conds == before, "no transitions after a terminal condition"
        if terminal_at is None and t in (C.JOB_SUCCEEDED, C.JOB_FAILED):
            terminal_at = i
            run = [c for c in conds if c["type"] == C.JOB_RUNNING]
            assert all(c["status"] == "False" for c in run)
