"""The PyTorchJob controller: informers -> work queue -> reconcile.

Behavioural contract (every rule cites the reference Go it reproduces):

* handlers — ``pkg/controller.v1/pytorch/job.go:35-150`` (add: decode +
  validate, invalid spec => ``InvalidPyTorchJobSpec`` event + Failed status;
  else default + ``Created`` condition, written into the cached object,
  enqueue, ``jobs_created_total++``; update: enqueue and re-arm the
  ``activeDeadlineSeconds`` timer), vendored ``jobcontroller/pod.go:20-160``
  and ``service.go:17-66`` (pod/service events -> expectations + enqueue);
* worker loop — ``controller.go:185-274`` (Forget on success,
  AddRateLimited on error, deleted job => ``jobs_deleted_total++``);
* sync/reconcile — ``controller.go:290-492`` (expectations gate with the
  reference's OR across replica types, terminal cleanup per
  ``cleanPodPolicy``, TTL, PodGroup, backoff / deadline failure, per-type
  pod reconcile, master-only headless service, status write only on change);
* pods — ``pod.go:49-289`` (index slicing, ``<job>-<rtype>-<i>`` names,
  labels, env ``MASTER_PORT/MASTER_ADDR/WORLD_SIZE/RANK/PYTHONUNBUFFERED``,
  restart-policy mapping, worker init container, gang annotations,
  ``ExitCode`` restart with retryable codes);
* status machine — ``status.go:63-272``.

MI355X additions (opt-in, never altering the reference fields): pods get
the ``amd.com/gpu`` resource normalised from legacy ``nvidia.com/gpu``
limits so the node agent pins GPUs.
"""
from __future__ import annotations

import copy
import logging
import threading
import time
from dataclasses import dataclass

from ..api import constants as C
from ..api.defaults import set_defaults
from ..api.types import (
    gen_expectation_pods_key, gen_expectation_services_key, gen_general_name, gen_labels, gen_owner_reference,
    get_port_from_job, is_failed, is_retryable_exit_code, is_succeeded, key_of, name_of, namespace_of,
    now_rfc3339, parse_rfc3339, replica_specs, split_key, total_replicas)
from ..api.validation import ValidationError, validate_spec
from ..apiserver.store import ApiError
from . import control
from .expectations import ControllerExpectations
from .informer import Informer
from .metrics import OperatorMetrics
from .workqueue import RateLimitingQueue

log = logging.getLogger("pytorch-operator")

DEFAULT_INIT_CONTAINER_TEMPLATE = """
- name: init-pytorch
  image: {InitContainerImage}
  imagePullPolicy: IfNotPresent
  resources:
    limits:
      cpu: 100m
      memory: 20Mi
    requests:
      cpu: 50m
      memory: 10Mi
  command: ['sh', '-c', 'until nslookup {MasterAddr}; do echo waiting for master; sleep 2; done;']"""
INIT_CONTAINER_TEMPLATE_FILE = "/etc/config/initContainer.yaml"


def get_init_container_template() -> str:
    """``pkg/common/config/config.go:9-30``: file override, else default."""
    try:
        with open(INIT_CONTAINER_TEMPLATE_FILE) as f:
            return f.read()
    except OSError:
        return DEFAULT_INIT_CONTAINER_TEMPLATE


def get_init_containers(template: str, master_addr: str, image: str) -> list[dict]:
    import yaml

    text = template.replace("{{.MasterAddr}}", master_addr).replace("{{.InitContainerImage}}", image)
    text = text.replace("{MasterAddr}", master_addr).replace("{InitContainerImage}", image)
    return yaml.safe_load(text) or []


@dataclass
class ControllerConfig:
    enable_gang_scheduling: bool = False
    gang_scheduler_name: str = "volcano"
    init_container_image: str = "alpine:3.10"
    threadiness: int = 1
    namespace: str | None = None
    job_resync_period: float = C.JOB_RESYNC_PERIOD_S
    # ExitCode restarts of a multi-replica job: "job" deletes every replica
    # when one fails retryably (a DDP world restarts as a whole); "pod"
    # deletes only the failed pod, as the reference does (pod.go:91-109)
    restart_scope: str = "job"


class Recorder:
    """EventRecorder: writes core/v1 Events and logs them
    (jobcontroller.go:159-163)."""

    def __init__(self, client):
        self.client = client

    def event(self, obj, etype, reason, message):
        log.info("event %s %s %s: %s", etype, reason, key_of(obj), message)
        try:
            self.client.record_event(obj, etype, reason, message)
        except Exception as e:  # events are best-effort
            log.debug("event write failed: %s", e)


def _filter_for_rtype(objs, rt: str):
    return [o for o in objs if (o.get("metadata", {}).get("labels") or {}).get(C.LABEL_REPLICA_TYPE) == rt]


def _index_slices(objs, replicas: int, what: str):
    slices = [[] for _ in range(replicas)]
    for o in objs:
        labels = o.get("metadata", {}).get("labels") or {}
        if C.LABEL_REPLICA_INDEX not in labels:
            log.warning("The %s do not have the index label.", what)
            continue
        try:
            idx = int(labels[C.LABEL_REPLICA_INDEX])
        except ValueError:
            log.warning("Error when strconv.Atoi: %s", labels[C.LABEL_REPLICA_INDEX])
            continue
        if idx < 0 or idx >= replicas:
            log.warning("The label index is not expected: %d", idx)
        else:
            slices[idx].append(o)
    return slices


# ---------------------------------------------------------------- status ---
def new_condition(ctype, reason, message):
    t = now_rfc3339()
    return {"type": ctype, "status": "True", "lastUpdateTime": t, "lastTransitionTime": t, "reason": reason,
            "message": message}


def get_condition(status, ctype):
    for c in status.get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def filter_out_condition(conditions, ctype):
    out = []
    for c in conditions or []:
        if ctype == C.JOB_RESTARTING and c.get("type") == C.JOB_RUNNING:
            continue
        if ctype == C.JOB_RUNNING and c.get("type") == C.JOB_RESTARTING:
            continue
        if c.get("type") == ctype:
            continue
        if ctype in (C.JOB_FAILED, C.JOB_SUCCEEDED) and c.get("type") == C.JOB_RUNNING:
            c = dict(c)
            c["status"] = "False"
        out.append(c)
    return out


def set_condition(status, cond):
    """status.go:226-247: frozen after a terminal condition; no-op when the
    same type has the same status and reason; keep lastTransitionTime if the
    status did not change."""
    if is_failed(status) or is_succeeded(status):
        return
    cur = get_condition(status, cond["type"])
    if cur is not None and cur.get("status") == cond["status"] and cur.get("reason") == cond["reason"]:
        return
    if cur is not None and cur.get("status") == cond["status"]:
        cond["lastTransitionTime"] = cur.get("lastTransitionTime")
    status["conditions"] = filter_out_condition(status.get("conditions"), cond["type"]) + [cond]


def update_job_conditions(job, ctype, reason, message):
    set_condition(job.setdefault("status", {}), new_condition(ctype, reason, message))


# ------------------------------------------------------------ controller ---
class PyTorchController:
    def __init__(self, client, config: ControllerConfig | None = None, pod_control=None, service_control=None,
                 metrics: OperatorMetrics | None = None, start_informers: bool = True):
        self.client = client
        self.config = config or ControllerConfig()
        self.metrics = metrics or OperatorMetrics()
        self.recorder = Recorder(client)
        self.pod_control = pod_control or control.RealPodControl(client, self.recorder)
        self.service_control = service_control or control.RealServiceControl(client, self.recorder)
        self.expectations = ControllerExpectations()
        self.queue = RateLimitingQueue(C.PLURAL)
        ns = self.config.namespace
        self.job_informer = Informer(client, "pytorchjobs", ns, resync_period=self.config.job_resync_period)
        self.pod_informer = Informer(client, "pods", ns)
        self.service_informer = Informer(client, "services", ns)
        # injectable handlers (controller.go:81-88)
        self.sync_handler = self.sync_pytorch_job
        self.update_status_handler = self.update_pytorch_job_status
        self.delete_pytorch_job_handler = self.delete_pytorch_job
        self.job_informer.add_event_handler(self.add_pytorch_job, self.update_pytorch_job, self.enqueue_job)
        self.pod_informer.add_event_handler(self.add_pod, self.update_pod, self.delete_pod)
        self.service_informer.add_event_handler(self.add_service, self.update_service, self.delete_service)
        self._workers: list[threading.Thread] = []
        self._stop = threading.Event()
        self._start_informers = start_informers

    # ---------------------------------------------------------- plumbing
    def enqueue_job(self, obj):
        self.queue.add(key_of(obj))

    def run(self, threadiness: int | None = None, wait_sync_timeout: float = 30.0):
        """Start informers + workers (non-blocking).  controller.go:185-210."""
        if self._start_informers:
            for inf in (self.job_informer, self.pod_informer, self.service_informer):
                inf.start()
        for inf in (self.job_informer, self.pod_informer, self.service_informer):
            if not inf.wait_for_sync(wait_sync_timeout):
                raise RuntimeError("failed to wait for caches to sync")
        n = threadiness or self.config.threadiness
        for i in range(n):
            t = threading.Thread(target=self._run_worker, name=f"pytorchjob-worker-{i}", daemon=True)
            t.start()
            self._workers.append(t)
        return self

    def stop(self):
        self._stop.set()
        self.queue.shutdown()
        for inf in (self.job_informer, self.pod_informer, self.service_informer):
            inf.stop()

    def _run_worker(self):
        while not self._stop.is_set():
            if not self.process_next_work_item():
                return

    def process_next_work_item(self, timeout: float | None = None) -> bool:
        key, quit_ = self.queue.get(timeout)
        if quit_:
            return False
        if key is None:
            return True
        try:
            job = self.job_informer.get_by_key(key)
            if job is None:
                log.info("PyTorchJob has been deleted: %s", key)
                self.metrics.jobs_deleted.inc()
                return True
            try:
                forget = self.sync_handler(key)
            except Exception as e:
                log.warning("error syncing job %s: %s", key, e)
                self.queue.add_rate_limited(key)
                return True
            if forget:
                self.queue.forget(key)
            return True
        finally:
            self.queue.done(key)

    # ---------------------------------------------------------- job events
    def _job_from_obj(self, obj):
        job = copy.deepcopy(obj)
        validate_spec(job.get("spec"))
        return job

    def add_pytorch_job(self, obj):
        try:
            job = self._job_from_obj(obj)
        except (ValidationError, TypeError, AttributeError) as e:
            msg = f"Failed to unmarshal the object to PyTorchJob: Spec is invalid {e}"
            log.warning(msg)
            self.recorder.event(obj, "Warning", C.REASON_INVALID_SPEC, msg)
            status = {"conditions": [{"type": C.JOB_FAILED, "status": "True", "lastUpdateTime": now_rfc3339(),
                                      "lastTransitionTime": now_rfc3339(), "reason": C.REASON_INVALID_SPEC,
                                      "message": msg}]}
            bad = copy.deepcopy(obj)
            bad["status"] = status
            bad["metadata"].pop("resourceVersion", None)
            try:
                self.client.update_status("pytorchjobs", bad, namespace_of(obj))
            except ApiError as e2:
                log.error("Could not update the PyTorchJob: %s", e2)
            return
        set_defaults(job)
        msg = f"PyTorchJob {name_of(job)} is created."
        log.info(msg)
        update_job_conditions(job, C.JOB_CREATED, C.REASON_CREATED, msg)
        # like the reference, the Created condition lives in the cached
        # object and is persisted by the first status write (job.go:97-104)
        self.job_informer.replace_in_cache(job)
        self.enqueue_job(job)
        self.metrics.jobs_created.inc()

    def update_pytorch_job(self, old, cur):
        try:
            oldj, curj = self._job_from_obj(old), self._job_from_obj(cur)
        except (ValidationError, TypeError, AttributeError):
            return
        key = key_of(curj)
        self.queue.add(key)
        start = curj.get("status", {}).get("startTime")
        ads = curj.get("spec", {}).get("activeDeadlineSeconds")
        if start and ads is not None:
            old_ads = oldj.get("spec", {}).get("activeDeadlineSeconds")
            if old_ads is None or old_ads != ads:
                passed = time.time() - parse_rfc3339(start)
                self.queue.add_after(key, float(ads) - passed)

    # ---------------------------------------------------------- pod events
    def _resolve_controller_ref(self, namespace, ref):
        if not ref or ref.get("kind") != C.KIND:
            return None
        job = self.job_informer.get_by_key(f"{namespace}/{ref.get('name')}")
        if job is None or job.get("metadata", {}).get("uid") != ref.get("uid"):
            return None
        return job

    @staticmethod
    def _controller_ref(obj):
        for r in obj.get("metadata", {}).get("ownerReferences") or []:
            if r.get("controller"):
                return r
        return None

    def add_pod(self, pod):
        md = pod.get("metadata", {})
        if md.get("deletionTimestamp"):
            self.delete_pod(pod)
            return
        ref = self._controller_ref(pod)
        if ref is None:
            return  # orphan: adoption happens on the next job sync
        job = self._resolve_controller_ref(md.get("namespace"), ref)
        if job is None:
            return
        rtype = (md.get("labels") or {}).get(C.LABEL_REPLICA_TYPE)
        if rtype is None:
            log.info("This pod maybe not created by pytorch-operator")
            return
        self.expectations.creation_observed(gen_expectation_pods_key(key_of(job), rtype))
        self.enqueue_job(job)

    def update_pod(self, old, cur):
        if old.get("metadata", {}).get("resourceVersion") == cur.get("metadata", {}).get("resourceVersion"):
            return
        ns = cur.get("metadata", {}).get("namespace")
        cur_ref, old_ref = self._controller_ref(cur), self._controller_ref(old)
        if (cur_ref or {}).get("uid") != (old_ref or {}).get("uid") and old_ref is not None:
            j = self._resolve_controller_ref(ns, old_ref)
            if j is not None:
                self.enqueue_job(j)
        if cur_ref is not None:
            j = self._resolve_controller_ref(ns, cur_ref)
            if j is not None:
                self.enqueue_job(j)

    def delete_pod(self, pod):
        md = pod.get("metadata", {})
        ref = self._controller_ref(pod)
        if ref is None:
            return
        job = self._resolve_controller_ref(md.get("namespace"), ref)
        if job is None:
            return
        rtype = (md.get("labels") or {}).get(C.LABEL_REPLICA_TYPE)
        if rtype is None:
            return
        self.expectations.deletion_observed(gen_expectation_pods_key(key_of(job), rtype))
        self.enqueue_job(job)

    def add_service(self, svc):
        md = svc.get("metadata", {})
        if md.get("deletionTimestamp"):
            return
        ref = self._controller_ref(svc)
        if ref is None:
            return
        job = self._resolve_controller_ref(md.get("namespace"), ref)
        if job is None:
            return
        rtype = (md.get("labels") or {}).get(C.LABEL_REPLICA_TYPE)
        if rtype is None:
            return
        self.expectations.creation_observed(gen_expectation_services_key(key_of(job), rtype))
        self.enqueue_job(job)

    def update_service(self, old, cur):
        # no-op in the reference (vendored service.go:58-61)
        return

    def delete_service(self, svc):
        # The reference ignores service deletions (service.go:63-66), so a
        # deleted master Service only came back on the next job event.  We
        # requeue the owner so it is recreated promptly.
        ref = self._controller_ref(svc)
        if ref is None:
            return
        job = self._resolve_controller_ref(svc.get("metadata", {}).get("namespace"), ref)
        if job is not None:
            self.enqueue_job(job)

    # ---------------------------------------------------------- sync
    def satisfied_expectations(self, job) -> bool:
        """All pod/service expectation keys of the job must be satisfied.

        The reference ORs the keys (controller.go:505-513).  Because the
        Worker *services* key is never set, that OR is always true for any
        job with workers, so a second sync before the informer observes the
        creations creates duplicate pods.  AND is the
        intended semantics (unknown keys count as satisfied, expectations
        still expire after 5 minutes)."""
        key = key_of(job)
        for rtype in replica_specs(job):
            if not self.expectations.satisfied(gen_expectation_pods_key(key, rtype)):
                return False
            if not self.expectations.satisfied(gen_expectation_services_key(key, rtype)):
                return False
        return True

    def sync_pytorch_job(self, key: str) -> bool:
        t0 = time.perf_counter()
        try:
            ns, name = split_key(key)
            if not ns or not name:
                raise ValueError(f"invalid job key {key!r}: either namespace or name is missing")
            shared = self.job_informer.get_by_key(key)
            if shared is None:
                log.info("PyTorchJob has been deleted: %s", key)
                self.metrics.jobs_deleted.inc()
                return True
            try:
                job = self._job_from_obj(shared)
            except ValidationError as e:
                self.recorder.event(shared, "Warning", C.REASON_INVALID_SPEC,
                                    f"Failed to unmarshal the object to PyTorchJob object: {e}")
                return True
            needs_sync = self.satisfied_expectations(job)
            set_defaults(job)
            if needs_sync and not job["metadata"].get("deletionTimestamp"):
                self.reconcile_pytorch_jobs(job)
            return True
        finally:
            dt = time.perf_counter() - t0
            self.metrics.sync_seconds.observe(dt)
            log.debug("Finished syncing job %r (%.3fms)", key, dt * 1e3)

    def get_pods_for_job(self, job):
        ns = namespace_of(job)
        pods = self.pod_informer.list(ns)
        return control.claim_objects(pods, job, gen_labels(name_of(job)), self.client, "pods",
                                     bool(job["metadata"].get("deletionTimestamp")))

    def get_services_for_job(self, job):
        ns = namespace_of(job)
        svcs = self.service_informer.list(ns)
        return control.claim_objects(svcs, job, gen_labels(name_of(job)), self.client, "services",
                                     bool(job["metadata"].get("deletionTimestamp")))

    def reconcile_pytorch_jobs(self, job):
        key = key_of(job)
        old_status = copy.deepcopy(job.get("status", {}))
        pods = self.get_pods_for_job(job)
        services = self.get_services_for_job(job)
        status = job.setdefault("status", {})

        if is_succeeded(status) or is_failed(status):
            self.delete_pods_and_services(job, pods, services)
            self.cleanup_pytorch_job(job)
            if self.config.enable_gang_scheduling:
                control.delete_pod_group(self.client, self.recorder, job)
            if is_succeeded(status):
                for rs in (status.get("replicaStatuses") or {}).values():
                    rs["succeeded"] = int(rs.get("succeeded", 0)) + int(rs.get("active", 0))
                    rs["active"] = 0
            if status != old_status:
                self.update_status_handler(job)
            return

        previous_retry = self.queue.num_requeues(key)
        active = sum(1 for p in pods if p.get("status", {}).get("phase") not in ("Succeeded", "Failed")
                     and not p["metadata"].get("deletionTimestamp"))
        failed = sum(1 for p in pods if p.get("status", {}).get("phase") == "Failed")
        total = total_replicas(job)
        prev_failed = sum(int(rs.get("failed", 0)) for rs in (status.get("replicaStatuses") or {}).values())

        failure_message = ""
        exceeds_limit = False
        backoff = job["spec"].get("backoffLimit")
        exceeds_backoff = past_backoff = False
        if backoff is not None:
            new_failure = failed > prev_failed
            exceeds_backoff = new_failure and active != total and previous_retry + 1 > int(backoff)
            past_backoff = self.past_backoff_limit(job, pods)
        if exceeds_backoff or past_backoff:
            exceeds_limit = True
            failure_message = f"PyTorchJob {name_of(job)} has failed because it has reached the specified backoff limit"
        elif self.past_active_deadline(job):
            exceeds_limit = True
            failure_message = (f"PyTorchJob {name_of(job)} has failed because it was active longer than specified "
                               f"deadline")

        if exceeds_limit:
            self.delete_pods_and_services(job, pods, services)
            if status.get("completionTime") is None:
                status["completionTime"] = now_rfc3339()
            self.cleanup_pytorch_job(job)
            if self.config.enable_gang_scheduling:
                control.delete_pod_group(self.client, self.recorder, job)
            self.recorder.event(job, "Normal", C.REASON_FAILED, failure_message)
            update_job_conditions(job, C.JOB_FAILED, C.REASON_FAILED, failure_message)
            self.metrics.jobs_failed.inc()
        else:
            if self.config.enable_gang_scheduling:
                try:
                    control.sync_pod_group(self.client, job, total)
                except ApiError as e:
                    log.warning("Sync PodGroup %s: %s", name_of(job), e)
            self.restart_wave(job, pods, total)
            for rtype, spec in replica_specs(job).items():
                self.reconcile_pods(job, pods, rtype, spec)
                if rtype != C.REPLICA_MASTER:
                    continue
                self.reconcile_services(job, services, rtype, spec)

        if job.get("status") != old_status:
            self.update_status_handler(job)

    def past_backoff_limit(self, job, pods) -> bool:
        limit = job["spec"].get("backoffLimit")
        if limit is None:
            return False
        result = 0
        for rtype, spec in replica_specs(job).items():
            if spec.get("restartPolicy") not in (C.RESTART_POLICY_ON_FAILURE, C.RESTART_POLICY_ALWAYS):
                continue
            for p in _filter_for_rtype(pods, rtype.lower()):
                st = p.get("status", {})
                if st.get("phase") in ("Running", "Pending"):
                    for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
                        result += int(cs.get("restartCount", 0))
        if int(limit) == 0:
            return result > 0
        return result >= int(limit)

    def past_active_deadline(self, job) -> bool:
        ads = job["spec"].get("activeDeadlineSeconds")
        start = job.get("status", {}).get("startTime")
        if ads is None or not start:
            return False
        return time.time() - parse_rfc3339(start) >= float(ads)

    # ---------------------------------------------------------- pods
    @staticmethod
    def _exit_code(pod) -> int | None:
        """Terminated exit code of the ``pytorch`` container (pod.go:91-101)."""
        for cs in pod.get("status", {}).get("containerStatuses") or []:
            term = (cs.get("state") or {}).get("terminated")
            if cs.get("name") == C.DEFAULT_CONTAINER_NAME and term:
                return int(term.get("exitCode", 0))
        return None

    def restart_wave(self, job, pods, total: int):
        """Job-level restart (``restart_scope="job"``).

        The reference deletes only the failed pod of an ``ExitCode`` replica
        (pod.go:91-109).  For a DDP world that is not enough: the surviving
        ranks keep the rendezvous store and communicators of the old world,
        sit in a collective with a dead peer until a timeout, and the
        recreated rank joins their store instead of a new one.  So when any
        replica failed with a retryable code, every other replica of the
        job is deleted in the same pass; the next reconcile recreates all of
        them, and the node manager starts the new pods only after every
        process of the old ones has exited (node/kubelet.py, restart gate).
        The failed pod itself goes through :meth:`reconcile_pods` as usual,
        which keeps the reference's ``ExitedWithCode`` events and the
        ``Restarting`` condition."""
        if self.config.restart_scope != "job" or total <= 1:
            return
        specs = replica_specs(job)
        failed = []
        for p in pods:
            if p.get("status", {}).get("phase") != "Failed":
                continue
            rt = (p["metadata"].get("labels") or {}).get(C.LABEL_REPLICA_TYPE, "")
            spec = next((s for t, s in specs.items() if t.lower() == rt), None)
            code = self._exit_code(p)
            if (spec is None or spec.get("restartPolicy") != C.RESTART_POLICY_EXIT_CODE or code is None
                    or not is_retryable_exit_code(code)):
                return  # a permanent failure: the job fails (reconcile_pods), nothing is restarted
            failed.append(name_of(p))
        if not failed:
            return
        others = [p for p in pods if name_of(p) not in failed and not p["metadata"].get("deletionTimestamp")]
        if not others:
            return
        msg = (f"PyTorchJob {name_of(job)}: {', '.join(sorted(failed))} failed with a retryable exit code; "
               f"restarting all {total} replicas")
        log.info(msg)
        self.recorder.event(job, "Normal", C.REASON_RESTARTING, msg)
        for p in others:
            self.pod_control.delete_pod(namespace_of(p), name_of(p), job)

    def reconcile_pods(self, job, pods, rtype, spec):
        rt = rtype.lower()
        pods = _filter_for_rtype(pods, rt)
        replicas = int(spec.get("replicas", 1))
        restart = False
        status = job.setdefault("status", {})
        status.setdefault("replicaStatuses", {})[rtype] = {"active": 0, "succeeded": 0, "failed": 0}
        for index, pslice in enumerate(_index_slices(pods, replicas, "pod")):
            if len(pslice) > 1:
                log.warning("We have too many pods for %s %d", rt, index)
            elif len(pslice) == 0:
                log.info("Need to create new pod: %s-%d", rt, index)
                self.create_new_pod(job, rtype, str(index), spec, rtype == C.REPLICA_MASTER)
            else:
                pod = pslice[0]
                if spec.get("restartPolicy") == C.RESTART_POLICY_EXIT_CODE:
                    exit_code = 0
                    for cs in pod.get("status", {}).get("containerStatuses") or []:
                        term = (cs.get("state") or {}).get("terminated")
                        if cs.get("name") == C.DEFAULT_CONTAINER_NAME and term:
                            exit_code = int(term.get("exitCode", 0))
                            msg = f"Pod: {namespace_of(pod)}.{name_of(pod)} exited with code {exit_code}"
                            log.info(msg)
                            self.recorder.event(job, "Normal", C.REASON_EXITED_WITH_CODE, msg)
                    if pod.get("status", {}).get("phase") == "Failed" and is_retryable_exit_code(exit_code):
                        log.info("Need to restart the pod: %s.%s", namespace_of(pod), name_of(pod))
                        self.pod_control.delete_pod(namespace_of(pod), name_of(pod), job)
                        restart = True
                phase = pod.get("status", {}).get("phase")
                rs = status["replicaStatuses"][rtype]
                if phase == "Running":
                    rs["active"] += 1
                elif phase == "Succeeded":
                    rs["succeeded"] += 1
                elif phase == "Failed":
                    rs["failed"] += 1
        self.update_status_single(job, rtype, replicas, restart)

    def create_new_pod(self, job, rtype, index: str, spec, master_role: bool):
        rt = rtype.lower()
        key = key_of(job)
        self.expectations.expect_creations(gen_expectation_pods_key(key, rt), 1)
        controller_ref = gen_owner_reference(job)
        labels = gen_labels(name_of(job))
        labels[C.LABEL_REPLICA_TYPE] = rt
        labels[C.LABEL_REPLICA_INDEX] = index
        if master_role:
            labels[C.LABEL_JOB_ROLE] = "master"
        tmpl = copy.deepcopy(spec.get("template") or {})
        tmpl.setdefault("metadata", {})
        tmpl["metadata"]["name"] = gen_general_name(name_of(job), rt, index)
        tmpl["metadata"].setdefault("labels", {})
        tmpl["metadata"]["labels"] = dict(tmpl["metadata"]["labels"] or {}, **labels)
        tmpl.setdefault("spec", {})
        self.set_cluster_spec(tmpl, job, total_replicas(job), index, rtype)
        if tmpl["spec"].get("restartPolicy"):
            msg = "Restart policy in pod template will be overwritten by restart policy in replica spec"
            log.warning(msg)
            self.recorder.event(job, "Warning", C.REASON_POD_TEMPLATE_RESTART_POLICY, msg)
        rp = spec.get("restartPolicy")
        tmpl["spec"]["restartPolicy"] = "Never" if rp == C.RESTART_POLICY_EXIT_CODE else rp
        if not master_role:
            master_addr = gen_general_name(name_of(job), C.REPLICA_MASTER.lower(), "0")
            tmpl["spec"].setdefault("initContainers", [])
            tmpl["spec"]["initContainers"] = list(tmpl["spec"]["initContainers"] or []) + get_init_containers(
                get_init_container_template(), master_addr, self.config.init_container_image)
        if self.config.enable_gang_scheduling:
            if self._non_gang_scheduler_set(job):
                msg = "Another scheduler is specified when gang-scheduling is enabled and it will not be overwritten"
                log.warning(msg)
                self.recorder.event(job, "Warning", C.REASON_POD_TEMPLATE_SCHEDULER_NAME, msg)
            else:
                tmpl["spec"]["schedulerName"] = self.config.gang_scheduler_name
            tmpl["metadata"].setdefault("annotations", {})
            tmpl["metadata"]["annotations"] = dict(tmpl["metadata"]["annotations"] or {})
            tmpl["metadata"]["annotations"][C.ANNOTATION_GANG_GROUP] = name_of(job)
        _normalise_gpu_resources(tmpl["spec"])
        try:
            self.pod_control.create_pods_with_controller_ref(namespace_of(job), tmpl, job, controller_ref)
        except ApiError as e:
            if e.code == 504:  # timeout: treated as success (pod.go:219-227)
                return
            raise

    def _non_gang_scheduler_set(self, job):
        for spec in replica_specs(job).values():
            sn = (spec.get("template") or {}).get("spec", {}).get("schedulerName")
            if sn and sn != self.config.gang_scheduler_name:
                return True
        return False

    @staticmethod
    def set_cluster_spec(tmpl, job, total: int, index: str, rtype: str):
        rank = int(index)
        master_port = get_port_from_job(job, C.REPLICA_MASTER)
        master_addr = gen_general_name(name_of(job), C.REPLICA_MASTER.lower(), "0")
        if rtype == C.REPLICA_MASTER:
            if rank != 0:
                raise ValueError("invalid config: There should be only a single master with index=0")
            master_addr = "localhost"
        else:
            rank += 1
        for c in tmpl["spec"].get("containers") or []:
            env = list(c.get("env") or [])
            env += [{"name": "MASTER_PORT", "value": str(master_port)},
                    {"name": "MASTER_ADDR", "value": master_addr},
                    {"name": "WORLD_SIZE", "value": str(total)},
                    {"name": "RANK", "value": str(rank)},
                    {"name": "PYTHONUNBUFFERED", "value": "0"}]
            c["env"] = env

    # ---------------------------------------------------------- services
    def reconcile_services(self, job, services, rtype, spec):
        rt = rtype.lower()
        replicas = int(spec.get("replicas", 1))
        services = _filter_for_rtype(services, rt)
        for index, sslice in enumerate(_index_slices(services, replicas, "service")):
            if len(sslice) > 1:
                log.warning("We have too many services for %s %d", rt, index)
            elif len(sslice) == 0:
                log.info("need to create new service: %s-%d", rt, index)
                self.create_new_service(job, rtype, str(index), spec)

    def create_new_service(self, job, rtype, index: str, spec):
        rt = rtype.lower()
        self.expectations.expect_creations(gen_expectation_services_key(key_of(job), rt), 1)
        labels = gen_labels(name_of(job))
        labels[C.LABEL_REPLICA_TYPE] = rt
        labels[C.LABEL_REPLICA_INDEX] = index
        port = get_port_from_job(job, rtype)
        svc = {"metadata": {"name": gen_general_name(name_of(job), rt, index), "labels": labels},
               "spec": {"clusterIP": "None", "selector": dict(labels),
                        "ports": [{"name": C.DEFAULT_PORT_NAME, "port": port}]}}
        try:
            self.service_control.create_services_with_controller_ref(namespace_of(job), svc, job,
                                                                     gen_owner_reference(job))
        except ApiError as e:
            if e.code == 504:
                return
            raise

    # ---------------------------------------------------------- status
    def update_status_single(self, job, rtype, replicas: int, restart: bool):
        status = job.setdefault("status", {})
        rs = status["replicaStatuses"][rtype]
        expected = replicas - int(rs["succeeded"])
        running, failed = int(rs["active"]), int(rs["failed"])
        log.info("PyTorchJob=%s, ReplicaType=%s expected=%d, running=%d, failed=%d", name_of(job), rtype, expected,
                 running, failed)
        if not status.get("startTime"):
            status["startTime"] = now_rfc3339()
            ads = job["spec"].get("activeDeadlineSeconds")
            if ads is not None:
                log.info("Job with ActiveDeadlineSeconds will sync after %s seconds", ads)
                self.queue.add_after(key_of(job), float(ads))
        if C.REPLICA_MASTER not in replica_specs(job):
            raise ValueError("invalid config: Job must contain master replica spec")
        if rtype == C.REPLICA_MASTER:
            if running > 0:
                update_job_conditions(job, C.JOB_RUNNING, C.REASON_RUNNING, f"PyTorchJob {name_of(job)} is running.")
            if expected == 0:
                msg = f"PyTorchJob {name_of(job)} is successfully completed."
                self.recorder.event(job, "Normal", C.REASON_SUCCEEDED, msg)
                if status.get("completionTime") is None:
                    status["completionTime"] = now_rfc3339()
                update_job_conditions(job, C.JOB_SUCCEEDED, C.REASON_SUCCEEDED, msg)
                self.metrics.jobs_successful.inc()
        if failed > 0:
            if restart:
                msg = f"PyTorchJob {name_of(job)} is restarting because {failed} {rtype} replica(s) failed."
                self.recorder.event(job, "Warning", C.REASON_RESTARTING, msg)
                update_job_conditions(job, C.JOB_RESTARTING, C.REASON_RESTARTING, msg)
                self.metrics.jobs_failed.inc()
                self.metrics.jobs_restarted.inc()
            else:
                msg = f"PyTorchJob {name_of(job)} is failed because {failed} {rtype} replica(s) failed."
                self.recorder.event(job, "Normal", C.REASON_FAILED, msg)
                if status.get("completionTime") is None:
                    status["completionTime"] = now_rfc3339()
                update_job_conditions(job, C.JOB_FAILED, C.REASON_FAILED, msg)
                self.metrics.jobs_failed.inc()

    def update_pytorch_job_status(self, job):
        cached = self.job_informer.get_by_key(key_of(job))
        obj = copy.deepcopy(job)
        # write against the latest cached resourceVersion (status subresource
        # writes never clobber spec; conflicts requeue via the error path)
        if cached is not None:
            obj["metadata"]["resourceVersion"] = cached["metadata"].get("resourceVersion")
        out = self.client.update_status("pytorchjobs", obj, namespace_of(job))
        self.job_informer.replace_in_cache(out)
        return out

    # ---------------------------------------------------------- cleanup
    def delete_pods_and_services(self, job, pods, services):
        if not pods:
            return
        policy = job["spec"].get("cleanPodPolicy")
        if policy == C.CLEAN_POD_POLICY_NONE:
            return
        for p in pods:
            if policy == C.CLEAN_POD_POLICY_RUNNING and p.get("status", {}).get("phase") != "Running":
                continue
            self.pod_control.delete_pod(namespace_of(p), name_of(p), job)
        for s in _filter_for_rtype(services, C.REPLICA_MASTER.lower()):
            self.service_control.delete_service(namespace_of(s), name_of(s), job)

    def cleanup_pytorch_job(self, job):
        ttl = job["spec"].get("ttlSecondsAfterFinished")
        if ttl is None:
            return
        done = job.get("status", {}).get("completionTime")
        if not done:  # the reference dereferences nil here
            return
        if time.time() > parse_rfc3339(done) + float(ttl):
            self.delete_pytorch_job_handler(job)
            return
        self.queue.add_rate_limited(key_of(job))

    def delete_pytorch_job(self, job):
        self.client.delete("pytorchjobs", namespace_of(job), name_of(job))


def _normalise_gpu_resources(pod_spec):
    """Map legacy ``nvidia.com/gpu`` limits (reference example YAMLs) onto
    ``amd.com/gpu`` so the MI355X node agent allocates them."""
    for c in pod_spec.get("containers") or []:
        res = c.get("resources") or {}
        for sec in ("limits", "requests"):
            d = res.get(sec) or {}
            for legacy in C.LEGACY_GPU_RESOURCES:
                if legacy in d and C.GPU_RESOURCE not in d:
                    d[C.GPU_RESOURCE] = d.pop(legacy)
