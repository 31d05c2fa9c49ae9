"""Node manager: turns Pod objects into supervised processes on the
MI355X node (the kubelet + device plugin + cluster DNS of the reference's
substrate), using the native agent for process control.

Per pod:
  1. admission — ``amd.com/gpu`` allocation by the agent's exclusive
     allocator; with gang scheduling (``scheduling.k8s.io/group-name``
     annotation + PodGroup ``minMember``) all members are admitted at once
     or none (kube-batch semantics, C30); unschedulable pods stay Pending
     with ``PodScheduled=False/Unschedulable``.
  2. init containers — the reference's ``init-pytorch`` DNS wait
     (``until nslookup <job>-master-0``) runs natively: wait until the
     master Service exists (and, on request, its port accepts
     connections); other init containers run as processes.
  3. containers — spawned through the agent with kubelet restart semantics;
     env = container env + GPU pinning (below); Service names in
     ``MASTER_ADDR`` resolve to the node address (single-node "DNS"), and
     ``MASTER_PORT`` is virtualised per job so concurrent jobs can all ask
     for 23456 (pods share the host network).  The values the process
     really gets are recorded in the ``pto.amd.com/effective-env`` pod
     annotation (shown by ``pto describe``): the pod spec keeps the
     reference's contract (``MASTER_ADDR=<job>-master-0``,
     ``MASTER_PORT=23456``, pod.go:245-274), the process sees
     ``127.0.0.1`` and the job's port.

GPU pinning (``gpu_visibility``, per pod: the ``pto.amd.com/gpu-visibility``
annotation):
  * ``job`` (default) — the process's own GPU is device 0 (``LOCAL_RANK=0``,
    so an image that just uses ``cuda:0`` lands on it, as under a device
    plugin), followed by the GPUs allocated to the OTHER replicas of the
    same job on this node (known at start: all of them with gang
    admission).  No other job's GPU is visible, but the job's own peers stay
    enumerable, so RCCL can pick its P2P/IPC transport over xGMI instead of
    staging through host memory, and the xGMI all-reduce can map the
    peers' buffers.
  * ``isolated`` — the process sees only its own GPUs
    (``HIP_VISIBLE_DEVICES`` = its allocation, ``LOCAL_RANK=0``), the
    Kubernetes device-plugin model: any image that just uses ``cuda:0``
    lands on its own GPU.
  * ``node`` — every replica sees ALL of the node's GPUs
    (``HIP_VISIBLE_DEVICES`` = the node's list, identical in every
    replica) and selects its own through ``LOCAL_RANK`` = the index of its
    allocated GPU.  This is what torchrun does, and it keeps the peers'
    devices enumerable by HIP: ``hipIpcOpenMemHandle`` of a peer buffer
    (the xGMI all-reduce) and RCCL's P2P transport both work on devices
    the process can see.  The allocator still hands each GPU to exactly
    one replica.  Jobs that all-reduce over peer memory (the fused trainer's
    xGMI transport) ask for it with the annotation; with ``isolated`` the
    xGMI autotune falls back to RCCL if the peer mapping fails on any rank.
  4. status — phase, containerStatuses (state, restartCount, exitCode),
     podIP/hostIP, written back through the status subresource.
  5. deletion — SIGTERM the process group, SIGKILL after the grace period,
     free the GPUs.

Restarts of a multi-replica job (a DDP world cannot take back one
restarted rank; docs/multi_gpu.md "Restarts"):
  * in place (``OnFailure``/``Always``): the job's containers form one
    restart group in the agent -- a failing member takes the others down,
    and all restart together once the last has exited;
  * recreated pods (``ExitCode``: the controller deletes every replica of
    the job, controller/pytorch.py ``restart_scope``): a new pod of the job
    is held Pending (``PreviousIncarnationRunning``) until every process of
    the job's torn-down pods has exited, so its master binds a closed port
    and no replica can reach the old incarnation's rendezvous store;
  * every wave gets ``PTO_RESTART_GENERATION`` (``<pod generation>.<in-place
    wave>``), which the trainers put in front of their rendezvous keys.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import re
import shlex
import socket
import sys
import threading
import time

from ..api import constants as C
from ..api.types import key_of, name_of, namespace_of, now_rfc3339, parse_rfc3339
from ..api.validation import gpus_requested
from ..apiserver.server import LOG_ANNOTATION
from ..apiserver.store import ApiError
from ..controller.informer import Informer
from .native import AgentClient

log = logging.getLogger("pto-kubelet")

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# "container images" -> entrypoints in the node's Python environment.  The
# reference images are mapped onto this package's runtimes.
DEFAULT_IMAGES = {
    "pto/pytorch-mnist:rocm": [sys.executable, "-m", "pytorch_operator_1_amd.train.mnist"],
    "gcr.io/kubeflow-ci/pytorch-dist-mnist-test:v1.0": [sys.executable, "-m", "pytorch_operator_1_amd.train.mnist"],
    "pto/pytorch-sendrecv:rocm": [sys.executable, "-m", "pytorch_operator_1_amd.train.sendrecv"],
    "gcr.io/kubeflow-ci/pytorch-dist-sendrecv-test:1.0": [sys.executable, "-m",
                                                          "pytorch_operator_1_amd.train.sendrecv"],
    "pto/pytorch-lm:rocm": [sys.executable, "-m", "pytorch_operator_1_amd.train.lm"],
    "pto/bench:rocm": [sys.executable, os.path.join(REPO_ROOT, "bench.py")],
    "pto/python:rocm": [sys.executable],
}
FIRST_STEP_ANNOTATION = "pto.amd.com/first-step-unix"
STARTUP_ANNOTATION = "pto.amd.com/startup-phases"  # the trainer's own startup breakdown (JSON)
THROUGHPUT_ANNOTATION = "pto.amd.com/samples-per-sec"
GPUS_ANNOTATION = "pto.amd.com/gpus"
EFFECTIVE_ENV_ANNOTATION = "pto.amd.com/effective-env"
# env keys whose effective value is recorded on the pod
_EFFECTIVE_KEYS = ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                   "HIP_VISIBLE_DEVICES", "PTO_MASTER_SERVICE", "PTO_MASTER_PORT_REQUESTED")
GPU_VISIBILITY_MODES = ("job", "node", "isolated")
# per-pod choice of the visibility model (pod template annotation); the
# node-wide default is --gpu-visibility / PTO_GPU_VISIBILITY
GPU_VISIBILITY_ANNOTATION = "pto.amd.com/gpu-visibility"
NODE_ADDRESS = "127.0.0.1"


def _port_free(port: int) -> bool:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind(("0.0.0.0", port))
        return True
    except OSError:
        return False
    finally:
        s.close()


_PORT_LOCK_DIR = os.path.join("/tmp", "pto-port-locks")


def _reserve_port(port: int):
    """Host-wide reservation of a virtual master port: an flock held by this
    process for its lifetime, so two kubelets on one host (e.g. concurrent
    test clusters) never hand the same port to two jobs before either
    master has bound it.  Returns the lock fd, or None if taken."""
    import fcntl

    os.makedirs(_PORT_LOCK_DIR, exist_ok=True)
    fd = os.open(os.path.join(_PORT_LOCK_DIR, f"{port}.lock"), os.O_CREAT | os.O_RDWR, 0o666)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        return fd
    except OSError:
        os.close(fd)
        return None


class PodRuntime:
    def __init__(self, pod):
        self.key = key_of(pod)
        self.uid = pod["metadata"].get("uid")
        # agent process ids and the GPU owner are per pod INCARNATION: a pod
        # recreated under the same name must never be confused with the
        # previous one, whose teardown may still be reaping its processes
        self.owner = _owner(pod)
        self.job_key = Kubelet._job_key(pod)
        self.stage = "admit"  # admit -> init -> run -> done
        self.gpus: list[int] = []
        self.init_index = 0
        self.started_at = None
        self.proc_ids: list[str] = []
        self.deleted = False
        self.last_status = None
        self.metrics_pos = 0
        self.annotated_first_step = False


def _pod_hbm(pod) -> float:
    """Per-GPU HBM bytes a pod asks for (max over its containers)."""
    from ..api.validation import hbm_requested

    return max([hbm_requested(c) for c in pod.get("spec", {}).get("containers", [])] or [0.0])


class Kubelet:
    def __init__(self, client, agent: AgentClient | None = None, node_name: str = "mi355x-0",
                 log_dir: str | None = None, images: dict | None = None, gpus: int | None = None,
                 poll_interval: float = 0.05, grace_seconds: float = 5.0, extra_env: dict | None = None,
                 hbm_per_gpu: float = C.HBM_PER_GPU_BYTES, gpu_visibility: str | None = None, metrics=None,
                 sysfs_root: str | None = None, gpu_share: int | None = None, group_restarts: bool = True):
        self.client = client
        self.gpu_visibility = gpu_visibility or os.environ.get("PTO_GPU_VISIBILITY", "job")
        if self.gpu_visibility not in GPU_VISIBILITY_MODES:
            raise ValueError(f"gpu_visibility must be one of {GPU_VISIBILITY_MODES}")
        # in-place restarts (OnFailure/Always) of a multi-replica job's
        # containers as one group (False: each container alone, as a kubelet)
        self.group_restarts = group_restarts
        # OperatorMetrics to feed with the trainers' reports and node HBM
        self.metrics = metrics
        self.sysfs_root = sysfs_root or os.environ.get("PTO_SYSFS_ROOT", "/sys")
        self._hbm_next = 0.0
        if gpus is None and agent is None:
            gpus = _visible_gpu_count()
        # TEST-ONLY rehearsal of multi-GPU jobs on a one-GPU box: every
        # physical GPU is offered as `gpu_share` allocatable slots, so N
        # replicas can be admitted onto the same device (they must then use
        # gloo + same-device xGMI IPC; RCCL refuses duplicate devices).
        self.gpu_share = max(1, int(gpu_share or os.environ.get("PTO_GPU_SHARE", "1")))
        if gpus is not None and agent is None:
            gpus *= self.gpu_share
        # warm starts (node/zygote.py) unless PTO_ZYGOTE=0
        self.agent = agent or AgentClient(gpus=gpus, hbm_per_gpu=hbm_per_gpu,
                                          zygote=os.environ.get("PTO_ZYGOTE", "1") == "1")
        self.node_name = node_name
        self.log_dir = log_dir or os.path.join(os.environ.get("TMPDIR", "/tmp"), "pto-pods")
        os.makedirs(self.log_dir, exist_ok=True)
        self.images = dict(DEFAULT_IMAGES, **(images or {}))
        self.poll = poll_interval
        self.grace = grace_seconds
        self.extra_env = extra_env or {}
        self.pods: dict[str, PodRuntime] = {}
        # restart generations (module doc, "Restarts"): agent ids of the
        # processes of torn-down pods, per job, until they have all exited;
        # jobs whose previous incarnation has just drained; generation per job
        self.retired: dict[str, set[str]] = {}
        self._drained: set[str] = set()
        self.job_gen: dict[str, int] = {}
        self.job_ports: dict[str, int] = {}
        self._gang_gpus: dict[str, dict] = {}  # job -> {owner: allocator slots} of its last gang admission
        self._port_locks: dict[int, int] = {}  # port -> flock fd of its host-wide reservation
        self.pod_informer = Informer(client, "pods")
        self.svc_informer = Informer(client, "services")
        self.pod_informer.add_event_handler(on_delete=self._on_pod_delete)
        self._stop = threading.Event()
        self._thread = None
        self._lock = threading.RLock()

    # ------------------------------------------------------------ lifecycle
    def start(self):
        self.pod_informer.start()
        self.svc_informer.start()
        self.pod_informer.wait_for_sync(10)
        self.svc_informer.wait_for_sync(10)
        self._register_node()
        self._thread = threading.Thread(target=self._loop, name="pto-kubelet", daemon=True)
        self._thread.start()
        return self

    def stop(self, kill_pods: bool = True):
        self._stop.set()
        if self._thread:
            self._thread.join(5)
        if kill_pods:
            for rt in list(self.pods.values()):
                for pid in rt.proc_ids:
                    self.agent.kill(pid, signal=9)
        self.pod_informer.stop()
        self.svc_informer.stop()
        self.agent.close()

    def _register_node(self):
        n = self.agent.gpus()["count"]
        node = {"metadata": {"name": self.node_name, "labels": {"kubernetes.io/hostname": self.node_name,
                                                                 "amd.com/gpu.product": "MI355X"}},
                "status": {"capacity": {C.GPU_RESOURCE: n, "cpu": os.cpu_count()},
                           "allocatable": {C.GPU_RESOURCE: n, "cpu": os.cpu_count()},
                           "addresses": [{"type": "InternalIP", "address": NODE_ADDRESS}]}}
        try:
            self.client.create("nodes", node)
        except ApiError:
            pass

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.sync_once()
            except Exception:
                log.exception("kubelet sync failed")
            if time.time() >= self._hbm_next:
                self._hbm_next = time.time() + 5.0
                try:
                    self.update_node_metrics()
                except Exception:
                    log.debug("HBM metrics read failed", exc_info=True)
            self._stop.wait(self.poll)

    # ------------------------------------------------------------ sync
    def sync_once(self):
        pods = self.pod_informer.list()
        procs = self.agent.status()
        with self._lock:
            for pod in pods:
                k = key_of(pod)
                rt = self.pods.get(k)
                if rt is None or rt.uid != pod["metadata"].get("uid"):
                    if rt is not None:  # same name, new incarnation
                        self._teardown(rt)
                    if (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                        continue  # finished before we knew it (e.g. kubelet restart)
                    rt = self.pods[k] = PodRuntime(pod)
                self._advance(pod, rt, procs)
            live = {key_of(p) for p in pods}
            for k in [k for k in self.pods if k not in live]:
                self._teardown(self.pods.pop(k))
            for jk in [jk for jk, ids in self.retired.items()
                       if all((procs.get(i) or {}).get("state") != "running" for i in ids)]:
                del self.retired[jk]
                self._drained.add(jk)
            self._release_job_ports(pods)

    def _on_pod_delete(self, pod):
        with self._lock:
            rt = self.pods.pop(key_of(pod), None)
            if rt is not None:
                self._teardown(rt)

    def _teardown(self, rt: PodRuntime):
        if rt.proc_ids and not rt.deleted:
            self.retired.setdefault(rt.job_key, set()).update(rt.proc_ids)
        for pid in rt.proc_ids:
            try:
                self.agent.kill(pid, signal=15, grace=self.grace)
            except Exception:
                pass
        threading.Thread(target=self._reap_later, args=(list(rt.proc_ids), rt.owner), daemon=True).start()
        rt.deleted = True

    def _reap_later(self, ids, owner):
        try:
            end = time.time() + self.grace + 5
            while time.time() < end and not self._stop.is_set():
                st = self.agent.status()
                if all(st.get(i, {}).get("state") != "running" for i in ids):
                    break
                time.sleep(0.1)
            for i in ids:
                self.agent.remove(i)
            self.agent.free(owner)
        except Exception:  # agent already shut down (node stopping)
            pass

    # ------------------------------------------------------------ stages
    def _advance(self, pod, rt: PodRuntime, procs):
        if rt.stage == "done":
            return
        if rt.stage == "admit":
            if not self._previous_incarnation_gone(pod, rt, procs) or not self._admit(pod, rt):
                return
            rt.stage = "init"
            rt.started_at = now_rfc3339()
            self._clear_pod_files(pod)
            self._annotate(pod, {LOG_ANNOTATION: self._log_path(pod), GPUS_ANNOTATION:
                                 ",".join(map(str, rt.gpus))})
        if rt.stage == "init":
            if not self._run_init(pod, rt, procs):
                return
            self._start_containers(pod, rt)
            rt.stage = "run"
            procs = self.agent.status()
        if rt.stage == "run":
            self._report(pod, rt, procs)

    def _previous_incarnation_gone(self, pod, rt, procs) -> bool:
        """Restart gate: a pod of a job whose earlier pods were torn down
        starts only once every process of those pods has exited.  Until
        then an old master may still be serving the job's rendezvous store
        on its port, and a new replica would join THAT world (the cause of
        the round-2 kill/rejoin stall, docs/multi_gpu.md "Restarts").  The
        first pod admitted after the drain opens a new restart generation
        for the job (PTO_RESTART_GENERATION), and if something outside the
        job still holds its port, the job moves to a fresh one."""
        jk = rt.job_key
        ids = self.retired.get(jk)
        if ids:
            live = sorted(i for i in ids if (procs.get(i) or {}).get("state") == "running")
            if live:
                self._write_status(pod, rt, {"phase": "Pending", "conditions": [
                    {"type": "PodScheduled", "status": "False", "reason": "PreviousIncarnationRunning",
                     "message": f"waiting for {len(live)} process(es) of the job's previous pods to exit"}]})
                return False
            del self.retired[jk]
            self._drained.add(jk)
        if jk in self._drained:
            self._drained.discard(jk)
            self.job_gen[jk] = self.job_gen.get(jk, 0) + 1
            port = self.job_ports.get(jk)
            peers = [r for r in self.pods.values() if r.job_key == jk and r is not rt and r.stage in ("init", "run")]
            if port is not None and not peers and not _port_free(port):
                log.warning("job %s: port %d still bound after its pods exited; taking a new one", jk, port)
                self._drop_job_port(jk)
        return True

    def _admit(self, pod, rt) -> bool:
        n = sum(gpus_requested(c) for c in pod.get("spec", {}).get("containers") or [])
        ann = pod["metadata"].get("annotations") or {}
        group = ann.get(C.ANNOTATION_GANG_GROUP)
        if n == 0 and not group:
            return True
        requests = [{"owner": rt.owner, "count": n, "hbm": _pod_hbm(pod)}]
        if group:
            members = [p for p in self.pod_informer.list(namespace_of(pod))
                       if (p["metadata"].get("annotations") or {}).get(C.ANNOTATION_GANG_GROUP) == group]
            try:
                pg = self.client.get("podgroups", namespace_of(pod), group)
                min_member = int(pg.get("spec", {}).get("minMember", len(members)))
            except ApiError:
                min_member = len(members)
            if len(members) < min_member:
                self._set_unschedulable(pod, rt, f"{len(members)}/{min_member} gang members present")
                return False
            requests = [{"owner": _owner(m), "count": sum(gpus_requested(c) for c in m["spec"].get("containers", [])),
                         "hbm": _pod_hbm(m)} for m in members]
        r = self.agent.alloc(requests)
        if not r.get("ok"):
            self._set_unschedulable(pod, rt, r.get("error", "insufficient amd.com/gpu"))
            return False
        rt.gpus = list(r["assigned"].get(rt.owner, []))
        if group:  # the whole gang's GPUs: "job" visibility shows them to every member
            self._gang_gpus[rt.job_key] = {o: list(g) for o, g in r["assigned"].items()}
        return True

    def _job_peer_devices(self, rt) -> list[int]:
        """Devices of the other replicas of rt's job on this node (live
        runtimes, plus the job's gang assignment for members not started)."""
        slots = set()
        for r in self.pods.values():
            if r is not rt and r.job_key == rt.job_key and r.gpus:
                slots.update(r.gpus)
        for owner, gs in self._gang_gpus.get(rt.job_key, {}).items():
            if owner != rt.owner:
                slots.update(gs)
        return sorted({g // self.gpu_share for g in slots})

    def _set_unschedulable(self, pod, rt, msg):
        st = {"phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False",
                                                 "reason": "Unschedulable", "message": msg}]}
        self._write_status(pod, rt, st)

    def _run_init(self, pod, rt, procs) -> bool:
        inits = pod.get("spec", {}).get("initContainers") or []
        while rt.init_index < len(inits):
            c = inits[rt.init_index]
            cmd = " ".join(c.get("command") or []) + " " + " ".join(c.get("args") or [])
            m = re.search(r"nslookup\s+([\w.-]+)", cmd)
            if c.get("name") == "init-pytorch" or m:
                svc = m.group(1) if m else None
                if svc and self.svc_informer.get_by_key(f"{namespace_of(pod)}/{svc}") is None:
                    self._write_status(pod, rt, self._pending_status(pod, "PodInitializing"))
                    return False
                rt.init_index += 1
                continue
            pid = f"{rt.owner}/init/{c.get('name')}"
            st = procs.get(pid)
            if st is None:
                self._spawn(pod, rt, c, pid, restart_policy="Never")
                self._write_status(pod, rt, self._pending_status(pod, "PodInitializing"))
                return False
            if st["state"] != "terminated":
                return False
            if st["exit_code"] != 0:
                if pod["spec"].get("restartPolicy") == "Never":
                    self._write_status(pod, rt, {"phase": "Failed", "reason": "InitContainerFailed"})
                    rt.stage = "done"
                    return False
                self.agent.remove(pid)  # retry
                return False
            rt.init_index += 1
        return True

    def _pending_status(self, pod, reason):
        return {"phase": "Pending", "hostIP": NODE_ADDRESS, "podIP": NODE_ADDRESS,
                "conditions": [{"type": "PodScheduled", "status": "True"},
                               {"type": "Initialized", "status": "False", "reason": reason}]}

    def _log_path(self, pod, container=None):
        base = f"{namespace_of(pod)}_{name_of(pod)}"
        return os.path.join(self.log_dir, base + (f".{container}" if container else "") + ".log")

    def _clear_pod_files(self, pod):
        """A new pod starts with empty logs and metrics, even when an earlier
        pod of the same name left files behind (its first-step record would
        otherwise be read as this pod's)."""
        names = [None, "metrics"] + [c.get("name") for c in (pod["spec"].get("containers") or []) +
                                     (pod["spec"].get("initContainers") or [])]
        for n in names:
            p = self._log_path(pod, n)
            for path in (p, p.replace(".log", ".jsonl")):
                try:
                    os.unlink(path)
                except FileNotFoundError:
                    pass

    @staticmethod
    def _job_key(pod) -> str:
        job = (pod["metadata"].get("labels") or {}).get(C.LABEL_JOB_NAME) or name_of(pod)
        return f"{namespace_of(pod)}/{job}"

    def _job_port(self, pod, wanted: int) -> int:
        jk = self._job_key(pod)
        if jk in self.job_ports:
            return self.job_ports[jk]
        used = set(self.job_ports.values())
        port = wanted
        while True:
            if port not in used and _port_free(port):
                fd = _reserve_port(port)
                if fd is not None:
                    self._port_locks[port] = fd
                    break
            port += 1
        self.job_ports[jk] = port
        return port

    def _release_job_ports(self, pods):
        """Give back the virtual master port (and its host-wide lock) of every
        job that no longer has a pod on this node.  A job keeps its port while
        any of its pods exists, so a replica restarted next to live peers
        gets the port they rendezvous on; a job whose pods are all gone (or
        re-submitted later) takes a fresh reservation."""
        live = {self._job_key(p) for p in pods}
        for jk in [jk for jk in self.job_ports if jk not in live and jk not in self.retired]:
            self._drop_job_port(jk)
        for jk in [jk for jk in self._gang_gpus if jk not in live]:
            del self._gang_gpus[jk]

    def _drop_job_port(self, jk):
        port = self.job_ports.pop(jk)
        fd = self._port_locks.pop(port, None)
        if fd is not None:
            try:
                os.close(fd)  # drops the flock
            except OSError:
                pass

    def _resolve_env(self, pod, c, rt) -> dict:
        env = {k: v for k, v in os.environ.items() if not k.startswith(("MASTER_", "RANK", "WORLD_SIZE",
                                                                          "LOCAL_RANK", "GROUP_RANK"))}
        pp = env.get("PYTHONPATH", "")
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
        env.update(self.extra_env)
        for e in c.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
            elif "valueFrom" in e:  # fieldRef subset
                fr = (e["valueFrom"] or {}).get("fieldRef", {}).get("fieldPath", "")
                env[e["name"]] = {"metadata.name": name_of(pod), "metadata.namespace": namespace_of(pod),
                                  "status.podIP": NODE_ADDRESS, "spec.nodeName": self.node_name}.get(fr, "")
        # single-node service "DNS" + per-job port virtualisation
        addr = env.get("MASTER_ADDR")
        if addr and addr != "localhost" and self.svc_informer.get_by_key(f"{namespace_of(pod)}/{addr}"):
            env["PTO_MASTER_SERVICE"] = addr
            env["MASTER_ADDR"] = NODE_ADDRESS
        if addr == "localhost":
            env["MASTER_ADDR"] = NODE_ADDRESS
        if "MASTER_PORT" in env:
            env["PTO_MASTER_PORT_REQUESTED"] = env["MASTER_PORT"]
            env["MASTER_PORT"] = str(self._job_port(pod, int(env["MASTER_PORT"])))
        # GPU pinning (module doc): one process per allocated GPU
        if gpus_requested(c) > 0 or rt.gpus:
            mine = sorted({g // self.gpu_share for g in rt.gpus})  # allocator slot -> device
            mode = (pod["metadata"].get("annotations") or {}).get(GPU_VISIBILITY_ANNOTATION) or self.gpu_visibility
            if mode not in GPU_VISIBILITY_MODES:
                mode = self.gpu_visibility
            if mode == "node":
                n = int(self.agent.gpus()["count"]) // self.gpu_share
                env["HIP_VISIBLE_DEVICES"] = _physical_ids(list(range(n)))
                env["LOCAL_RANK"] = str(mine[0] if mine else 0)
                env["LOCAL_WORLD_SIZE"] = env.get("WORLD_SIZE", "1")  # single node: every replica is local
            elif mode == "job":
                peers = [d for d in self._job_peer_devices(rt) if d not in mine]
                env["HIP_VISIBLE_DEVICES"] = _physical_ids(mine + peers)
                env["LOCAL_RANK"] = "0"
                env["LOCAL_WORLD_SIZE"] = "1"
            else:
                env["HIP_VISIBLE_DEVICES"] = _physical_ids(mine)
                env["LOCAL_RANK"] = "0"
                env["LOCAL_WORLD_SIZE"] = "1"
            env["PTO_GPU_IDS"] = _physical_ids(mine)
        else:
            env["HIP_VISIBLE_DEVICES"] = ""
            env["PTO_NO_GPU"] = "1"
        env.setdefault("LOCAL_RANK", "0")
        env.setdefault("LOCAL_WORLD_SIZE", "1")
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
        # one TCPStore implementation for every replica of a job: the
        # zygote-forked ones must use the classic store (node/zygote.py), and
        # a libuv server with classic clients was seen to hang the rendezvous
        env.setdefault("USE_LIBUV", "0")
        # every replica runs on this node and the rendezvous address is
        # 127.0.0.1: gloo's transport binds to the loopback device directly
        # instead of resolving the machine's hostname (on a box whose
        # resolver times out, every rank of a 4-replica job was seen stuck in
        # the ProcessGroupGloo constructor for minutes)
        env.setdefault("GLOO_SOCKET_IFNAME", "lo")
        env["PTO_RESTART_GENERATION"] = str(self.job_gen.get(rt.job_key, 0))
        env["PTO_POD_NAME"] = name_of(pod)
        env["PTO_NAMESPACE"] = namespace_of(pod)
        env["PTO_JOB_NAME"] = (pod["metadata"].get("labels") or {}).get(C.LABEL_JOB_NAME, "")
        env["PTO_METRICS_FILE"] = self._log_path(pod, "metrics").replace(".log", ".jsonl")
        return env

    def _argv(self, c) -> list[str]:
        if c.get("command"):
            argv = list(c["command"])
        else:
            image = c.get("image", "")
            if image not in self.images:
                raise KeyError(f"image {image!r} is not available on this node")
            argv = list(self.images[image])
        argv += [str(a) for a in c.get("args") or []]
        if argv and argv[0] in ("python", "python3"):
            argv[0] = sys.executable
        return argv

    def _spawn(self, pod, rt, c, pid, restart_policy, group=""):
        log_path = self._log_path(pod) if c.get("name") == C.DEFAULT_CONTAINER_NAME else \
            self._log_path(pod, c.get("name"))
        try:
            argv = self._argv(c)
        except KeyError as e:
            self._write_status(pod, rt, {"phase": "Pending", "containerStatuses": [
                {"name": c.get("name"), "ready": False, "restartCount": 0, "image": c.get("image"),
                 "state": {"waiting": {"reason": "ErrImagePull", "message": str(e)}}}]})
            return
        env = self._resolve_env(pod, c, rt)
        # The rank that hosts the rendezvous TCPStore server of a multi-rank
        # job starts as a fresh interpreter: in a zygote-forked one the
        # store server hung in its constructor (observed on the GPU box:
        # master stuck in _create_c10d_store while the 3 workers had
        # connected; replicas that are only store clients were fine).
        multi = int(env.get("WORLD_SIZE", "1") or 1) > 1
        hosts_store = env.get("RANK") == "0" and multi
        # the replicas of a multi-rank job restart in place as one group
        # (node_agent.cpp "restart groups"): a DDP world cannot take back a
        # single restarted rank
        self.agent.spawn(pid, argv, env=env, cwd=c.get("workingDir") or REPO_ROOT,
                         log=log_path, restart_policy=restart_policy, launcher="exec" if hosts_store else "auto",
                         group=rt.job_key if (group and multi) else "")
        rt.proc_ids.append(pid)
        if c.get("name") == C.DEFAULT_CONTAINER_NAME:
            eff = {k: env[k] for k in _EFFECTIVE_KEYS if k in env}
            self._annotate(pod, {EFFECTIVE_ENV_ANNOTATION: json.dumps(eff, sort_keys=True)})

    def _start_containers(self, pod, rt):
        policy = pod.get("spec", {}).get("restartPolicy") or "Always"
        # only replicas the node restarts in place form the restart group: a
        # Never pod (ExitCode jobs: the controller recreates it under a new
        # generation) must not be killed by an in-place wave, nor be waited for
        in_place = policy in ("OnFailure", "Always")
        for c in pod["spec"].get("containers") or []:
            self._spawn(pod, rt, c, f"{rt.owner}/{c.get('name')}", restart_policy=policy,
                        group=rt.job_key if (self.group_restarts and in_place) else "")

    def _report(self, pod, rt, procs):
        statuses = []
        running = terminated_ok = terminated_bad = waiting = 0
        for c in pod["spec"].get("containers") or []:
            st = procs.get(f"{rt.owner}/{c.get('name')}")
            cs = {"name": c.get("name"), "image": c.get("image"), "restartCount": 0, "ready": False}
            if st is None:
                cs["state"] = {"waiting": {"reason": "ContainerCreating"}}
                waiting += 1
            else:
                cs["restartCount"] = st["restart_count"]
                if st["state"] == "running":
                    cs["state"] = {"running": {"startedAt": _ts(st["started_at"])}}
                    cs["ready"] = True
                    running += 1
                elif st["state"] == "terminated":
                    cs["state"] = {"terminated": {"exitCode": st["exit_code"], "signal": st["signal"],
                                                  "reason": st["reason"], "startedAt": _ts(st["started_at"]),
                                                  "finishedAt": _ts(st["finished_at"])}}
                    if st["exit_code"] == 0:
                        terminated_ok += 1
                    else:
                        terminated_bad += 1
                else:
                    cs["state"] = {"waiting": {"reason": st["reason"]}}
                    waiting += 1
                if st["restart_count"] > 0:
                    cs["lastState"] = {"terminated": {"exitCode": st["last_exit_code"],
                                                      "finishedAt": _ts(st["last_finished_at"])}}
            statuses.append(cs)
        n = len(statuses)
        if terminated_ok == n and n:
            phase = "Succeeded"
        elif terminated_ok + terminated_bad == n and terminated_bad:
            phase = "Failed"
        elif running or waiting:
            phase = "Running" if (running or any(s["restartCount"] for s in statuses)) else "Pending"
        else:
            phase = "Pending"
        status = {"phase": phase, "hostIP": NODE_ADDRESS, "podIP": NODE_ADDRESS, "startTime": rt.started_at,
                  "containerStatuses": statuses,
                  "conditions": [{"type": "PodScheduled", "status": "True"},
                                 {"type": "Initialized", "status": "True"},
                                 {"type": "Ready", "status": "True" if phase == "Running" else "False"}]}
        if pod["spec"].get("initContainers"):
            status["initContainerStatuses"] = [{"name": c.get("name"), "restartCount": 0, "ready": True,
                                                "state": {"terminated": {"exitCode": 0, "reason": "Completed"}}}
                                               for c in pod["spec"]["initContainers"]]
        # metrics first: a pod seen Succeeded already carries its first-step
        # annotation (readers act on the phase)
        self._read_metrics(pod, rt)
        self._write_status(pod, rt, status)
        if phase in ("Succeeded", "Failed"):
            rt.stage = "done"
            self.agent.free(rt.owner)

    def _read_metrics(self, pod, rt):
        """Tail the trainer's metrics stream ($PTO_METRICS_FILE): first
        optimizer step and throughput become pod annotations and, with an
        OperatorMetrics attached, the pytorchjob_* Prometheus series
        (the reference's per-pod cAdvisor PromQL,
        docs/monitoring/README.md:18-47)."""
        path = self._log_path(pod, "metrics").replace(".log", ".jsonl")
        if not os.path.exists(path):
            return
        ann = {}
        labels = pod["metadata"].get("labels") or {}
        job = labels.get(C.LABEL_JOB_NAME) or name_of(pod)
        replica = f"{labels.get(C.LABEL_REPLICA_TYPE, '')}-{labels.get(C.LABEL_REPLICA_INDEX, '')}"
        m = self.metrics
        with open(path) as f:
            f.seek(rt.metrics_pos)
            while True:
                pos = f.tell()
                line = f.readline()
                if not line:
                    break
                if not line.endswith("\n"):  # partial write: re-read next time
                    f.seek(pos)
                    break
                try:
                    rec = json.loads(line)
                except json.JSONDecodeError:
                    continue
                ev = rec.get("event")
                if ev == "first_step" and not rt.annotated_first_step:
                    ann[FIRST_STEP_ANNOTATION] = repr(float(rec["t"]))
                    rt.annotated_first_step = True
                    if m is not None and rec.get("rank", 0) == 0:
                        created = self._job_created(pod, job)
                        if created is not None:
                            m.submit_to_first_step.labels(job=job).set(max(0.0, float(rec["t"]) - created))
                if ev == "startup":
                    ann[STARTUP_ANNOTATION] = json.dumps({k: v for k, v in rec.items() if k != "event"})
                if "samples_per_sec" in rec:
                    ann[THROUGHPUT_ANNOTATION] = str(rec["samples_per_sec"])
                    if m is not None:
                        m.samples_per_second.labels(job=job, replica=replica).set(float(rec["samples_per_sec"]))
                if m is not None and "step_seconds" in rec:
                    m.step_seconds.labels(job=job, replica=replica).set(float(rec["step_seconds"]))
                if m is not None and ev == "comm":
                    us = rec.get("xgmi_us") if rec.get("transport") == "xgmi" else rec.get("rccl_us")
                    if us is not None:
                        m.allreduce_seconds.labels(job=job, replica=replica).set(float(us) * 1e-6)
            rt.metrics_pos = f.tell()
        if ann:
            self._annotate(pod, ann)

    def _job_created(self, pod, job) -> float | None:
        """Job creation time (unix seconds): sub-second from the API server
        when it has it, else creationTimestamp."""
        fn = getattr(self.client, "created_unix", None)
        try:
            t = fn("pytorchjobs", namespace_of(pod), job) if fn else None
            if t is not None:
                return t
            j = self.client.get("pytorchjobs", namespace_of(pod), job)
        except (ApiError, OSError):
            return None
        return parse_rfc3339(j.get("metadata", {}).get("creationTimestamp"))

    def update_node_metrics(self):
        """Per-GPU HBM used/total from the amdgpu sysfs counters
        (``<sysfs>/class/drm/card*/device/mem_info_vram_{used,total}``)."""
        if self.metrics is None:
            return
        for gpu, used, total in read_hbm(self.sysfs_root):
            self.metrics.gpu_hbm_used.labels(gpu=gpu).set(used)
            self.metrics.gpu_hbm_total.labels(gpu=gpu).set(total)

    def _annotate(self, pod, ann):
        try:
            self.client.patch("pods", namespace_of(pod), name_of(pod), {"metadata": {"annotations": ann}})
        except ApiError:
            pass

    def _write_status(self, pod, rt, status):
        if status == rt.last_status:
            return
        try:
            cur = self.client.get("pods", namespace_of(pod), name_of(pod))
        except ApiError:
            return
        if cur["metadata"].get("uid") != rt.uid:
            return
        cur["status"] = status
        try:
            self.client.update_status("pods", cur)
            rt.last_status = copy.deepcopy(status)
        except ApiError as e:
            log.debug("pod status write failed: %s", e)

    # ------------------------------------------------------------ faults
    def inject_fault(self, namespace, name, container="pytorch", signal=9):
        """SIGKILL (or other signal) a running replica: the fault-injection
        hook for the kill/rejoin path.  The process may be
        restarted by its restart policy (exit 137 is retryable)."""
        rt = self.pods.get(f"{namespace}/{name}")
        if rt is None:
            raise KeyError(f"pod {namespace}/{name} is not running on this node")
        return self.agent.kill(f"{rt.owner}/{container}", signal=signal, restartable=True)


def _owner(pod) -> str:
    return f"{key_of(pod)}@{pod['metadata'].get('uid', '')}"


def read_hbm(sysfs_root: str = "/sys") -> list[tuple[str, int, int]]:
    """[(card, vram_used_bytes, vram_total_bytes)] for every amdgpu card."""
    import glob

    out = []
    for d in sorted(glob.glob(os.path.join(sysfs_root, "class", "drm", "card*", "device"))):
        try:
            with open(os.path.join(d, "mem_info_vram_used")) as f:
                used = int(f.read().strip())
            with open(os.path.join(d, "mem_info_vram_total")) as f:
                total = int(f.read().strip())
        except (OSError, ValueError):
            continue
        out.append((os.path.basename(os.path.dirname(d)), used, total))
    return out


def _visible_gpu_count() -> int:
    """GPUs this node manager may hand out: the HIP-visible devices of its
    own process (torch.cuda.device_count() does not initialise the GPU)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:
        return 0


def _physical_ids(idx: list[int]) -> str:
    """Allocator indices are relative to this process's visible devices;
    translate through an inherited HIP/CUDA_VISIBLE_DEVICES list so the
    child sees exactly the allocated physical GPUs."""
    parent = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if parent:
        plist = [p.strip() for p in parent.split(",") if p.strip()]
        return ",".join(plist[i] for i in idx if i < len(plist))
    return ",".join(map(str, idx))


def _ts(t):
    if not t:
        return None
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))
