"""Pod / Service / PodGroup control and claim-adopt logic.

Reference (vendored): ``tf-operator/pkg/control/pod_control.go:55-177``
(RealPodControl: create from template with labels, annotations,
finalizers, ownerRef; events SuccessfulCreatePod / FailedCreatePod /
SuccessfulDeletePod / FailedDeletePod; DeletePod skips terminating pods and
ignores NotFound), ``service_control.go:42-219`` (+ FakeServiceControl
with CreateLimit/Err injection), ``k8s.io/kubernetes/pkg/controller/
controller_utils.go:610-690`` (FakePodControl), ``controller_ref_manager.go``
(claim/adopt/release), ``jobcontroller.go:224-278`` (PodGroup sync).
"""
from __future__ import annotations

import copy
import threading

from ..api import constants as C
from ..apiserver.store import ApiError


class RealPodControl:
    def __init__(self, client, recorder):
        self.client, self.recorder = client, recorder

    def create_pods_with_controller_ref(self, namespace, template, owner, controller_ref):
        pod = {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {
                "name": template["metadata"]["name"],
                "namespace": namespace,
                "labels": copy.deepcopy(template.get("metadata", {}).get("labels") or {}),
                "annotations": copy.deepcopy(template.get("metadata", {}).get("annotations") or {}),
                "ownerReferences": [controller_ref],
            },
            "spec": copy.deepcopy(template.get("spec") or {}),
        }
        if template.get("metadata", {}).get("finalizers"):
            pod["metadata"]["finalizers"] = list(template["metadata"]["finalizers"])
        try:
            out = self.client.create("pods", pod, namespace)
        except ApiError as e:
            self.recorder.event(owner, "Warning", "FailedCreatePod", f"Error creating: {e.message}")
            raise
        self.recorder.event(owner, "Normal", "SuccessfulCreatePod", f"Created pod: {pod['metadata']['name']}")
        return out

    def delete_pod(self, namespace, name, owner):
        try:
            pod = self.client.get("pods", namespace, name)
        except ApiError as e:
            if e.code == 404:
                return
            raise
        if pod["metadata"].get("deletionTimestamp"):
            return
        try:
            self.client.delete("pods", namespace, name)
        except ApiError as e:
            if e.code == 404:
                return
            self.recorder.event(owner, "Warning", "FailedDeletePod", f"Error deleting: {e.message}")
            raise
        self.recorder.event(owner, "Normal", "SuccessfulDeletePod", f"Deleted pod: {name}")


class RealServiceControl:
    def __init__(self, client, recorder):
        self.client, self.recorder = client, recorder

    def create_services_with_controller_ref(self, namespace, service, owner, controller_ref):
        svc = copy.deepcopy(service)
        svc.setdefault("apiVersion", "v1")
        svc.setdefault("kind", "Service")
        svc["metadata"]["namespace"] = namespace
        svc["metadata"]["ownerReferences"] = [controller_ref]
        try:
            out = self.client.create("services", svc, namespace)
        except ApiError as e:
            self.recorder.event(owner, "Warning", "FailedCreateService", f"Error creating: {e.message}")
            raise
        self.recorder.event(owner, "Normal", "SuccessfulCreateService",
                            f"Created service: {svc['metadata']['name']}")
        return out

    def delete_service(self, namespace, name, owner):
        try:
            self.client.delete("services", namespace, name)
        except ApiError as e:
            if e.code == 404:
                return
            self.recorder.event(owner, "Warning", "FailedDeleteService", f"Error deleting: {e.message}")
            raise
        self.recorder.event(owner, "Normal", "SuccessfulDeleteService", f"Deleted service: {name}")


class FakePodControl:
    """Records templates instead of creating pods (test double)."""

    def __init__(self):
        self.lock = threading.Lock()
        self.templates, self.controller_refs, self.delete_pod_names = [], [], []
        self.err = None
        self.create_limit = 0
        self.create_call_count = 0

    def create_pods_with_controller_ref(self, namespace, template, owner, controller_ref):
        with self.lock:
            self.create_call_count += 1
            if self.create_limit and self.create_call_count > self.create_limit:
                raise ApiError(500, "InternalError", "not creating pod, limit exceeded")
            if self.err:
                raise self.err
            self.templates.append(copy.deepcopy(template))
            self.controller_refs.append(controller_ref)

    def delete_pod(self, namespace, name, owner):
        with self.lock:
            if self.err:
                raise self.err
            self.delete_pod_names.append(name)

    def clear(self):
        with self.lock:
            self.templates, self.controller_refs, self.delete_pod_names = [], [], []
            self.create_call_count = 0


class FakeServiceControl:
    def __init__(self):
        self.lock = threading.Lock()
        self.templates, self.controller_refs, self.delete_service_names = [], [], []
        self.err = None
        self.create_limit = 0
        self.create_call_count = 0

    def create_services_with_controller_ref(self, namespace, service, owner, controller_ref):
        with self.lock:
            self.create_call_count += 1
            if self.create_limit and self.create_call_count > self.create_limit:
                raise ApiError(500, "InternalError", "not creating service, limit exceeded")
            if self.err:
                raise self.err
            self.templates.append(copy.deepcopy(service))
            self.controller_refs.append(controller_ref)

    def delete_service(self, namespace, name, owner):
        with self.lock:
            if self.err:
                raise self.err
            self.delete_service_names.append(name)


def claim_objects(objs, job, selector_labels, client, resource, job_deleting: bool):
    """ControllerRefManager.Claim: keep objects this job controls, adopt
    matching orphans (unless the job is being deleted), release objects it
    controls that no longer match the selector."""
    uid = job["metadata"].get("uid")
    out = []
    for o in objs:
        md = o.get("metadata", {})
        labels = md.get("labels") or {}
        matches = all(labels.get(k) == v for k, v in selector_labels.items())
        refs = md.get("ownerReferences") or []
        ctrl = next((r for r in refs if r.get("controller")), None)
        if ctrl is not None:
            if ctrl.get("uid") != uid:
                continue  # owned by someone else
            if matches:
                out.append(o)
            elif client is not None:  # release
                try:
                    client.patch(resource, md.get("namespace"), md["name"],
                                 {"metadata": {"ownerReferences": [r for r in refs if r.get("uid") != uid]}})
                except ApiError:
                    pass
            continue
        if not matches or job_deleting or md.get("deletionTimestamp"):
            continue
        if client is not None:  # adopt orphan
            from ..api.types import gen_owner_reference

            try:
                o = client.patch(resource, md.get("namespace"), md["name"],
                                 {"metadata": {"ownerReferences": refs + [gen_owner_reference(job)]}})
            except ApiError:
                continue
        out.append(o)
    return out


def sync_pod_group(client, job, min_available: int):
    """Create the kube-batch PodGroup (minMember = total replicas) owned by
    the job if missing (jobcontroller.go:224-248)."""
    from ..api.types import gen_owner_reference, gen_pod_group_name, name_of, namespace_of

    ns, name = namespace_of(job), gen_pod_group_name(name_of(job))
    try:
        return client.get("podgroups", ns, name)
    except ApiError as e:
        if e.code != 404:
            raise
    pg = {"apiVersion": "scheduling.incubator.k8s.io/v1alpha1", "kind": "PodGroup",
          "metadata": {"name": name, "namespace": ns, "ownerReferences": [gen_owner_reference(job)]},
          "spec": {"minMember": int(min_available)}}
    return client.create("podgroups", pg, ns)


def delete_pod_group(client, recorder, job):
    from ..api.types import gen_pod_group_name, name_of, namespace_of

    try:
        client.delete("podgroups", namespace_of(job), gen_pod_group_name(name_of(job)))
    except ApiError as e:
        if e.code != 404:
            recorder.event(job, "Warning", "FailedDeletePodGroup", f"Error deleting: {e.message}")
            raise
        return
    recorder.event(job, "Normal", "SuccessfulDeletePodGroup", f"Deleted PodGroup: {name_of(job)}")
