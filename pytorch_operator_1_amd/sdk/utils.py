"""SDK helpers (reference ``sdk/python/kubeflow/pytorchjob/utils/utils.py:19-75``)."""
import os

from . import constants


def is_running_in_k8s():
    return os.path.isdir("/var/run/secrets/kubernetes.io/")


def get_current_k8s_namespace():
    with open("/var/run/secrets/kubernetes.io/serviceaccount/namespace", "r") as f:
        return f.readline()


def get_default_target_namespace():
    if not is_running_in_k8s():
        return os.environ.get("PTO_NAMESPACE", "default")
    return get_current_k8s_namespace()


def set_pytorchjob_namespace(pytorchjob):
    md = pytorchjob.get("metadata", {}) if isinstance(pytorchjob, dict) else (pytorchjob.metadata or {})
    ns = md.get("namespace") if isinstance(md, dict) else md.namespace
    return ns or get_default_target_namespace()


def get_labels(name, master=False, replica_type=None, replica_index=None):
    """Label selector for a job's pods.  Unlike the reference (which tests
    ``if replica_index:``), index 0 is honoured."""
    labels = {
        constants.PYTORCHJOB_GROUP_LABEL: "kubeflow.org",
        constants.PYTORCHJOB_CONTROLLER_LABEL: "pytorch-operator",
        constants.PYTORCHJOB_NAME_LABEL: name,
    }
    if master:
        labels[constants.PYTORCHJOB_ROLE_LABEL] = "master"
    if replica_type:
        labels[constants.PYTORCHJOB_TYPE_LABEL] = str.lower(replica_type)
    if replica_index is not None:
        labels[constants.PYTORCHJOB_INDEX_LABEL] = str(replica_index)
    return labels


def to_selector(labels):
    return ",".join("{0}={1}".format(k, v) for k, v in labels.items())
