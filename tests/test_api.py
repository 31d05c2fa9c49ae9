"""API schema: defaulting, validation (reference validation_test.go cases),
CRD OpenAPI constraints, naming helpers, exit-code table."""
import copy
import os

import pytest
import yaml

from pytorch_operator_1_amd.api import constants as C
from pytorch_operator_1_amd.api import crd
from pytorch_operator_1_amd.api.defaults import set_defaults
from pytorch_operator_1_amd.api.types import (gen_general_name, gen_labels, gen_owner_reference,
                                               get_port_from_job, is_retryable_exit_code, new_job, total_replicas)
from pytorch_operator_1_amd.api.validation import ValidationError, validate_resources, validate_spec

EXAMPLES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")


def _spec(containers, rtype="Master", replicas=None):
    s = {"template": {"spec": {"containers": containers}}}
    if replicas is not None:
        s["replicas"] = replicas
    return {"pytorchReplicaSpecs": {rtype: s}}


# The six invalid specs of pkg/apis/pytorch/validation/validation_test.go:26-114
INVALID = [
    ({"pytorchReplicaSpecs": None}, "PyTorchJobSpec is not valid"),
    (_spec([]), "containers definition expected in Master"),
    (_spec([{"image": ""}]), "Image is undefined in the container of Master"),
    (_spec([{"name": "", "image": "gcr.io/kubeflow-ci/pytorch-dist-mnist_test:1.0"}]),
     "There is no container named pytorch in Master"),
    (_spec([{"name": "pytorch", "image": "gcr.io/kubeflow-ci/pytorch-dist-mnist_test:1.0"}], replicas=2),
     "There must be only 1 master replica"),
    (_spec([{"name": "pytorch", "image": "gcr.io/kubeflow-ci/pytorch-dist-mnist_test:1.0"}], rtype="Worker",
           replicas=1), "Master ReplicaSpec must be present"),
]


@pytest.mark.parametrize("spec,msg", INVALID)
def test_validation_rejects(spec, msg):
    with pytest.raises(ValidationError) as e:
        validate_spec(spec)
    assert msg in str(e.value)


def test_validation_bad_replica_type():
    spec = _spec([{"name": "pytorch", "image": "x"}])
    spec["pytorchReplicaSpecs"]["PS"] = {"template": {"spec": {"containers": [{"name": "pytorch", "image": "x"}]}}}
    with pytest.raises(ValidationError, match="PyTorchReplicaType is PS but must be one of"):
        validate_spec(spec)


def test_valid_job_passes():
    validate_spec(new_job("ok", workers=3)["spec"])


def test_defaults():
    job = new_job("d", workers=2)
    spec = job["spec"]["pytorchReplicaSpecs"]
    spec["master"] = spec.pop("Master")  # case-insensitive key normalisation
    spec["worker"] = spec.pop("Worker")
    del spec["worker"]["replicas"]
    del spec["master"]["restartPolicy"]
    set_defaults(job)
    s = job["spec"]
    assert s["cleanPodPolicy"] == "None"
    assert set(s["pytorchReplicaSpecs"]) == {"Master", "Worker"}
    assert s["pytorchReplicaSpecs"]["Worker"]["replicas"] == 1
    assert s["pytorchReplicaSpecs"]["Master"]["restartPolicy"] == "OnFailure"
    ports = s["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]["ports"]
    assert ports == [{"name": "pytorchjob-port", "containerPort": 23456}]
    assert "ports" not in s["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
    # idempotent
    j2 = copy.deepcopy(job)
    set_defaults(j2)
    assert j2 == job
    assert get_port_from_job(job) == 23456


def test_default_port_prefers_container_named_pytorch():
    job = new_job("p", workers=0)
    cs = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"]
    cs.insert(0, {"name": "sidecar", "image": "s"})
    set_defaults(job)
    assert "ports" not in cs[0]
    assert cs[1]["ports"][0]["containerPort"] == 23456


def test_names_and_labels():
    assert gen_general_name("job", "Master", 0) == "job-master-0"
    assert gen_general_name("ns/job", "Worker", 3) == "ns-job-worker-3"
    assert gen_labels("j") == {"group-name": "kubeflow.org", "job-name": "j", "pytorch-job-name": "j",
                               "controller-name": "pytorch-operator"}
    job = new_job("j")
    job["metadata"]["uid"] = "u1"
    ref = gen_owner_reference(job)
    assert ref["controller"] and ref["blockOwnerDeletion"] and ref["kind"] == "PyTorchJob" and ref["uid"] == "u1"
    assert total_replicas(new_job("w", workers=7)) == 8


@pytest.mark.parametrize("code,retry", [(1, False), (2, False), (126, False), (127, False), (128, False),
                                        (139, False), (130, True), (137, True), (138, True), (143, True),
                                        (0, False), (255, False)])
def test_exit_codes(code, retry):
    assert is_retryable_exit_code(code) == retry


def test_crd_openapi_constraints():
    job = new_job("c", workers=1)
    assert crd.openapi_check(job) is None
    job["spec"]["pytorchReplicaSpecs"]["Master"]["replicas"] = 2
    assert "less than or equal to 1" in crd.openapi_check(job)
    job = new_job("c", workers=1)
    job["spec"]["pytorchReplicaSpecs"]["Worker"]["replicas"] = 0
    assert "greater than or equal to 1" in crd.openapi_check(job)
    m = crd.crd_manifest()
    assert m["metadata"]["name"] == "pytorchjobs.kubeflow.org"
    assert m["spec"]["subresources"] == {"status": {}}
    assert m["spec"]["additionalPrinterColumns"][0]["JSONPath"] == ".status.conditions[-1:].type"


def test_example_manifests_validate():
    n = 0
    for root, _, files in os.walk(EXAMPLES):
        for f in files:
            if f.endswith(".yaml"):
                for doc in yaml.safe_load_all(open(os.path.join(root, f))):
                    if doc and doc.get("kind") == C.KIND:
                        set_defaults(doc)
                        validate_spec(doc["spec"])
                        validate_resources(doc)
                        assert crd.openapi_check(doc) is None
                        n += 1
    assert n >= 3


def test_generated_artifacts_up_to_date():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "hack", "gen_manifests.py"), "--verify"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("q,v", [("288Gi", 288 * 2 ** 30), ("200G", 200e9), ("1.5e3", 1500.0), (7, 7.0),
                                 ("512Mi", 512 * 2 ** 20), ("1k", 1000.0)])
def test_parse_quantity(q, v):
    from pytorch_operator_1_amd.api.validation import parse_quantity

    assert parse_quantity(q) == v


def test_hbm_request_validation():
    job = new_job("h", workers=1, gpus=1)
    c = job["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
    c.setdefault("resources", {}).setdefault("limits", {})[C.HBM_RESOURCE] = "200G"
    validate_resources(job)
    c["resources"]["limits"][C.HBM_RESOURCE] = "300G"
    with pytest.raises(ValidationError, match="an MI355X has 288 GB"):
        validate_resources(job)
