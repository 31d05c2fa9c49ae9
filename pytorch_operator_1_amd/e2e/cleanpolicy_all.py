"""e2e "cleanpolicy-all": with ``cleanPodPolicy: All`` every pod of the
succeeded job is deleted by the operator, then the job itself is deleted
(reference ``test/e2e/v1/cleanpolicy/cleanpolicy_all.go:145-224``)."""
from __future__ import annotations

import sys

from ..api import constants as C
from ..utils.misc import pformat
from .common import expect_deleted_job, main, make_job, wait_finished, wait_gone


def scenario(client, args, name):
    client.create(C.PLURAL, make_job(args, name, clean_pod_policy="All"), args.namespace)
    job = wait_finished(client, args.namespace, name, args.timeout, args.poll)
    if job is None or not any(c.get("type") == C.JOB_SUCCEEDED for c in job["status"].get("conditions", [])):
        raise RuntimeError(f"PyTorchJob {name} did not succeed;\n{pformat(job)}")
    selector = f"group-name={C.GROUP_NAME},pytorch-job-name={name.replace('/', '-')}"
    if not wait_gone(lambda: not client.list("pods", args.namespace, label_selector=selector)["items"],
                     args.timeout, args.poll):
        raise RuntimeError(f"Not all pods are successfully deleted for PyTorchJob {name}.")
    expect_deleted_job(client, args.namespace, name, args)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:], "e2e-cleanpolicy-all", scenario))
