"""e2e "defaults": a default-policy job (cleanPodPolicy None) succeeds,
all its pods exist afterwards, and deleting the job removes it
(reference ``test/e2e/v1/default/defaults.go:145-246``)."""
from __future__ import annotations

import sys

from ..api import constants as C
from ..utils.misc import pformat
from .common import expect_deleted_job, expect_pods_exist, main, make_job, wait_finished


def scenario(client, args, name):
    original = make_job(args, name)
    client.create(C.PLURAL, original, args.namespace)
    job = wait_finished(client, args.namespace, name, args.timeout, args.poll)
    if job is None or not any(c.get("type") == C.JOB_SUCCEEDED for c in job["status"].get("conditions", [])):
        raise RuntimeError(f"PyTorchJob {name} did not succeed;\n{pformat(job)}")
    expect_pods_exist(client, args.namespace, original)  # policy None keeps every pod
    expect_deleted_job(client, args.namespace, name, args)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:], "e2e-defaults", scenario))
