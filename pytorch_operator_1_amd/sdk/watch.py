"""Streaming status table (reference ``api/py_torch_job_watch.py:28-59``:
NAME / STATE / TIME rows until the job is Succeeded or Failed; retried up
to 20 times one second apart on stream errors)."""
from __future__ import annotations

import sys
import time

from . import constants, utils


def _row(name, state, t, out):
    out.write(f"{name:<30}{state:<20}{t:<30}\n")
    out.flush()


def watch(api, name=None, namespace=None, timeout_seconds=600, out=None, retries=20):
    out = out or sys.stdout
    if namespace is None:
        namespace = utils.get_default_target_namespace()
    _row("NAME", "STATE", "TIME", out)
    end = time.time() + timeout_seconds
    def rows(job):
        jname = job["metadata"]["name"]
        conds = job.get("status", {}).get("conditions", []) or []
        status = conds[-1].get("type", "") if conds else ""
        t = conds[-1].get("lastTransitionTime", "") if conds else ""
        return jname, status, t

    for attempt in range(retries):
        try:
            # list first (current state), then stream changes from that version
            lst = api.list(constants.PYTORCHJOB_PLURAL, namespace)
            for job in lst.get("items", []):
                jname, status, t = rows(job)
                if name and name != jname:
                    continue
                _row(jname, status, t, out)
                if name == jname and status in ("Succeeded", "Failed"):
                    return job
            stream = api.watch(constants.PYTORCHJOB_PLURAL, namespace,
                               resource_version=lst.get("metadata", {}).get("resourceVersion"),
                               timeout_seconds=max(1, int(end - time.time())))
            for _, job in stream:
                jname = job["metadata"]["name"]
                if name and name != jname:
                    continue
                conds = job.get("status", {}).get("conditions", []) or []
                status = conds[-1].get("type", "") if conds else ""
                t = conds[-1].get("lastTransitionTime", "") if conds else ""
                _row(jname, status, t, out)
                if name == jname and status in ("Succeeded", "Failed"):
                    stream.stop()
                    return job
                if time.time() > end:
                    stream.stop()
                    return None
            return None
        except Exception:
            if attempt == retries - 1:
                raise
            time.sleep(1)
