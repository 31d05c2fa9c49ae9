#!/usr/bin/env python3
"""Submit -> first optimizer step latency through the whole local stack
(apiserver -> controller -> kubelet -> node agent [-> zygote] -> trainer).

Prints one JSON line per run: {"zygote": bool, "submit_to_first_step_s": t}.
``--gpu`` runs the fused HIP trainer on one GPU (rccl backend, world 1);
otherwise the eager trainer on CPU (gloo).  The cluster (and the zygote's
imports) are warmed up before the first timed submit, like a node that is
already up when a job arrives."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--zygote", choices=["0", "1", "both"], default="both")
    args = ap.parse_args()
    os.environ.setdefault("TMPDIR", "/tmp")
    from pytorch_operator_1_amd.api.types import new_job
    from pytorch_operator_1_amd.cluster import LocalCluster

    modes = ["0", "1"] if args.zygote == "both" else [args.zygote]
    for z in modes:
        os.environ["PTO_ZYGOTE"] = z
        with LocalCluster(gpus=None if args.gpu else 0) as c:
            if z == "1":
                c.kubelet.agent.wait_warm(120)
            for i in range(args.runs):
                name = f"lat-z{z}-{i}"
                margs = (["--backend", "rccl", "--impl", "fused"] if args.gpu else ["--backend", "gloo", "--no-cuda"])
                margs += ["--max-steps", "20", "--log-interval", "10", "--no-test", "--train-size", "2048"]
                job = new_job(name, image="pto/pytorch-mnist:rocm", master_args=margs, workers=0,
                              gpus=1 if args.gpu else 0)
                t0 = time.time()
                c.submit(job)
                j = c.wait_for_condition(name, timeout=300)
                pod = c.store.get("pods", "default", f"{name}-master-0")
                ann = pod["metadata"].get("annotations", {})
                first = float(ann.get("pto.amd.com/first-step-unix", "nan"))
                st = j["status"]["conditions"][-1]["type"]
                print(json.dumps({"zygote": z == "1", "run": i, "state": st, "gpu": args.gpu,
                                  "submit_to_first_step_s": round(first - t0, 3)}), flush=True)
                c.store.delete("pytorchjobs", "default", name)


if __name__ == "__main__":
    main()
