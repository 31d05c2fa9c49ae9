#!/usr/bin/env python3
"""Does the hardware honour a stream's CU mask, eagerly and under HIP-graph
replay?  (utils/cu_partition.py)

For the unmasked default stream and for every partition k of n (n = 2, 4, 8;
layouts "block" and "stride"), launch k_cu_id (8192 one-wave workgroups that
each read HW_REG_XCC_ID / HW_REG_HW_ID and idle ~10 µs) eagerly and from a
replayed graph, and record which physical CUs (XCD, SE, SH, CU) ran them.
Prints one JSON document; with --out also writes it there.

    python tools/cu_partition_probe.py --out gpurun_out/cu_partition_probe.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(parts_list=(2, 4, 8), layouts=("block", "stride")) -> dict:
    import torch

    from pytorch_operator_1_amd.utils import cu_partition as cp

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    full = cp.probe_cus(torch.cuda.current_stream(dev))
    all_cus = set(full["cus"])
    out = {"device_cus": torch.cuda.get_device_properties(dev).multi_processor_count,
           "unmasked": {"n_cus": full["n_cus"], "cus_per_xcc": full["cus_per_xcc"], "queues": full["queues"]},
           "partitions": []}
    for layout in layouts:
        for n in parts_list:
            seen = []
            for k in range(n):
                p = cp.Partition(dev, k, n, layout=layout)
                e = cp.probe_cus(p.stream)
                g = cp.probe_cus(p.stream, graph=True)
                ce, cg = set(e["cus"]), set(g["cus"])
                seen.append(ce | cg)
                out["partitions"].append({
                    "layout": layout, "parts": n, "index": k, "mask_cus": len(p.bits),
                    "eager_cus": len(ce), "graph_cus": len(cg), "graph_within_eager": cg <= ce,
                    "eager_cus_per_xcc": e["cus_per_xcc"], "graph_cus_per_xcc": g["cus_per_xcc"],
                    "outside_unmasked_set": len((ce | cg) - all_cus)})
                p.close()
            overlap = sum(len(seen[a] & seen[b]) for a in range(n) for b in range(a + 1, n))
            out["partitions"].append({"layout": layout, "parts": n, "summary": True, "pairwise_overlap_cus": overlap,
                                      "union_cus": len(set().union(*seen))})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    a = ap.parse_args()
    res = run()
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
