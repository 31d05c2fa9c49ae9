"""Point-to-point smoke test (reference ``examples/smoke-dist/dist_sendrecv.py``).

Rank 0 sends a 2x2 fp32 tensor to every worker in turn and receives back
its element-wise square; the env contract is logged first.  On GPUs the
tensors live in HBM and travel over RCCL p2p (xGMI); on CPU over gloo.
Exit code 0 only if every returned tensor is exactly the square.
"""
from __future__ import annotations

import logging
import os
import sys

import torch
import torch.distributed as dist

from ..utils import dist as pdist


def run(device) -> bool:
    rank, size = dist.get_rank(), dist.get_world_size()
    g = torch.Generator().manual_seed(1234)
    inp = torch.randn(2, 2, generator=g).to(device)
    result = torch.zeros(2, 2, device=device)
    ok = True
    if rank == 0:
        for i in range(1, size):
            dist.send(tensor=inp, dst=i)
            dist.recv(tensor=result, src=i)
            logging.info("Result from worker %d : %s", i, result.cpu().tolist())
            ok &= torch.equal(result.cpu(), (inp * inp).cpu())
    else:
        dist.recv(tensor=inp, src=0)
        result = torch.mul(inp, inp)
        dist.send(tensor=result, dst=0)
    return ok


def main():
    logging.getLogger().setLevel(logging.INFO)
    logging.info("Torch version: %s", torch.__version__)
    for k in ("MASTER_PORT", "MASTER_ADDR", "WORLD_SIZE", "RANK"):
        logging.info("%s: %s", k, os.environ.get(k, "{}"))
    use_gpu = torch.cuda.is_available() and os.environ.get("PTO_NO_GPU") != "1"
    backend = os.environ.get("PTO_BACKEND") or ("nccl" if use_gpu else "gloo")
    _, device = pdist.init_distributed(backend, use_gpu=use_gpu)
    ok = run(device)
    pdist.cleanup()
    logging.info("sendrecv %s", "OK" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
