#!/usr/bin/env python3
"""Run the LDS access-pattern probe kernels (tools/probes/lds_patterns.hip)
once; meant to run under rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT.
Usage: python tools/lds_patterns_probe.py [--build]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "probes", "lds_patterns.hip")
SO = os.path.join(ROOT, "tools", "probes", "liblds_patterns.so")


def main():
    if "--build" in sys.argv:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                               "-shared", "-o", SO, SRC])
        print("built", SO)
        return
    import torch

    out = torch.zeros(256, dtype=torch.int32, device="cuda")
    lib = ctypes.CDLL(SO)
    lib.probe_lds_patterns.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rc = lib.probe_lds_patterns(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0, rc
    lib.probe_lds_rules.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rc = lib.probe_lds_rules(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0, rc
    print("ok", int(out.sum()))
    print("p_rule dispatch order: kind (b32, read2 a/a+1, b64 at 2a) x mode (consecutive, one address, "
          "lane&15, lane>>2, wgrad patch, patch w/o 2g, stride 2, one bank)")


if __name__ == "__main__":
    main()
