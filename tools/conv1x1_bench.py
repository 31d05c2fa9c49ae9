#!/usr/bin/env python3
"""ResNet-50's 1x1 stride-1 convolutions (batch 256, bf16, channels-last):
MIOpen (aten convolution / convolution_backward) vs the GEMM forms of
ops/conv1x1.py, per pass, us per call (median of 20).  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_operator_1_amd.ops import _lib  # noqa: E402

SHAPES = [  # (N, H, Ci, Co)
    (256, 56, 64, 64), (256, 56, 256, 64), (256, 56, 64, 256),
    (256, 28, 512, 128), (256, 28, 128, 512),
    (256, 14, 1024, 256), (256, 14, 256, 1024),
    (256, 7, 2048, 512), (256, 7, 512, 2048),
]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for N, H, ci, co in SHAPES:
        x = torch.randn(N, ci, H, H, device=dev, dtype=bf).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, 1, 1, device=dev, dtype=bf).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, co, H, H, device=dev, dtype=bf).contiguous(memory_format=torch.channels_last)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
        w2 = w.view(co, ci)
        g = torch.randn_like(x)
        g2 = g.permute(0, 2, 3, 1).reshape(-1, ci)
        r = {"shape": [N, H, ci, co]}
        r["miopen_fwd"] = timeit(lambda: F.conv2d(x, w))
        r["gemm_fwd"] = timeit(lambda: torch.mm(x2, w2.t()))
        # the owned MFMA forward (pto_conv1x1_fwd), without / with the BN
        # statistics partials
        L, st = _lib.lib(), _lib.stream_ptr(dev)
        yo = torch.empty(N, co, H, H, device=dev, dtype=bf, memory_format=torch.channels_last)
        part = torch.empty(((N * H * H + 255) // 64) * 2 * co, device=dev, dtype=torch.float32)
        for nb in (2, 3, 1):  # pto_conv1x1_set_variant: LDS buffers (1 = the default), 3 = resident grid
            _lib.check(L.pto_conv1x1_set_variant(nb), "set_variant")
            sfx = "" if nb == 1 else f"_nb{nb}"
            r["owned_fwd" + sfx] = timeit(lambda: L.pto_conv1x1_fwd(x.data_ptr(), w.data_ptr(), yo.data_ptr(), None,
                                                                    N, H, H, ci, co, 1, st))
            r["owned_fwd_stats" + sfx] = timeit(lambda: L.pto_conv1x1_fwd(x.data_ptr(), w.data_ptr(), yo.data_ptr(),
                                                                          part.data_ptr(), N, H, H, ci, co, 1, st))
            yo.zero_()
            L.pto_conv1x1_fwd(x.data_ptr(), w.data_ptr(), yo.data_ptr(), None, N, H, H, ci, co, 1, st)
            ref = F.conv2d(x, w).float()
            r["owned_err" + sfx] = float((yo.float() - ref).abs().max() / ref.abs().max())
        r["owned_err"] = float((yo.float() - F.conv2d(x, w).float()).abs().max() / F.conv2d(x, w).float().abs().max())
        r["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
        r["gemm_dgrad"] = timeit(lambda: torch.mm(dy2, w2))
        r["gemm_dgrad_acc"] = timeit(lambda: g2.addmm_(dy2, w2))
        r["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
        r["gemm_wgrad"] = timeit(lambda: torch.mm(dy2.t(), x2))
        r["gemm_wgrad_f32out"] = timeit(lambda: torch.mm(x2.t(), dy2))
        M = x2.shape[0]
        for S in (16, 64, 256):  # split-K over the N*H*W rows: S batched GEMMs, fp32 out, then the sum
            if M % S:
                continue
            dyb, xb = dy2.view(S, M // S, co).transpose(1, 2), x2.view(S, M // S, ci)
            r[f"bmm_wgrad_s{S}"] = timeit(lambda: torch.bmm(dyb, xb, out_dtype=torch.float32).sum(0))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
