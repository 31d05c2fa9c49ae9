"""Transposed-weight linear (dX from a W^T copy) vs F.linear autograd, on
CPU in fp32 (the HIP transpose kernel is covered in test_llm_gpu.py)."""
import torch
import torch.nn.functional as F

from pytorch_operator_1_amd.ops import llm


def test_linear_tw_grads_match_linear():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 16, dtype=torch.float64, requires_grad=True)
    w = torch.randn(24, 16, dtype=torch.float64, requires_grad=True)
    wt = torch.empty(16, 24, dtype=torch.float64)
    llm.transpose_into(w.detach(), wt)
    y = llm.linear_tw(x, w, wt)
    ref = F.linear(x, w)
    assert torch.allclose(y, ref)
    g = torch.randn_like(ref)
    dx, dw = torch.autograd.grad(y, (x, w), g)
    rx, rw = torch.autograd.grad(ref, (x, w), g)
    assert torch.allclose(dx, rx) and torch.allclose(dw, rw)


def test_linear_tw_skips_unneeded_grads():
    x = torch.randn(3, 8)
    w = torch.randn(4, 8, requires_grad=True)
    wt = w.detach().t().contiguous()
    (dw,) = torch.autograd.grad(llm.linear_tw(x, w, wt).sum(), (w,))
    assert torch.allclose(dw, torch.ones(3, 4).t().mm(x))
