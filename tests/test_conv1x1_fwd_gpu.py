"""ops/conv1x1.py forward on the owned MFMA kernel (``pto_conv1x1_fwd``: the
implicit GEMM of csrc/kernels/conv3x3.hip with one tap) against fp32
``F.conv2d`` of the same bf16 operands for every 1x1 shape of ResNet-50
(batch scaled down, the strided downsample convs included), its
BN-statistics epilogue against sums over the stored output, the backward
through the owned forward, and a whole bottleneck (conv1 -> bn1 -> 3x3 ->
bn2 -> conv3 -> bn3 + residual) against the MIOpen-forward path."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

# (Ci, Co, input H = W, stride): conv1 / conv3 / downsample of the four stages
SHAPES = [(64, 64, 56, 1), (256, 64, 56, 1), (64, 256, 56, 1), (256, 256, 56, 1),
          (256, 128, 56, 1), (256, 512, 56, 2), (512, 128, 28, 1), (128, 512, 28, 1),
          (512, 1024, 28, 2), (1024, 256, 14, 1), (256, 1024, 14, 1), (1024, 2048, 14, 2),
          (2048, 512, 7, 1), (512, 2048, 7, 1)]


@pytest.fixture(autouse=True)
def _owned_forward(monkeypatch):
    monkeypatch.setenv("PTO_CONV1X1_FWD", "1")


def relerr(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


def _conv(ci, co, stride):
    return nn.Conv2d(ci, co, 1, stride=stride, bias=False).to(DEV, memory_format=torch.channels_last)


def _x(N, C, H):
    return torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def test_owned_forward_is_the_native_kernel():
    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.ops import conv1x1 as c1

    conv = _conv(64, 64, 1)
    x = _x(2, 64, 8)
    assert c1.owned_fwd_supported(x, conv.weight, torch.bfloat16)
    with torch.no_grad():
        c1.conv1x1(x, conv)
    assert _lib.loaded_path() is not None and hasattr(conv, "_pto_c1_wb")


@pytest.mark.parametrize("ci,co,H,stride", SHAPES)
def test_conv1x1_fwd_and_stats_match_fp32(ci, co, H, stride):
    from pytorch_operator_1_amd.ops import conv1x1 as c1
    from pytorch_operator_1_amd.ops.conv3x3 import ConvStats, stats_tiles

    torch.manual_seed(ci + co + H + stride)
    N = 4 if H >= 28 else 8
    conv = _conv(ci, co, stride)
    x = _x(N, ci, H)
    st = ConvStats()
    with torch.no_grad():
        y = c1.conv1x1(x, conv, stats=st)
        ref = F.conv2d(x.float(), conv.weight.to(torch.bfloat16).float(), stride=stride)
    assert y.dtype == torch.bfloat16 and y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert relerr(y, ref) < 8e-3, relerr(y, ref)
    part, nblk = st.take()
    assert part is not None and nblk == stats_tiles(N, ref.shape[2], ref.shape[3], co)
    p = part.view(nblk, 2, co).double().sum(0)
    yf = y.double()
    s_ref, q_ref = yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))
    assert float((p[0] - s_ref).abs().max() / s_ref.abs().max()) < 1e-5
    assert float((p[1] - q_ref).abs().max() / q_ref.abs().max()) < 1e-5


@pytest.mark.parametrize("ci,co,H,stride", [(64, 256, 56, 1), (256, 512, 56, 2), (2048, 512, 7, 1)])
def test_conv1x1_backward_through_owned_forward(ci, co, H, stride):
    """dX / dW of the GEMM backward (fed by the owned forward's saved bf16
    filter image) against fp32 autograd of the same bf16 operands."""
    from pytorch_operator_1_amd.ops import conv1x1 as c1

    torch.manual_seed(11 + ci)
    conv = _conv(ci, co, stride)
    x = _x(4, ci, H)
    xa = x.clone().requires_grad_(True)
    y = c1.conv1x1(xa, conv)
    dy = torch.randn_like(y.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    xr = x.float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    F.conv2d(xr, wr, stride=stride).backward(dy.float())
    assert relerr(xa.grad, xr.grad) < 1e-2, relerr(xa.grad, xr.grad)
    assert conv.weight.grad.dtype == torch.float32
    assert relerr(conv.weight.grad, wr.grad) < 1e-2, relerr(conv.weight.grad, wr.grad)


@pytest.mark.parametrize("cin,width,stride,down", [(256, 64, 1, False), (256, 128, 2, True)])
def test_bottleneck_owned_1x1_matches_miopen_forward(monkeypatch, cin, width, stride, down):
    """A whole bottleneck with the owned 1x1 forwards (statistics from their
    epilogues) against the same block with MIOpen's 1x1 forwards (BN
    statistics pass), bf16 autocast: output, input / weight gradients and
    running statistics."""
    from pytorch_operator_1_amd.models.resnet import Bottleneck

    torch.manual_seed(5)
    blocks = [Bottleneck(cin, width, stride, down).to(DEV, memory_format=torch.channels_last) for _ in range(2)]
    blocks[1].load_state_dict(blocks[0].state_dict())
    x0 = _x(4, cin, 28)
    outs = []
    for blk, owned in zip(blocks, ("1", "0")):
        monkeypatch.setenv("PTO_CONV1X1_FWD", owned)
        x = x0.clone().requires_grad_(True)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            y = blk(x)
        y.float().square().mean().backward()
        outs.append((y.float(), x.grad.float(), blk.conv1.weight.grad, blk.conv3.weight.grad, blk.bn3.running_mean,
                     blk.bn1.running_var))
    assert hasattr(blocks[0].conv1, "_pto_c1_wb") and not hasattr(blocks[1].conv1, "_pto_c1_wb")
    for a, b in zip(*outs):
        assert relerr(a, b) < 2e-2, relerr(a, b)


@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("ci,co,H,stride", [(64, 256, 56, 1), (1024, 2048, 14, 2), (2048, 512, 7, 1)])
def test_conv1x1_kernel_variants_agree(variant, ci, co, H, stride):
    """Every launch variant of pto_conv1x1_fwd (one / two LDS buffers, the
    resident grid walking the tiles) computes the same output and the same
    statistics partials (same MFMA order per tile)."""
    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.ops import conv1x1 as c1
    from pytorch_operator_1_amd.ops.conv3x3 import ConvStats

    torch.manual_seed(ci + co)
    conv = _conv(ci, co, stride)
    x = _x(4 if H >= 28 else 8, ci, H)
    L = _lib.lib()
    outs = []
    for v in (1, variant):
        _lib.check(L.pto_conv1x1_set_variant(v), "set_variant")
        st = ConvStats()
        with torch.no_grad():
            y = c1.conv1x1(x, conv, stats=st)
        part, _ = st.take()
        outs.append((y.clone(), part.clone()))
    _lib.check(L.pto_conv1x1_set_variant(1), "set_variant")
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
