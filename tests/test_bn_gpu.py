"""Fused BatchNorm(+add)(+ReLU) HIP kernels (ops/bn.py) vs a plain PyTorch
fp32 reference of the same math: outputs, running statistics, and the
gradients of x, gamma, beta and the residual."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def relerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("C,HW", [(64, 28), (256, 14), (2048, 7), (8, 5)])
@pytest.mark.parametrize("variant", ["plain", "relu", "add_relu"])
def test_bn_act_matches_fp32_reference(C, HW, variant):
    from pytorch_operator_1_amd.ops.bn import BatchNormAct, fused_supported

    torch.manual_seed(C + HW)
    N = 6
    x = (torch.randn(N, C, HW, HW, device=DEV) * 3 + 1).bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x) if variant == "add_relu" else None
    relu = variant != "plain"
    assert fused_supported(x)
    m = BatchNormAct(C).to(DEV)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    ref = BatchNormAct(C).to(DEV)
    ref.load_state_dict(m.state_dict())
    xa = x.clone().requires_grad_(True)
    ra = res.clone().requires_grad_(True) if res is not None else None
    y = m(xa, residual=ra, relu=relu)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    # fp32 reference
    xb = x.float().requires_grad_(True)
    rb = res.float().requires_grad_(True) if res is not None else None
    yr = F.batch_norm(xb, ref.running_mean, ref.running_var, ref.weight, ref.bias, True, 0.1, 1e-5)
    if rb is not None:
        yr = yr + rb
    if relu:
        yr = F.relu(yr)
    assert relerr(y, yr) < 1e-2
    assert relerr(m.running_mean, ref.running_mean) < 1e-4
    assert relerr(m.running_var, ref.running_var) < 1e-4
    assert int(m.num_batches_tracked) == 1
    dy = torch.randn_like(yr)
    y.backward(dy.bfloat16().contiguous(memory_format=torch.channels_last))
    yr.backward(dy)
    assert relerr(xa.grad, xb.grad) < 2e-2
    assert relerr(m.weight.grad, ref.weight.grad) < 1e-2
    assert relerr(m.bias.grad, ref.bias.grad) < 1e-2
    if res is not None:
        assert relerr(ra.grad, rb.grad) < 1e-2


def test_resnet_fused_bn_grads_match_stock_bn():
    """A small ResNet-50 (64x64 images) with the fused BN path and the same
    weights through stock MIOpen BN (PTO_FUSED_BN=0), both under bf16
    autocast, each compared with an fp32 run of the model: the fused path
    must be as close to fp32 as the stock bf16 path is (50 layers of bf16
    backprop at batch 4 are noisy for both)."""
    import os

    from pytorch_operator_1_amd.models.resnet import resnet50

    torch.manual_seed(0)
    models = [resnet50(10).to(DEV, memory_format=torch.channels_last) for _ in range(3)]
    for m in models[1:]:
        m.load_state_dict(models[0].state_dict())
    x = torch.randn(4, 3, 64, 64, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=DEV)
    losses = []
    for mdl, mode in zip(models, ("fused", "stock", "fp32")):
        os.environ["PTO_FUSED_BN"] = "1" if mode == "fused" else "0"
        try:
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                out = mdl(x)
            loss = F.cross_entropy(out.float(), y)
            loss.backward()
        finally:
            os.environ.pop("PTO_FUSED_BN", None)
        losses.append(loss.item())
    assert abs(losses[0] - losses[2]) <= 2 * abs(losses[1] - losses[2]) + 1e-2
    fused, stock, ref = (dict(m.named_parameters()) for m in models)
    worse = []
    for n, pr in ref.items():
        if pr.grad is None or pr.grad.norm() == 0:
            continue
        ef, es = relerr(fused[n].grad, pr.grad), relerr(stock[n].grad, pr.grad)
        if ef > 1.5 * es + 0.02:
            worse.append((n, ef, es))
    assert not worse, worse[:5]


@pytest.mark.parametrize("down,stride", [(False, 1), (True, 1), (True, 2)])
def test_conv1x1_gemm_bottleneck_matches_miopen(down, stride):
    """ops/conv1x1.py: the block's 1x1 convs with GEMM input gradients and
    split-K fp32 weight gradients; in an identity bottleneck bn3's residual
    gradient folded into conv1's input-gradient GEMM instead of autograd's
    add; in a downsample block (stride 1 or 2) the two 1x1 convs' input
    gradients merged into one tensor.  Every gradient (input included)
    under bf16 autocast must be as close to an fp32 run as the stock path's
    (PTO_CONV1X1_GEMM=0) is."""
    import os

    from pytorch_operator_1_amd.models.resnet import Bottleneck

    torch.manual_seed(0)
    cin = 128 if down else 256
    blocks = [Bottleneck(cin, 64, stride=stride, down=down).to(DEV, memory_format=torch.channels_last)
              for _ in range(3)]
    for b in blocks[1:]:
        b.load_state_dict(blocks[0].state_dict())
    x0 = torch.randn(4, cin, 28, 28, device=DEV).contiguous(memory_format=torch.channels_last)
    dout = torch.randn(4, 256, 28 // stride, 28 // stride, device=DEV).contiguous(memory_format=torch.channels_last)
    grads = []
    for blk, mode in zip(blocks, ("gemm", "miopen", "fp32")):
        os.environ["PTO_CONV1X1_GEMM"] = "0" if mode == "miopen" else "1"
        try:
            # the block input is the previous block's bf16 output under autocast
            x = (x0 if mode == "fp32" else x0.to(torch.bfloat16)).clone().requires_grad_(True)
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                out = blk(x)
            out.float().backward(dout)
        finally:
            os.environ.pop("PTO_CONV1X1_GEMM", None)
        g = {n: p.grad.float().clone() for n, p in blk.named_parameters() if p.grad is not None}
        g["input"] = x.grad.float().clone()
        grads.append(g)
    gemm, mi, ref = grads
    worse = []
    for n, gr in ref.items():
        if gr.norm() == 0:
            continue
        eg, em = relerr(gemm[n], gr), relerr(mi[n], gr)
        if eg > 1.5 * em + 0.02:
            worse.append((n, eg, em))
    assert not worse, worse[:5]
    assert set(gemm) == set(ref)


def test_conv1x1_res_fp32_matches_conv_plus_residual():
    """fp32: conv1x1_res's input gradient = F.conv2d's input gradient + the
    stashed residual gradient (one GEMM with beta = 1); output and weight
    gradient equal F.conv2d's."""
    import torch.nn as nn

    from pytorch_operator_1_amd.ops.conv1x1 import GradStash, conv1x1_res

    torch.manual_seed(1)
    conv = nn.Conv2d(96, 40, 1, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(3, 96, 17, 19, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    res = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
    st = GradStash()
    y = conv1x1_res(x, conv, st)
    dy = torch.randn_like(y)
    st.put(res.clone())
    y.backward(dy)
    gw = conv.weight.grad.clone()
    conv.weight.grad = None
    y2 = conv(x2)
    y2.backward(dy)
    assert relerr(y, y2) < 1e-5
    assert relerr(x.grad, x2.grad + res) < 1e-5
    assert relerr(gw, conv.weight.grad) < 1e-5
    assert gw.stride() == conv.weight.stride()


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_matches_fp32_conv(stride):
    """ops/conv1x1.py conv1x1 in fp32 (stride 1 and the strided downsample
    form): output, input and weight gradients equal F.conv2d's."""
    import torch.nn as nn

    from pytorch_operator_1_amd.ops.conv1x1 import conv1x1

    torch.manual_seed(stride)
    conv = nn.Conv2d(48, 80, 1, stride=stride, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(2, 48, 15, 14, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    y = conv1x1(x, conv)
    dy = torch.randn_like(y)
    y.backward(dy)
    gw = conv.weight.grad.clone()
    conv.weight.grad = None
    y2 = conv(x2)
    y2.backward(dy)
    assert y.shape == y2.shape and relerr(y, y2) < 1e-5
    assert relerr(x.grad, x2.grad) < 1e-5
    assert relerr(gw, conv.weight.grad) < 1e-5 and gw.stride() == conv.weight.stride()


@pytest.mark.parametrize("M,co,ci", [(6272, 64, 256), (12544, 512, 128), (1000, 40, 96)])
def test_splitk_weight_grad_matches_fp32(M, co, ci):
    """ops/conv1x1.py weight_grad_1x1: S batched GEMMs over K = N*H*W with
    fp32 outputs, summed, vs an fp32 matmul of the same bf16 values."""
    from pytorch_operator_1_amd.ops.conv1x1 import _splitk, weight_grad_1x1

    torch.manual_seed(M)
    dy = torch.randn(M, co, device=DEV).bfloat16()
    x = torch.randn(M, ci, device=DEV).bfloat16()
    got = weight_grad_1x1(dy, x)
    assert got.dtype == torch.float32 and got.shape == (co, ci)
    assert (_splitk(M) > 1) == (M >= 6272)
    assert relerr(got, dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((3, 16, 7, 9), 3, 2, 1),
                                         ((2, 8, 10, 10), 2, 2, 0), ((2, 24, 9, 8), 3, 1, 1)])
def test_maxpool_matches_fp32_reference(shape, k, s, p):
    """HIP max pool (ops/pool.py) vs F.max_pool2d in fp32 on the same bf16
    values: forward bitwise (a max selects an input), backward through the
    argmax codes -- including ties (coarsely quantised inputs: the first
    maximum wins, as in torch) and windows whose taps overlap."""
    from pytorch_operator_1_amd.ops.pool import _MaxPool, maxpool_supported

    torch.manual_seed(sum(shape) + k)
    x = (torch.randint(-4, 5, shape, device=DEV).float() / 2).bfloat16().contiguous(memory_format=torch.channels_last)
    assert maxpool_supported(x, k, s, p)
    xr = x.float().detach().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    xh = x.detach().requires_grad_(True)
    yh = _MaxPool.apply(xh, k, s, p)
    assert yh.shape == yr.shape and yh.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(yh.float(), yr.detach())
    g = torch.randn_like(yr).bfloat16()
    yr.backward(g.float())
    yh.backward(g)
    assert xh.grad.dtype == torch.bfloat16
    torch.testing.assert_close(xh.grad.float(), xr.grad.bfloat16().float(), rtol=1e-2, atol=1e-2)
    # NaN propagates like torch
    xn = x.clone()
    xn[0, 0, 1, 1] = float("nan")
    assert torch.equal(torch.isnan(_MaxPool.apply(xn, k, s, p).float()), torch.isnan(F.max_pool2d(xn.float(), k, s, p)))


@pytest.mark.parametrize("N", [2, 5])
def test_stem_conv_matches_fp32_reference(N):
    """ops/stem.py: the MFMA implicit-GEMM stem conv (7x7/2, pad 3, 3 -> 64,
    channels-last bf16) vs an fp32 conv of the same bf16 values; weight
    gradient (MIOpen) vs the fp32 reference; both weight layouts."""
    import torch.nn as nn

    from pytorch_operator_1_amd.ops.stem import stem_conv, stem_supported

    torch.manual_seed(N)
    for cl in (True, False):
        conv = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
        if cl:
            conv = conv.to(memory_format=torch.channels_last)
        x = torch.randn(N, 3, 224, 224, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
        assert stem_supported(x, conv)
        y = stem_conv(x, conv)
        assert y.dtype == torch.bfloat16 and y.shape == (N, 64, 112, 112)
        assert y.is_contiguous(memory_format=torch.channels_last)
        wr = conv.weight.detach().bfloat16().float().requires_grad_(True)
        yr = F.conv2d(x.float(), wr, stride=2, padding=3)
        assert relerr(y, yr) < 4e-3
        dy = torch.randn_like(yr)
        y.backward(dy.bfloat16())
        yr.backward(dy)
        assert conv.weight.grad.dtype == torch.float32 and conv.weight.grad.stride() == conv.weight.stride()
        assert relerr(conv.weight.grad, wr.grad) < 2e-2
