"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of
the same op (MI355X only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib_loaded():
    from pytorch_operator_1_amd.ops import _lib

    _lib.lib()
    assert _lib.loaded_path() is not None


def rel_err(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def test_library_is_native():
    _lib_loaded()
    import os

    from pytorch_operator_1_amd.ops import _lib

    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert os.path.basename(_lib.LIB_PATH) in maps


@pytest.mark.parametrize("B", [64, 7, 100])
def test_conv1_relu_pool(B):
    from pytorch_operator_1_amd import ops

    torch.manual_seed(0)
    x = torch.randn(B, 1, 28, 28, device=DEV, requires_grad=True)
    w = (torch.randn(20, 1, 5, 5, device=DEV) * 0.2).requires_grad_()
    b = (torch.randn(20, device=DEV) * 0.1).requires_grad_()
    y = ops.conv2d_bias_relu_maxpool(x, w, b)
    yr = F.max_pool2d(F.relu(F.conv2d(x, w, b)), 2, 2)
    assert rel_err(y, yr) < 1e-5
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), g)
    gxr, gwr, gbr = torch.autograd.grad(yr, (x, w, b), g)
    assert rel_err(gw, gwr) < 1e-4
    assert rel_err(gb, gbr) < 1e-4
    assert rel_err(gx, gxr) < 1e-4


@pytest.mark.parametrize("B", [64, 5])
def test_conv2_relu_pool(B):
    from pytorch_operator_1_amd import ops

    torch.manual_seed(1)
    x = torch.relu(torch.randn(B, 20, 12, 12, device=DEV)).requires_grad_()
    w = (torch.randn(50, 20, 5, 5, device=DEV) * 0.05).requires_grad_()
    b = (torch.randn(50, device=DEV) * 0.1).requires_grad_()
    y = ops.conv2d_bias_relu_maxpool(x, w, b)
    yr = F.max_pool2d(F.relu(F.conv2d(x, w, b)), 2, 2)
    assert rel_err(y, yr) < 1e-5
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), g)
    gxr, gwr, gbr = torch.autograd.grad(yr, (x, w, b), g)
    assert rel_err(gw, gwr) < 1e-4
    assert rel_err(gb, gbr) < 1e-4
    assert rel_err(gx, gxr) < 1e-4


@pytest.mark.parametrize("B", [64, 3])
def test_conv12_fused_forward(B):
    """F12: conv1+conv2 (+bias/ReLU/pool) in one launch vs torch fp32, with
    the image copy-out for the backward; deterministic run to run."""
    from pytorch_operator_1_amd.ops import _lib

    L = _lib.lib()
    torch.manual_seed(2)
    x = torch.randn(B, 1, 28, 28, device=DEV)
    w1 = torch.randn(20, 1, 5, 5, device=DEV) * 0.2
    b1 = torch.randn(20, device=DEV) * 0.1
    w2 = torch.randn(50, 20, 5, 5, device=DEV) * 0.05
    b2 = torch.randn(50, device=DEV) * 0.1
    a1r = F.max_pool2d(F.relu(F.conv2d(x, w1, b1)), 2, 2)
    a2r = F.max_pool2d(F.relu(F.conv2d(a1r, w2, b2)), 2, 2)
    outs = []
    for _ in range(2):
        a1p = torch.full((B * 2880,), float("nan"), device=DEV)
        a2p = torch.full((B * 800,), float("nan"), device=DEV)
        c1 = torch.empty(B * 2880, dtype=torch.uint8, device=DEV)
        c2 = torch.empty(B * 800, dtype=torch.uint8, device=DEV)
        xo = torch.full((B * 784,), float("nan"), device=DEV)
        _lib.check(L.pto_conv12_fwd_lazy_x(x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                                           a1p.data_ptr(), c1.data_ptr(), a2p.data_ptr(), c2.data_ptr(), B, None, None,
                                           None, 0, None, None, 0.0, 0.0, 1.0, 0, xo.data_ptr(), None, None, 1, 0,
                                           _lib.stream_ptr()), "conv12")
        torch.cuda.synchronize()
        outs.append((a1p.clone(), a2p.clone(), c1.clone(), c2.clone()))
        assert torch.equal(xo.view(B, 1, 28, 28), x)
    a1p, a2p, c1, c2 = outs[0]
    assert rel_err(a1p.view(B, 20, 12, 12), a1r) < 1e-5
    assert rel_err(a2p.view(B, 50, 4, 4), a2r) < 1e-5
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)


@pytest.mark.parametrize("M,N,K,relu", [(64, 500, 800, True), (64, 10, 500, False), (33, 70, 129, True),
                                        (1, 16, 4, False)])
def test_linear(M, N, K, relu):
    from pytorch_operator_1_amd import ops

    torch.manual_seed(2)
    x = torch.randn(M, K, device=DEV, requires_grad=True)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).requires_grad_()
    b = torch.randn(N, device=DEV, requires_grad=True)
    y = ops.linear(x, w, b, relu=relu)
    yr = F.linear(x, w, b)
    if relu:
        yr = F.relu(yr)
    assert rel_err(y, yr) < 1e-5
    g = torch.randn_like(y)
    gs = torch.autograd.grad(y, (x, w, b), g)
    grs = torch.autograd.grad(yr, (x, w, b), g)
    for a, r in zip(gs, grs):
        assert rel_err(a, r) < 1e-5


@pytest.mark.parametrize("M", [64, 7, 100])
def test_fc1_forward_split_k(M):
    """pto_fc1_fwd_split (two workgroups per 16x16 tile, halves added by fp32
    atomics onto a zeroed buffer) against fp32 x W^T; two addends onto +0
    make the sum independent of arrival order, so repeats are bitwise equal."""
    from pytorch_operator_1_amd.ops import _lib

    torch.manual_seed(3)
    L = _lib.lib()
    x = torch.randn(M, 800, device=DEV)
    w = torch.randn(500, 800, device=DEV) / 800 ** 0.5
    outs = []
    for _ in range(3):
        h = torch.zeros(M * 500, device=DEV)
        _lib.check(L.pto_fc1_fwd_split(x.data_ptr(), w.data_ptr(), h.data_ptr(), M, _lib.stream_ptr()), "fc1 split")
        outs.append(h.view(M, 500).clone())
    torch.cuda.synchronize()
    ref = x.double() @ w.double().t()
    assert rel_err(outs[0].double(), ref) < 1e-5
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("split", ["1", "0"])
def test_fused_trainer_fc1_forms_match_eager(monkeypatch, split):
    """Both fc1 forward forms of the fused step (split-K with bias/ReLU in F4dx,
    and one workgroup per tile) against the stock PyTorch step, graphs on."""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer
    from pytorch_operator_1_amd.train.runner import EagerMnistTrainer

    monkeypatch.setenv("PTO_FC1_SPLIT", split)
    dev = torch.device(DEV)
    fused = FusedMnistTrainer(dev, batch_size=64, dataset_size=640, seed=1, graph="full")
    assert (fused.h1a is not None) == (split == "1")
    eager = EagerMnistTrainer(dev, batch_size=64, dataset_size=640, seed=1)
    fused.run(1)
    fused.run(7)
    for _ in range(8):
        eager.step()
    torch.cuda.synchronize()
    assert abs(fused.last_loss() - eager.last_loss()) < 1e-4
    for name, t in eager.model.state_dict().items():
        assert rel_err(fused.p[name], t) < 1e-4, name
    if split == "1":  # k_bwd_all leaves the accumulation buffer zeroed for the next F3
        assert not fused.h1a.any()


def test_log_softmax_and_ce():
    from pytorch_operator_1_amd import ops

    torch.manual_seed(3)
    x = torch.randn(64, 10, device=DEV, requires_grad=True)
    t = torch.randint(0, 10, (64,), device=DEV)
    y = ops.log_softmax(x)
    yr = F.log_softmax(x, dim=1)
    assert rel_err(y, yr) < 1e-6
    g = torch.randn_like(y)
    assert rel_err(torch.autograd.grad(y, x, g)[0], torch.autograd.grad(yr, x, g)[0]) < 1e-5
    l = ops.cross_entropy(x, t)
    lr_ = F.cross_entropy(x, t)
    assert abs(l.item() - lr_.item()) < 1e-5
    assert rel_err(torch.autograd.grad(l, x)[0], torch.autograd.grad(lr_, x)[0]) < 1e-5


def test_fused_sgd_matches_torch():
    from pytorch_operator_1_amd.ops import FusedSGD

    torch.manual_seed(4)
    ps = [torch.randn(s, device=DEV, requires_grad=True) for s in [(7,), (1000, 3), (5001,)]]
    qs = [p.detach().clone().requires_grad_() for p in ps]
    o1 = FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    o2 = torch.optim.SGD(qs, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    for _ in range(3):
        gs = [torch.randn_like(p) for p in ps]
        for p, q, g in zip(ps, qs, gs):
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            q.grad = g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ps, qs):
        assert rel_err(p.detach(), q.detach()) < 1e-6


def test_mnist_module_hip_matches_torch():
    from pytorch_operator_1_amd.models.mnist import MnistNet

    torch.manual_seed(5)
    m1 = MnistNet(impl="hip").to(DEV)
    m2 = MnistNet(impl="torch").to(DEV)
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(64, 1, 28, 28, device=DEV)
    t = torch.randint(0, 10, (64,), device=DEV)
    l1 = F.nll_loss(m1(x), t)
    l2 = F.nll_loss(m2(x), t)
    assert abs(l1.item() - l2.item()) < 1e-5
    l1.backward()
    l2.backward()
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert rel_err(p1.grad, p2.grad) < 1e-4, n


@pytest.mark.parametrize("graph", ["none", "full"])
def test_fused_trainer_matches_eager(graph):
    """Fused step == stock PyTorch step (same init, same batches) over 5
    SGD-momentum steps."""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer
    from pytorch_operator_1_amd.train.runner import EagerMnistTrainer

    dev = torch.device(DEV)
    fused = FusedMnistTrainer(dev, batch_size=64, dataset_size=640, seed=1, graph=graph)
    eager = EagerMnistTrainer(dev, batch_size=64, dataset_size=640, seed=1)
    for name, t in eager.model.state_dict().items():
        assert torch.equal(fused.p[name], t), name
    for _ in range(5):
        fused.step()
        eager.step()
    torch.cuda.synchronize()
    assert abs(fused.last_loss() - eager.last_loss()) < 1e-4
    for name, t in eager.model.state_dict().items():
        assert rel_err(fused.p[name], t) < 1e-4, name


def test_fused_trainer_converges():
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    tr = FusedMnistTrainer(torch.device(DEV), batch_size=64, dataset_size=6400, seed=3)
    first = None
    for i in range(300):
        tr.step()
        if i == 0:
            first = tr.last_loss()
    assert tr.last_loss() < 0.5 * first


def test_cross_lane_helpers():
    """The DPP / v_permlane{16,32}_swap exchanges the reductions use
    (mfma_f32.h) against their definitions on one wave."""
    import numpy as np

    from pytorch_operator_1_amd.ops import _lib

    g = torch.Generator().manual_seed(7)
    a = torch.randn(64, generator=g)
    b = torch.randn(64, generator=g)
    out = torch.empty(11 * 64, device=DEV)
    ad, bd = a.to(DEV), b.to(DEV)  # keep the device copies alive until the launch has run
    _lib.check(_lib.lib().pto_lane_ops_selftest(ad.data_ptr(), bd.data_ptr(), out.data_ptr(), _lib.stream_ptr()),
               "lane_ops")
    torch.cuda.synchronize()
    o = out.view(11, 64).cpu().numpy().astype(np.float64)
    x, y, lane = a.numpy().astype(np.float64), b.numpy().astype(np.float64), np.arange(64)
    np.testing.assert_array_equal(o[0], x[lane ^ 1])
    np.testing.assert_array_equal(o[1], x[lane ^ 2])
    np.testing.assert_array_equal(o[2], x[lane ^ 7])
    np.testing.assert_array_equal(o[3], x[lane ^ 8])
    f32 = lambda v: v.astype(np.float32).astype(np.float64)
    np.testing.assert_array_equal(o[4], f32(x + x[lane ^ 32]))
    # halving step: a lane with the bit clear keeps slot a and adds its
    # partner's a; with the bit set, slot b plus the partner's b
    np.testing.assert_array_equal(o[5], f32(np.where(lane & 32, y + y[lane ^ 32], x + x[lane ^ 32])))
    np.testing.assert_array_equal(o[6], f32(np.where(lane & 16, y + y[lane ^ 16], x + x[lane ^ 16])))
    rows = x.reshape(4, 16)
    np.testing.assert_allclose(o[7], np.repeat(rows.sum(1), 16), rtol=1e-6)
    np.testing.assert_array_equal(o[8], np.repeat(rows.max(1), 16))
    np.testing.assert_allclose(o[9], np.full(64, x.sum()), rtol=1e-5)
    np.testing.assert_array_equal(o[10], np.full(64, x.max()))


def _synth_host(n: int, key: int):
    """numpy twin of k_synth_mnist: same hash, same float32 rounding."""
    import numpy as np

    from pytorch_operator_1_amd.models.mnist import BLOB_COLS, BLOB_ROWS

    r = np.arange(784) // 28
    c = np.arange(784) % 28
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64)[:, None] * np.uint64(785) + np.arange(785, dtype=np.uint64)[None]
        z = ctr * np.uint64(0x9E3779B97F4A7C15) + np.uint64(key)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    lab = (z[:, 784] % np.uint64(10)).astype(np.int64)
    u = (z[:, :784] >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    v = u * np.float32(0.3)
    y0, x0 = np.array(BLOB_ROWS)[lab][:, None], np.array(BLOB_COLS)[lab][:, None]
    blob = (r >= y0) & (r < y0 + 6) & (c >= x0) & (c < x0 + 6)
    v = np.clip(np.where(blob, v + np.float32(0.7), v).astype(np.float32), np.float32(0), np.float32(1))
    return (v - np.float32(0.1307)) / np.float32(0.3081), lab


def test_synthetic_mnist_kernel_matches_host_formula():
    """k_synth_mnist (the operator image's GPU data generator) against its
    numpy twin: labels exact, pixels within 1e-6, balanced classes,
    deterministic."""
    from pytorch_operator_1_amd.models.mnist import _synth_key, synthetic_mnist

    n = 3000
    x, y = synthetic_mnist(n, DEV, seed=5, source="hash")
    torch.cuda.synchronize()
    hx, hy = _synth_host(n, _synth_key(5))
    assert torch.equal(y.cpu(), torch.from_numpy(hy))  # labels: exact integer hash
    # pixels: the same float32 operations; the device division may differ
    # from the host's in the last bit
    assert float((x.view(n, 784).cpu() - torch.from_numpy(hx)).abs().max()) < 1e-6
    counts = torch.bincount(y.cpu(), minlength=10)
    assert int(counts.min()) > n // 20
    x2, y2 = synthetic_mnist(n, DEV, seed=5, source="hash")
    assert torch.equal(x, x2) and torch.equal(y, y2)  # deterministic
