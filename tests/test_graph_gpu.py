"""HIP-graph execution modes of the fused trainer: the U-step unrolled
graph and the DDP step with its RCCL all-reduces captured inside the graph
(exercised at world size 1 so it runs on a one-GPU box)."""
import os
import socket

import pytest
from mp_util import collect
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("B,tol", [(4, 0.0), (1, 0.0), (64, 2e-3)])
def test_unrolled_graph_matches_single_steps(B, tol):
    """U-step graph replays walk the same trajectory as single steps.  When
    every fp32-atomic gradient address receives exactly one add the step is
    bitwise deterministic and the two must agree exactly: at B <= 6 there is
    one conv2-wgrad chunk per tile and every sample adds into its own conv1
    gradient replica.  At B=64 the atomics' arrival order varies run to run
    and a ReLU at the edge can flip, which amplifies last-bit differences
    chaotically over 21 steps; there the check is a loose trajectory check."""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    a = FusedMnistTrainer(dev, batch_size=B, dataset_size=B * 12, seed=2, unroll=8)
    b = FusedMnistTrainer(dev, batch_size=B, dataset_size=B * 12, seed=2, unroll=1)
    a.run(21)  # 2 unrolled replays + one closing 5-step replay
    for _ in range(21):
        b.step()
    torch.cuda.synchronize()
    assert a.steps_done == b.steps_done == 21
    assert int(a.batch_idx.item()) == int(b.batch_idx.item()) == 21 % 12
    if tol == 0.0:
        assert torch.equal(a.params, b.params)
        assert torch.equal(a.mom, b.mom)
    else:
        assert rel(a.params, b.params) < tol
        assert abs(a.last_loss() - b.last_loss()) < 1e-2


def _captured_ddp_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      PTO_CAPTURE_COMM="1")
    import torch.distributed as dist

    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    # B=4: one fp32-atomic add per gradient address, so neither trainer has
    # run-to-run noise (at B=64 the atomics' arrival order varies and 10
    # steps amplify last-bit differences to ~1e-5)
    ddp = FusedMnistTrainer(dev, batch_size=4, dataset_size=4 * 10, seed=3, force_ddp=True, unroll=4)
    assert ddp.graph_mode == "full"
    ref = FusedMnistTrainer(dev, batch_size=4, dataset_size=4 * 10, seed=3, graph="none")
    ddp.run(10)
    for _ in range(10):
        ref.step()
    torch.cuda.synchronize()
    q.put(rel(ddp.params, ref.params))
    dist.destroy_process_group()


def _capture_fail_worker(port, q):
    """First-run safety: RCCL refuses graph capture of its all-reduce (as an
    older RCCL or driver would).  The trainer falls back to split graphs
    (collective between two graphs), records it in comm_info, and trains on
    with the same numerics."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch.distributed as dist

    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    orig = FusedMnistTrainer._allreduce_update
    failed = []

    def refuse_capture(self):
        if torch.cuda.is_current_stream_capturing() and not failed:
            failed.append(1)
            raise RuntimeError("simulated: RCCL refused stream capture")
        return orig(self)

    FusedMnistTrainer._allreduce_update = refuse_capture
    ddp = FusedMnistTrainer(dev, batch_size=4, dataset_size=4 * 10, seed=3, force_ddp=True, unroll=4)
    ref = FusedMnistTrainer(dev, batch_size=4, dataset_size=4 * 10, seed=3, graph="none")
    ddp.run(10)
    for _ in range(10):
        ref.step()
    torch.cuda.synchronize()
    q.put((failed == [1], ddp.graph_mode, ddp.comm_info.get("graph_mode"), rel(ddp.params, ref.params)))
    dist.destroy_process_group()


def test_rccl_capture_failure_falls_back_to_split_graphs():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_capture_fail_worker, args=(port, q))
    p.start()
    refused, mode, info, err = collect(q, [p], 1)[0]
    p.join(60)
    assert p.exitcode == 0
    assert refused and mode == "split" and info == "split (capture failed)"
    assert err < 1e-5


def test_captured_rccl_allreduce_in_graph():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_captured_ddp_worker, args=(port, q))
    p.start()
    err = collect(q, [p], 1)[0]
    p.join(60)
    assert p.exitcode == 0
    assert err < 1e-5


@pytest.mark.parametrize("graph,unroll", [("none", 1), (None, 1), (None, 4)])
def test_fused_optimizer_schedule_matches_sgd_launch(graph, unroll):
    """The one-process schedule (no SGD launch: every update inside
    k_bwd_all, conv1's applied on the fly by the next step's F12 and
    committed by its F4dx) leaves the parameters, momentum and batch cursor
    of the DDP code path (grads-only backward + the multi-tensor SGD launch,
    force_ddp at world size 1) at every point the host can observe them
    (params / state_dict / evaluate), including an LR change and a
    checkpoint reload mid-run.  (Not bitwise: the schedules evaluate the
    same update in a different op order; a missed or doubled conv1 update
    would be off by ~lr*grad, orders of magnitude above the tolerance.)"""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    # B=4: one fp32-atomic add per gradient address (see the unroll test),
    # so neither schedule has run-to-run noise to amplify
    kw = dict(batch_size=4, dataset_size=4 * 9, seed=4, graph=graph, unroll=unroll, weight_decay=1e-4)
    a = FusedMnistTrainer(dev, **kw)
    b = FusedMnistTrainer(dev, force_ddp=True, **kw)
    assert a.schedule == "fused-opt" and b.schedule == "ddp-rccl"
    for t in (a, b):
        t.run(7)
    torch.cuda.synchronize()
    assert rel(a.params, b.params) < 1e-5
    assert rel(a.mom, b.mom) < 1e-4
    for name in a.p:
        assert rel(a.p[name], b.p[name]) < 1e-5, name
    assert int(a.batch_idx.item()) == int(b.batch_idx.item()) == 7 % 9
    for t in (a, b):
        t.set_lr(0.02)
        t.run(6)
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa["model"]:
        assert rel(sa["model"][k], sb["model"][k]) < 1e-5, k
        assert rel(sa["momentum"][k], sb["momentum"][k]) < 1e-4, k
    x = torch.randn(256, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (256,), device=dev)
    (la, aa), (lb, ab) = a.evaluate(x, y), b.evaluate(x, y)
    assert abs(la - lb) < 1e-4 and abs(aa - ab) <= 2 / 256
    # reload mid-run: both continue identically
    a.load_state_dict(sb)
    for t in (a, b):
        t.run(3)
    assert rel(a.params, b.params) < 1e-5
    assert abs(a.last_loss() - b.last_loss()) < 1e-4


@pytest.mark.parametrize("B,steps,unroll", [(4, 7, 4), (64, 45, 16)])
def test_xgmi_step_at_world_1_matches_sgd_launch(B, steps, unroll):
    """The multi-GPU xGMI step run in one process trains like the grads-only
    step + the multi-tensor SGD launch.  Overlapped schedule: step k's
    exchange (conv role: replica fold, one-shot all-reduce + SGD, publish,
    gradient zeroing; fc role) runs inside step k+1's F12 launch, whose conv
    blocks wait for the conv role and read its write-through parameters;
    the backward advances the cursor; every graph closes with the roles
    alone.  Runs of several graph sizes (run(7) = 4 + 2 + 1, run(45) = 32 +
    8 + 4 + 1)."""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    kw = dict(batch_size=B, dataset_size=B * 9, seed=8, unroll=unroll, weight_decay=1e-4, force_ddp=True)
    a = FusedMnistTrainer(dev, comm="xgmi", **kw)
    b = FusedMnistTrainer(dev, comm="rccl", **kw)
    assert a.schedule == "ddp-xgmi" and a.comm_info["correct"] and b.schedule == "ddp-rccl"
    assert a.overlap and a._inline  # world 1: the exchange inside the next F12
    for t in (a, b):
        t.run(steps)
    torch.cuda.synchronize()
    tol = 1e-5 if steps < 10 else 2e-4
    assert rel(a.params, b.params) < tol
    assert rel(a.mom, b.mom) < 10 * tol
    assert int(a.batch_idx.item()) == int(b.batch_idx.item()) == steps % 9
    assert int(a._xgmi.error_word()) == 0
    assert float(a.c1rep.abs().max()) == 0.0 and float(a.grads[a._split:].abs().max()) == 0.0


@pytest.mark.parametrize("B", [8, 64])
def test_bwd_all_matches_stock_pytorch(B):
    """The all-in-one backward launch (k_bwd_all: conv2.weight updated by the
    last-arriving wgrad chunk of each tile, dgrad from F12's weight
    snapshot, every other update in its producer's epilogue) walks the
    trajectory of stock PyTorch fp32 (nn.Conv2d/Linear + SGD momentum, same
    init and batches).  B=8: two wgrad chunks per tile, so the arrival
    counters and the atomic-exchange consume run; B=64: eleven."""
    from pytorch_operator_1_amd.models.mnist import param_offsets
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer
    from pytorch_operator_1_amd.train.runner import EagerMnistTrainer

    dev = torch.device("cuda", 0)
    a = FusedMnistTrainer(dev, batch_size=B, dataset_size=B * 9, seed=6, unroll=4, weight_decay=1e-4)
    ref = EagerMnistTrainer(dev, batch_size=B, dataset_size=B * 9, seed=6, weight_decay=1e-4)
    a.run(7)
    for _ in range(7):
        ref.step()
    torch.cuda.synchronize()
    for name, t in ref.model.state_dict().items():
        assert rel(a.p[name], t) < 2e-4, name
    assert abs(a.last_loss() - ref.last_loss()) < 1e-3
    assert int(a.batch_idx.item()) == 7 % 9
    assert int(a.c2_ctr.abs().sum().item()) == 0  # counters re-armed
    c2 = param_offsets()[0]["conv2.weight"][0]
    assert float(a.grads[c2:c2 + 25000].abs().max()) == 0.0  # consumed gradients re-zeroed


def test_deterministic_mode_b64_bitwise_and_resume(monkeypatch):
    """PTO_DETERMINISTIC=1: no floating-point atomics in k_bwd_all (conv2
    wgrad partial tiles summed in chunk order by the last arriver, conv1
    grads one replica per sample summed in replica order).  At B=64 two runs
    are bitwise identical, a checkpoint/resume in the middle reproduces the
    uninterrupted run bit for bit, and the trajectory matches the default
    (atomic) schedule within fp32 reordering noise."""
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    kw = dict(batch_size=64, dataset_size=64 * 9, seed=4, unroll=4)
    monkeypatch.setenv("PTO_DETERMINISTIC", "1")

    a = FusedMnistTrainer(dev, **kw)
    assert a.deterministic and a.c1_nrep == 64 and a.wpart is not None
    a.run(10)
    b = FusedMnistTrainer(dev, **kw)
    b.run(10)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params), "two deterministic runs differ"
    assert torch.equal(a.mom, b.mom)

    c = FusedMnistTrainer(dev, **kw)
    c.run(4)
    sd = c.state_dict()
    d = FusedMnistTrainer(dev, **kw)
    d.load_state_dict(sd)
    d.run(6)
    torch.cuda.synchronize()
    assert torch.equal(a.params, d.params), "resume from step 4 diverged from the uninterrupted run"
    assert int(a.c2_ctr.abs().sum().item()) == 0  # counters re-armed

    monkeypatch.setenv("PTO_DETERMINISTIC", "0")
    e = FusedMnistTrainer(dev, **kw)
    e.run(10)
    torch.cuda.synchronize()
    for name in a.p:
        assert rel(a.p[name], e.p[name]) < 2e-4, name
