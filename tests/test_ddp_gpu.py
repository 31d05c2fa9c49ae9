"""Data-parallel fused trainer on the GPU: 2 ranks share the box's one
MI355X.  RCCL refuses two ranks on one device, so the process group is
gloo: ``host-allreduce`` exercises the grads-only step + a host-side
all-reduce between split graphs (the RCCL schedule's structure, not RCCL
itself); ``xgmi`` / ``xgmi-det`` run the peer-memory all-reduce kernel with
its SGD epilogue inside the whole-step graph.  Checked against a
single-process stock-PyTorch reference that averages the two ranks'
gradients by hand."""
import os
import socket

import pytest
from mp_util import collect
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

STEPS = 4
N = 64 * 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, comm, steps=STEPS):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    # "-inline": every rank on its own CU partition of the shared GPU
    # (utils/cu_partition), so the trainer takes the schedule of one rank per
    # GPU -- the exchange roles inside the next step's F12 launch
    inline = comm.endswith("-inline")
    comm = comm[:-len("-inline")] if inline else comm
    if inline and world > 2:
        # 4+ processes stacked on one GPU: one pooled hardware queue each, or
        # the scheduler time-slices the oversubscribed queues (set before the
        # HIP runtime starts in this process; profiles/cu_partition_r6.md)
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    if comm == "xgmi-det":  # deterministic backward: per-sample conv1 replicas folded by the all-reduce
        comm = "xgmi"
        os.environ["PTO_DETERMINISTIC"] = "1"
    if comm == "host-allreduce":
        comm = "rccl"  # "not xGMI": with a gloo group the collective is gloo's host all-reduce
    if comm.startswith("xgmi-fenced"):
        os.environ["PTO_XGMI_PROTOCOL"] = "fenced"
        comm = "xgmi"
    race = comm == "auto-race"
    import torch.distributed as dist

    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer, build_fused_trainer

    verify_fail = comm == "xgmi-verify-fail"
    if verify_fail:
        # first-run safety on a new node: the xGMI kernel maps the peers but
        # returns wrong sums (here: it does nothing) -> autotune's check
        # against the host all-reduce fails on every rank -> every rank
        # falls back to the collective, and says so in comm_info
        from pytorch_operator_1_amd.parallel import xgmi

        xgmi.XgmiAllReduce.allreduce_ = lambda self, *a, **k: None
        comm = "auto"

    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if inline:
        from pytorch_operator_1_amd.utils import cu_partition

        part = cu_partition.activate_for_rank(rank, world, dev)
        assert part is not None and cu_partition.active(dev) is part
    pre = 0
    if race:
        # the schedule race of build_fused_trainer, deferred past the job's
        # first step: the verified xGMI steps vs the collective step from the
        # state that step left, every candidate rolled back afterwards, the
        # winner continuing from it
        tr = build_fused_trainer(dev, batch_size=64, dataset_size=N, seed=1, rank=rank, comm="auto")
        tr.run(1)  # the first optimizer step: eager launches, no race in front of it
        assert "schedule_autotune" not in tr.comm_info
        tr.prepare()  # the race (a second run()/step() would start it too), then capture
        pre = 1
        res = tr.comm_info["schedule_autotune"]
        cands = res["candidates"]
        assert res["correct"] and set(cands) == {"ddp-xgmi+overlap", "ddp-xgmi", "ddp-rccl"}, res
        for name in ("ddp-xgmi+overlap", "ddp-xgmi"):
            assert cands[name]["identical"] and cands[name]["param_rel_err"] < 1e-4, res
        assert all(c["step_us"] > 0 and c["spread_us"] >= 0 for c in cands.values()), res
        assert res["kept"] == tr.schedule + ("+overlap" if tr.overlap else ""), res
        assert tr.steps_done == 1 and int(tr.batch_idx.item()) == 1
        if inline:  # the overlapped candidate that raced was the inline form
            assert cands["ddp-xgmi+overlap"]["exchange"] == "inside the next F12 launch", res
            assert cands["ddp-xgmi+overlap"]["correct"], res
    else:
        tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=N, seed=1, rank=rank, comm=comm)
    if race:
        pass
    elif comm == "xgmi":
        assert tr.comm_info["transport"] == "xgmi" and tr.graph_mode == "full" and tr.schedule == "ddp-xgmi"
        assert tr._inline == inline and tr._xgmi.partitioned == inline and tr._xgmi.colocated != inline
        if inline:
            assert "next step's F12 launch" in tr.comm_info["overlap"], tr.comm_info
            assert tr.comm_info["cu_partition"]["parts"] == world, tr.comm_info
    else:
        assert tr.comm_info["transport"] == "host-allreduce (gloo)" and tr.graph_mode == "split"
        assert tr.schedule == "ddp-rccl"
    if verify_fail:
        assert tr.comm_info["correct"] is False and tr.comm_info["use_xgmi"] is False, tr.comm_info
    assert tr.comm_info["world_size"] == world
    if steps == STEPS:
        for _ in range(steps - pre):
            tr.step()
    else:
        tr.run(steps)  # the long run goes through the captured multi-step graphs
    torch.cuda.synchronize()
    assert int(tr.batch_idx.item()) == steps % (N // 64)
    assert float(tr.grads[tr._split:].abs().max()) == 0.0  # atomically accumulated range zeroed
    # conv1 gradient replicas: folded by the xGMI all-reduce before the
    # exchange, or all-reduced with the gradients and folded by the SGD
    # launch (host-allreduce / RCCL); zeroed either way
    assert tr.c1_nrep > 1
    assert float(tr.c1rep.abs().max()) == 0.0
    q.put((rank, tr.params.cpu()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["host-allreduce", "xgmi", "xgmi-fenced", "xgmi-det", "xgmi-verify-fail",
                                  "auto-race", "xgmi-inline", "auto-race-inline"])
def test_fused_ddp_two_ranks_matches_reference(comm):
    _run_and_compare(comm, STEPS, 1e-4)


@pytest.mark.parametrize("comm", ["host-allreduce", "xgmi", "xgmi-inline"])
def test_fused_ddp_two_ranks_200_steps(comm):
    """Long horizon: 200 steps of the 2-rank xGMI and
    host-allreduce schedules, replayed from the 32-step graphs, against the
    stock-PyTorch DDP-equivalent reference."""
    _run_and_compare(comm, 200, 2e-3)


@pytest.mark.parametrize("world", [4, 8])
def test_fused_ddp_inline_more_ranks(world):
    """The inline exchange (roles inside the next F12 launch) at world 4 and
    8, each rank on its own 1/world of the GPU's CUs, 40 steps through the
    captured graphs, against the stock-PyTorch reference."""
    _run_and_compare("xgmi-inline", 40, 1e-3, world=world)


def _run_and_compare(comm, steps, tol, world=2):
    """host-allreduce: grads-only step, gloo all-reduce between split graphs,
    SGD launch; xgmi: one peer-memory all-reduce of the whole buffer with the
    SGD epilogue inside the whole-step graph (no optimizer launch); xgmi-det:
    the same with the deterministic backward; xgmi-verify-fail: the kernel
    fails autotune's verification and every rank falls back to the host
    all-reduce; xgmi-fenced: the kernel's fenced visibility protocol;
    auto-race: build_fused_trainer races the two schedules first."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, comm, steps)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(collect(q, procs, world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert torch.equal(res[0], res[r]), f"ranks 0 and {r} diverged"

    from pytorch_operator_1_amd.models.mnist import MnistNet, param_offsets, synthetic_mnist

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    m = MnistNet().to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.5)
    data = [synthetic_mnist(N, dev, seed=1 + 1000 * r) for r in range(world)]
    for i in range(steps):
        bi = i % (N // 64)
        opt.zero_grad()
        grads = None
        for x, y in data:
            m.zero_grad()
            F.nll_loss(m(x[bi * 64:(bi + 1) * 64]), y[bi * 64:(bi + 1) * 64]).backward()
            g = [p.grad.clone() for p in m.parameters()]
            grads = g if grads is None else [a + b for a, b in zip(grads, g)]
        for p, g in zip(m.parameters(), grads):
            p.grad = g / world
        opt.step()
    offs, _ = param_offsets()
    flat = res[0]
    for name, t in m.state_dict().items():
        off, shape = offs[name]
        got = flat[off:off + t.numel()].view(shape)
        err = ((got - t.cpu()).abs().max() / t.abs().max()).item()
        assert err < tol, (name, err)


def _diverge_worker(rank, world, port, q, flip, inline=False):
    """Self-verifying multi-GPU run: every captured graph
    ends with a hash of the rank's parameters published into every rank's
    flag page; run() compares them.  ``flip``: after two clean chunks rank 1
    perturbs one parameter -- the next graph's hashes must differ and every
    rank must raise XgmiDivergence (retryable exit 138 in the trainer CLI)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist

        from pytorch_operator_1_amd.parallel.xgmi import XgmiDivergence
        from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer
        from pytorch_operator_1_amd.utils import dist as pdist

        dist.init_process_group("gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if inline:
            from pytorch_operator_1_amd.utils import cu_partition

            cu_partition.activate_for_rank(rank, world, dev)
        tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=N, seed=1, rank=rank, comm="xgmi", unroll=8)
        assert tr._hash and "consistency" in tr.comm_info
        assert tr._inline == inline
        for _ in range(2):
            tr.run(8)
        compared = tr._xgmi.hashes_compared
        detected = None
        if flip:
            if rank == 1:
                with torch.no_grad():
                    tr._params[1000] += 1e-3
            pdist.host_barrier(tag="flip")
            try:
                tr.run(8)  # its last graph hashed the perturbed parameters
            except XgmiDivergence as e:
                detected = str(e)
            pdist.host_barrier(tag="after")  # every rank's hash of that graph is published by now
            if detected is None:
                try:
                    tr.check_comm()
                except XgmiDivergence as e:
                    detected = str(e)
        else:
            tr.run(8, blocking_check=False)
            tr.run(8, blocking_check=False)
            pdist.host_barrier(tag="after")
            tr.check_comm()
        q.put((rank, compared, detected, tr._xgmi.hashes_compared))
        q.close()
        q.join_thread()  # the verdict is flushed to the parent before the hard exit
        os._exit(0)  # peers may still spin on a rank that raised; the test only needs the verdicts
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, 0))
        raise


@pytest.mark.parametrize("inline", [False, True])
@pytest.mark.parametrize("flip", [False, True])
def test_xgmi_ranks_self_verify_parameter_hash(flip, inline):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_diverge_worker, args=(r, 2, port, q, flip, inline)) for r in range(2)]
    for p in ps:
        p.start()
    res = collect(q, ps, 2, timeout=110)
    for p in ps:
        p.join(30)
    for rank, compared, detected, total in res:
        assert not isinstance(compared, str), compared
        assert compared > 0, (rank, compared)  # clean chunks: hashes of the same graphs compared, all equal
        if flip:
            assert detected and "diverged" in detected, (rank, detected)
        else:
            assert detected is None and total > compared, (rank, total)
