"""xGMI peer all-reduce protocol tests.  The box has ONE GPU, so W ranks
share it (separate processes, IPC-mapped buffers, gloo for the handle
exchange): the barrier/visibility protocol is the same as across GPUs.
Checked: exact sums over many back-to-back calls with changing data, two
channels in flight on two streams, HIP-graph capture + replay, identical
results on every rank."""
import os
import socket

import pytest
from mp_util import collect
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _expected(n, world, it, dev):
    tot = torch.zeros(n, device=dev)
    for r in range(world):
        g = torch.Generator(device=dev).manual_seed(1000 * it + r)
        tot += torch.randn(n, generator=g, device=dev)
    return tot


def _fill(buf, rank, it):
    g = torch.Generator(device=buf.device).manual_seed(1000 * it + rank)
    buf.copy_(torch.randn(buf.shape, generator=g, device=buf.device))


def _worker(rank, world, port, q, protocol="coherent"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n = 431_296  # MNIST flat gradient size (param_offsets, 64-aligned)
        split = 405_632  # fc bucket | conv bucket boundary
        buf = torch.zeros(n, device=dev)
        ar = XgmiAllReduce(buf, protocol=protocol)
        worst = 0.0
        side = torch.cuda.Stream(dev)
        for it in range(12):
            _fill(buf, rank, it)
            if it % 2 == 0:
                ar.allreduce_(0, n)
            else:  # two channels concurrently: bucket 0 on a side stream
                side.wait_stream(torch.cuda.current_stream(dev))
                ar.allreduce_(0, split, chan=0, stream=side)
                ar.allreduce_(split, n - split, chan=1)
                torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            worst = max(worst, (buf - _expected(n, world, it, dev)).abs().max().item())
        ar.check()
        # graph capture + replay (pointers fixed, epochs advance on device)
        _fill(buf, rank, 99)
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            ar.allreduce_(0, n)  # warm on the capture stream
        torch.cuda.synchronize(dev)
        _fill(buf, rank, 99)
        dist.barrier()
        with torch.cuda.graph(g):
            ar.allreduce_(0, n)
        for it in range(100, 104):
            _fill(buf, rank, it)
            torch.cuda.synchronize(dev)
            g.replay()
            torch.cuda.synchronize(dev)
            worst = max(worst, (buf - _expected(n, world, it, dev)).abs().max().item())
        ar.check()
        # identical on every rank
        chk = buf.cpu()
        allv = [None] * world
        dist.all_gather_object(allv, chk)
        same = all(torch.equal(allv[0], v) for v in allv)
        tune = ar.autotune([(0, split), (split, n - split)], iters=10)
        ar.close()
        dist.destroy_process_group()
        q.put((rank, worst, same, tune))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False, None))
        raise


@pytest.mark.parametrize("world,protocol", [(2, "coherent"), (4, "coherent"), (2, "fenced")])
def test_xgmi_allreduce_exact(world, protocol):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, protocol)) for r in range(world)]
    for p in ps:
        p.start()
    res = collect(q, ps, world, timeout=110)
    for p in ps:
        p.join(60)
    for rank, worst, same, tune in res:
        assert not isinstance(worst, str), worst
        assert worst < 1e-4, (rank, worst)
        assert same
        assert tune["correct"] and tune["protocol"] == protocol, tune
    print("autotune", res[0][3])
    for p in ps:
        assert p.exitcode == 0


def _sgd_worker(rank, world, port, q):
    """All-reduce + SGD epilogue vs (sum of the ranks' grads, scaled) fed to
    the same SGD formula in torch; two buckets on two streams, weight decay,
    nesterov, device LR, zero range and batch cursor; graph replay."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n, split = 431_296, 405_632
        lr, mom, wd = 0.05, 0.9, 1e-3
        buf = torch.zeros(n, device=dev)
        ar = XgmiAllReduce(buf)
        g0 = torch.Generator(device=dev).manual_seed(7)
        p = torch.randn(n, generator=g0, device=dev)  # same start on every rank
        m = torch.zeros(n, device=dev)
        pr, mr = p.clone(), m.clone()
        lr_dev = torch.tensor([lr], device=dev)
        cursor = torch.zeros(1, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(dev)

        def step():
            kw = dict(params=p, mom=m, lr_dev=lr_dev, momentum=mom, weight_decay=wd, gscale=1.0 / world,
                      nesterov=True, zero_from=split)
            side.wait_stream(torch.cuda.current_stream(dev))
            ar.allreduce_sgd_(0, split, chan=0, stream=side, **kw)
            ar.allreduce_sgd_(split, n - split, chan=1, cursor=cursor, n_batches=5, **kw)
            torch.cuda.current_stream(dev).wait_stream(side)

        def ref(it):
            d = _expected(n, world, it, dev) / world + wd * pr
            mr.mul_(mom).add_(d)
            pr.sub_(lr * (d + mom * mr))

        worst, zero_ok = 0.0, True
        for it in range(6):
            _fill(buf, rank, it)
            step()
            torch.cuda.synchronize(dev)
            ref(it)
            worst = max(worst, (p - pr).abs().max().item(), (m - mr).abs().max().item())
            zero_ok &= float(buf[split:].abs().max()) == 0.0
        # graph capture + replay
        _fill(buf, rank, 50)
        s = torch.cuda.Stream(dev)
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step()
        torch.cuda.synchronize(dev)
        for it in range(60, 63):
            _fill(buf, rank, it)
            torch.cuda.synchronize(dev)
            g.replay()
            torch.cuda.synchronize(dev)
            ref(it)
            worst = max(worst, (p - pr).abs().max().item(), (m - mr).abs().max().item())
        ar.check()
        allv = [None] * world
        dist.all_gather_object(allv, p.cpu())
        same = all(torch.equal(allv[0], v) for v in allv)
        cur = int(cursor.item())
        ar.close()
        dist.destroy_process_group()
        q.put((rank, worst, same and zero_ok, cur))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False, None))
        raise


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_sgd_epilogue(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_sgd_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = collect(q, ps, world, timeout=110)
    for p in ps:
        p.join(60)
    for rank, worst, ok, cur in res:
        assert not isinstance(worst, str), worst
        assert worst < 1e-4, (rank, worst)
        assert ok
        assert cur == 9 % 5  # 6 eager + 3 replayed steps (the capture itself does not run)
    for p in ps:
        assert p.exitcode == 0


def _stall_worker(rank, world, port, q):
    """Rank 1 stalls on the host for 5 timeouts before its all-reduce:
    rank 0's first barrier times out, every later launch returns at once,
    and NO parameter, momentum or gradient is written on either rank."""
    try:
        import time

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce, XgmiTimeout

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n, split = 431_296, 405_632
        buf = torch.zeros(n, device=dev)
        ar = XgmiAllReduce(buf, timeout_ms=300)
        p = torch.randn(n, device=dev)
        m = torch.randn(n, device=dev)
        lr_dev = torch.tensor([0.1], device=dev)
        kw = dict(params=p, mom=m, lr_dev=lr_dev, momentum=0.5, weight_decay=0.0, gscale=0.5, nesterov=False,
                  zero_from=split)
        _fill(buf, rank, 1)
        ar.allreduce_sgd_(0, n, **kw)  # one healthy step first
        torch.cuda.synchronize(dev)
        ar.check()
        ar.poll()  # non-blocking check: captures the (clean) word for the next poll
        _fill(buf, rank, 2)
        snap = [t.clone() for t in (p, m, buf)]
        dist.barrier()
        t0 = time.perf_counter()
        if rank == 1:
            time.sleep(1.5)
        for _ in range(4):
            ar.allreduce_sgd_(0, split, chan=0, **kw)
            ar.allreduce_sgd_(split, n - split, chan=1, **kw)
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        unchanged = all(torch.equal(a, b) for a, b in zip((p, m, buf), snap))
        try:
            ar.check()
            raised = False
        except XgmiTimeout:
            raised = True
        # once failed, a launch returns without waiting
        t1 = time.perf_counter()
        ar.allreduce_sgd_(0, n, **kw)
        torch.cuda.synchronize(dev)
        after = time.perf_counter() - t1
        # poll() reports the word captured by the PREVIOUS poll: clean, then the failure
        polls = []
        for _ in range(2):
            try:
                ar.poll()
                polls.append("ok")
            except XgmiTimeout:
                polls.append("raise")
        q.put((rank, elapsed, unchanged, raised, after, polls))
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False, False, None, None))
        raise


def test_xgmi_timeout_fails_fast_without_updates():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_stall_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(collect(q, ps, 2, timeout=110))
    for p in ps:
        p.join(60)
    for rank, elapsed, unchanged, raised, after, polls in res:
        assert not isinstance(elapsed, str), elapsed
        assert raised, (rank, "error word not set")
        assert polls == ["ok", "raise"], (rank, polls)
        assert unchanged, (rank, "params/momentum/grads written by a failed all-reduce")
        assert after < 0.1, (rank, after)
    # rank 0: one 300 ms timeout for 8 launches, not one per barrier
    assert res[0][1] < 1.2, res[0]


@pytest.mark.parametrize("partitioned", [False, True])
def test_trainer_exits_retryable_when_xgmi_peer_killed(tmp_path, partitioned):
    """Two fused-trainer ranks on the one GPU (gloo for rendezvous, xGMI
    kernel for the gradients); rank 1 SIGKILLs itself at step 100.  Rank 0
    must exit 138 (retryable) within 5 s of the kill.  ``partitioned``: each
    rank on its own CU partition (utils/cu_partition.py), so the ranks run
    the schedule of one rank per GPU -- the exchange as roles INSIDE the next
    step's F12 launch, whose conv workgroups wait on those roles -- and the
    dead peer must surface through that in-launch wait's bounded spin."""
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PTO_XGMI_TIMEOUT_MS="500", PYTHONPATH=root)
        if partitioned:
            env.update(PTO_CU_PARTITION="1", LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2")
        cmd = [sys.executable, "-m", "pytorch_operator_1_amd.train.mnist", "--backend", "gloo", "--impl", "fused",
               "--comm", "xgmi", "--max-steps", "2000", "--log-interval", "50", "--no-test", "--train-size", "8192",
               "--fail-at-step", "100", "--fail-rank", "1", "--dir", ""]
        procs.append(subprocess.Popen(cmd, env=env, cwd=str(tmp_path), stdout=open(tmp_path / f"r{r}.log", "w"),
                                      stderr=subprocess.STDOUT))
    t_kill = None
    end = time.time() + 200
    while time.time() < end:
        if t_kill is None and procs[1].poll() is not None:
            t_kill = time.time()
        if procs[0].poll() is not None and t_kill is not None:
            break
        time.sleep(0.02)
    t_exit = time.time()
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()
    log0 = (tmp_path / "r0.log").read_text()
    log1 = (tmp_path / "r1.log").read_text()
    assert procs[1].returncode == -9, "rank 1:\n" + log1[-2000:] + "\nrank 0:\n" + log0[-2000:]
    assert procs[0].returncode == 138, log0[-3000:]
    assert "timed out" in log0
    assert t_kill is not None and t_exit - t_kill < 5.0, (t_exit - t_kill, log0[-2000:])
    if partitioned:  # the run took the one-rank-per-GPU (inline) schedule
        assert "next step's F12 launch" in log0 and "'partitioned': True" in log0, log0[-3000:]


def _bucket_worker(rank, world, port, q, dtype_name):
    """GradBucketer's xGMI comm hook: a small Llama in
    bf16 (or fp32), several buckets, every bucket forced onto the peer
    kernel (comm="xgmi"), launched from the backward hooks on the comm
    stream; summed gradients checked against both ranks' own gradients
    summed by hand in fp32."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.models.llama import Llama, LlamaConfig, synthetic_tokens
        from pytorch_operator_1_amd.parallel.ddp import GradBucketer

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dt = getattr(torch, dtype_name)
        cfg = LlamaConfig(dim=128, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=256, ffn_dim=256)
        torch.manual_seed(0)
        m = Llama(cfg, impl="torch", dtype=dt).to(dev)
        bk = GradBucketer(m, bucket_mb=0.1, comm="xgmi")
        assert bk.comm_info["transport"] == "xgmi+rccl", bk.comm_info
        assert len(bk.buckets) >= 3 and all(b["transport"] == "xgmi" for b in bk.buckets)
        worst = 0.0
        for it in range(3):
            tok, lab = synthetic_tokens(2, 16, cfg.vocab_size, dev, seed=100 * it + rank)
            m(tok, lab).backward()
            bk.finish()
            mine = {n: p.grad.float().clone() for n, p in m.named_parameters()}
            ref = Llama(cfg, impl="torch", dtype=dt).to(dev)
            ref.load_state_dict(m.state_dict())
            total = None
            for r in range(world):
                ref.zero_grad()
                t, lb = synthetic_tokens(2, 16, cfg.vocab_size, dev, seed=100 * it + r)
                ref(t, lb).backward()
                g = {n: p.grad.float().clone() for n, p in ref.named_parameters()}
                total = g if total is None else {n: total[n] + g[n] for n in g}
            for n in total:
                worst = max(worst, ((mine[n] - total[n]).abs().max() / total[n].abs().max().clamp_min(1e-6)).item())
            bk.release()
        torch.cuda.synchronize(dev)
        bk.remove()
        dist.destroy_process_group()
        q.put((rank, worst))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("dtype_name", ["bfloat16", "float32"])
def test_grad_bucketer_xgmi_hook(dtype_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q, dtype_name)) for r in range(2)]
    for p in ps:
        p.start()
    res = collect(q, ps, 2, timeout=110)
    for p in ps:
        p.join(60)
    tol = 3e-2 if dtype_name == "bfloat16" else 1e-4
    for rank, worst in res:
        assert not isinstance(worst, str), worst
        assert worst < tol, (rank, worst)
    for p in ps:
        assert p.exitcode == 0


def _uneven_worker(rank, world, port, q):
    """MI355X_MICROARCH "test every hand-off under UNEVEN load": each call is
    preceded by a random host delay (0-3 ms, different per rank) and a
    matmul on a side stream that competes for the CUs while the kernel's
    barriers spin; the output buffer is read (cache-warm) before being
    refilled.  Every word of every call is checked against the exact sum."""
    try:
        import random
        import time

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n = 431_296
        buf = torch.zeros(n, device=dev)
        ar = XgmiAllReduce(buf, timeout_ms=5000)
        side = torch.cuda.Stream(dev)
        a = torch.randn(2048, 2048, device=dev)
        rng = random.Random(rank)
        worst, bad_calls = 0.0, 0
        for it in range(40):
            float(buf[:4096].sum())  # read the previous result's lines first
            _fill(buf, rank, 500 + it)
            with torch.cuda.stream(side):
                for _ in range(rng.randint(0, 3)):
                    a = a @ a * 1e-3
            time.sleep(rng.random() * 0.003)
            ar.allreduce_(0, n, chan=it % 2)
            torch.cuda.synchronize(dev)
            err = (buf - _expected(n, world, 500 + it, dev)).abs().max().item()
            worst = max(worst, err)
            bad_calls += err > 1e-4
        ar.check()
        ar.close()
        dist.destroy_process_group()
        q.put((rank, worst, bad_calls))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None))
        raise


def test_xgmi_allreduce_uneven_load():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_uneven_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = collect(q, ps, 2, timeout=110)
    for p in ps:
        p.join(60)
    for rank, worst, bad in res:
        assert not isinstance(worst, str), worst
        assert bad == 0 and worst < 1e-4, (rank, worst, bad)
    for p in ps:
        assert p.exitcode == 0


def _overlap_pair_worker(rank, world, port, q):
    """The overlapped MNIST step's exchange at any world size: the one-shot
    rank-split conv role (channel 2: every rank's gradient AND replicas
    read from the registered buffer and summed, all-reduce + SGD, parameter
    written through, one publish per workgroup, gradient and replicas
    zeroed after its second barrier) and the rank-split fc role
    (channel 1, barrier 0 of its own).  Even ranks run both roles as ONE
    launch (the MNIST forward launch with no conv blocks, as a run's
    closing exchange), odd ranks as two stand-alone launches: the
    decompositions must pair block by block.  Parameters and momentum vs the
    same SGD in torch on the exact sum (folded replicas included), every
    rank bit-identical, gradients and replicas zero after every exchange,
    the publish counter = role workgroups per call."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from pytorch_operator_1_amd.ops import _lib
        from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        nfc, nconv = 81_920, 25_664  # fc range > the one-shot limit, conv range = MNIST's
        n = nfc + nconv
        stride, nrep = 576, 4  # replicated tail (MNIST: conv1, 8 replicas)
        rep_from = n - stride
        lr, mom, wd = 0.05, 0.9, 1e-3
        full = torch.zeros(n + (nrep - 1) * stride, device=dev)  # gradients + replicas, registered together
        buf, rep = full[:n], full[n:]
        ready = torch.zeros(1, dtype=torch.int32, device=dev)
        ar = XgmiAllReduce(full, timeout_ms=20000)
        p = torch.randn(n, generator=torch.Generator(device=dev).manual_seed(7), device=dev)
        m = torch.zeros(n, device=dev)
        pr, mr = p.clone(), m.clone()
        lr_dev = torch.tensor([lr], device=dev)
        L = _lib.lib()
        s = torch.cuda.current_stream(dev).cuda_stream
        cnb = L.pto_ar_oneshot_role_blocks(nconv, world)
        worst, zero_ok, ready_ok = 0.0, True, True
        for it in range(8):
            _fill(buf, rank, 700 + it)
            g = torch.Generator(device=dev).manual_seed(9000 + 31 * it + rank)
            rep.copy_(torch.randn(rep.shape, generator=g, device=dev))
            mine = buf.clone()
            for r in range(nrep - 1):
                mine[rep_from:] += rep[r * stride:(r + 1) * stride]
            tot = mine.cpu()
            dist.all_reduce(tot)  # the exact sum over ranks (gloo, fp32)
            ready.zero_()
            upd = ar.update_args(p, m, lr_dev, mom, wd, 1.0 / world, True)
            if rank % 2 == 0:
                _lib.check(L.pto_conv12_fwd_ar(*([None] * 9), 0, None, None, *ar.exchange_args(), *upd,
                                               0, nfc, 1, n, nfc, nconv, 2, n, nrep, stride, rep_from,
                                               ready.data_ptr(), s), "conv12_fwd_ar(B=0)")
            else:
                _lib.check(L.pto_ar_oneshot_role_sgd(*ar.role_args(nfc, nconv, 2, p, m, lr_dev, mom, wd,
                                                                   1.0 / world, True, n)[:-1],
                                                     n, nrep, stride, rep_from, ready.data_ptr(), s),
                           "ar_oneshot_role_sgd")
                _lib.check(L.pto_ar_role_sgd(*ar.role_args(0, nfc, 1, p, m, lr_dev, mom, wd, 1.0 / world, True, n),
                                             s), "ar_role_sgd")
            torch.cuda.synchronize(dev)
            d = tot.to(dev) / world + wd * pr
            mr.mul_(mom).add_(d)
            pr.sub_(lr * (d + mom * mr))
            worst = max(worst, (p - pr).abs().max().item(), (m - mr).abs().max().item())
            zero_ok &= float(buf[nfc:].abs().max()) == 0.0 and float(rep.abs().max()) == 0.0
            ready_ok &= int(ready.item()) == cnb
        ar.check()
        allv = [None] * world
        dist.all_gather_object(allv, p.cpu())
        same = all(torch.equal(allv[0], v) for v in allv)
        ar.close()
        dist.destroy_process_group()
        q.put((rank, worst, same, zero_ok and ready_ok))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False, False))
        raise


@pytest.mark.parametrize("world", [2, 3, 8])
def test_xgmi_overlap_pair_any_world(world):
    """World sizes 2, 3 (S = 341, idle threads in every role workgroup) and
    8 (the node's full world, 8 rank groups of 128 threads)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_overlap_pair_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = collect(q, ps, world, timeout=110)
    for p in ps:
        p.join(60)
    for rank, worst, same, zero_ok in res:
        assert not isinstance(worst, str), worst
        assert worst < 1e-4, (rank, worst)
        assert same and zero_ok, (rank, same, zero_ok)
    for p in ps:
        assert p.exitcode == 0
