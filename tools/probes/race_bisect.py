"""Bisect the 2-rank (shared GPU) schedule-race failure of round 5: which
ingredient of build_fused_trainer's race makes the overlapped xGMI
trainer's run(8) time out.  Usage: python tools/probes/race_bisect.py MODE
MODE: alone | plain | twin | both | twinrun"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=512, seed=1, rank=rank, comm="xgmi")
        data = dict(data=tr.data.view(-1, 784), target=tr.target.view(-1))
        extra = []
        if mode in ("plain", "both"):
            extra.append(FusedMnistTrainer(dev, batch_size=64, dataset_size=512, seed=1, rank=rank, comm="xgmi",
                                           overlap=False, **data))
        if mode in ("twin", "both", "twinrun"):
            extra.append(FusedMnistTrainer(dev, batch_size=64, dataset_size=512, seed=1, rank=rank, comm="rccl",
                                           **data))
        if mode == "twinrun":
            extra[-1].run(8)
            torch.cuda.synchronize()
        tr._align_ranks("go")
        tr.run(8)
        torch.cuda.synchronize()
        q.put((rank, "ok", int(tr._xgmi.error_word()), None))
    except Exception as e:  # noqa: BLE001
        import ctypes

        x = tr._xgmi
        ep = x.epochs.cpu().tolist()
        hip = ctypes.CDLL("libamdhip64.so")
        words = x.epochs.numel() * 2 * 8  # AR_CHANNELS * 2 phases * 256 blocks * 8 ranks
        buf = (ctypes.c_uint32 * words)()
        hip.hipMemcpy(buf, ctypes.c_void_p(x._flags), ctypes.c_size_t(words * 4), 2)

        def fl(chan, phase, blk, src):
            return buf[((chan * 2 + phase) * 256 + blk) * 8 + src]

        info = {"ep_c1": ep[256:256 + 4] + ["..."] + ep[256 + 96:256 + 102], "ep_c2": ep[512:512 + 14],
                "ready": int(tr._ready.item()),
                "f_c2_p0": [(b, fl(2, 0, b, 0), fl(2, 0, b, 1)) for b in range(13)],
                "f_c2_p1": [(b, fl(2, 1, b, 0), fl(2, 1, b, 1)) for b in range(13)],
                "f_c1_p0": [(b, fl(1, 0, b, 0), fl(1, 0, b, 1)) for b in (0, 1, 50, 99)],
                "f_c1_p1": [(b, fl(1, 1, b, 0), fl(1, 1, b, 1)) for b in (0, 1, 50, 99)]}
        q.put((rank, repr(e)[:120], int(tr._xgmi.err.item()), info))
    dist.destroy_process_group()


if __name__ == "__main__":
    mode = sys.argv[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    for o in sorted(out, key=lambda t: t[0]):
        print(mode, o, flush=True)
