"""The production MNIST training step: hand-written gfx950 kernels, flat
buffers, HIP-graph replay.

Behavioural parity: one call of :meth:`FusedMnistTrainer.step` does what one
iteration of the reference loop does (``examples/mnist/mnist.py:37-43``):
``zero_grad`` → forward → ``nll_loss(log_softmax)`` → ``backward`` (DDP mean
all-reduce) → ``SGD(lr, momentum).step()`` — in fp32, with PyTorch's
initialisation, loss, and update semantics (numerics checked against the
stock-PyTorch trainer in tests/test_kernels_gpu.py and tests/test_graph_gpu.py).

MI355X design:
  * parameters, gradients and momentum each live in ONE flat fp32 buffer
    (431,296 elements incl. 256-B alignment padding).  The DDP gradient
    all-reduce is therefore a single 1.7 MB message (one RCCL call, or the
    xGMI one-shot kernel from :mod:`pytorch_operator_1_amd.parallel.xgmi`),
    and the optimizer is a single fused launch that also zeroes the grads
    (so atomically accumulated grads start from zero next step).
  * every op is a kernel from ``csrc/kernels/mnist_kernels.hip``; activations
    stay resident in HBM.  Four launches per step: F12 (conv1+conv2
    forward), fc1, F4dx (fc2 + loss + d(a2p)) and ``k_bwd_all`` (the whole
    backward).  Single process: every parameter update runs inside those
    launches (``fused_opt``: ``k_bwd_all`` updates fc/conv2 -- conv2.weight
    by the last-arriving wgrad chunk of each tile -- and conv1's update is
    applied on the fly by the next step's F12 and committed by its F4dx).
    DDP: ``k_bwd_all`` in grads-only mode, then one all-reduce of the flat
    buffer whose epilogue is the SGD update (xGMI) or the all-reduce + one
    multi-tensor SGD launch (RCCL).
  * steps are captured into HIP graphs and replayed (``run(n)``: the
    largest multi-step graphs first, one replay per 32 steps + one); the
    batch index is a device counter advanced inside the graph, so replays
    walk the dataset like the eager loop does.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from ..models.mnist import PARAM_SHAPES, MnistNet, param_offsets, synthetic_mnist
from ..ops import _lib


class FusedMnistTrainer:
    def __init__(self, device, batch_size=64, lr=0.01, momentum=0.5, dataset_size=60000, seed=1, rank=0,
                 weight_decay=0.0, nesterov=False, graph: str | None = None, comm: str | None = None,
                 data=None, target=None, unroll: int | None = None, force_ddp: bool = False,
                 fused_opt: bool | None = None):
        assert device.type == "cuda", "FusedMnistTrainer runs on a HIP device"
        import os

        self.L = _lib.lib()
        self.device = device
        self.B = int(batch_size)
        self.lr = float(lr)
        self.momentum = float(momentum)
        self.weight_decay = float(weight_decay)
        self.nesterov = bool(nesterov)
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        # DDP code path (bucketed, overlapped all-reduce); forced for tests
        # of the collective path at world size 1
        self.ddp = self.world > 1 or force_ddp
        # steps per graph replay in run(): amortises the host launch gap
        self.unroll = int(unroll if unroll is not None else os.environ.get("PTO_GRAPH_UNROLL", "32"))
        # gradient all-reduce transport: "rccl", "xgmi" (peer-memory kernel,
        # parallel/xgmi.py) or "auto" (xGMI if it verifies and beats RCCL on
        # these buckets, measured at startup; same choice on every rank)
        self.comm = comm or os.environ.get("PTO_COMM", "auto")

        offs, total = param_offsets()
        self.numel = total
        f32 = dict(device=device, dtype=torch.float32)
        self._params = torch.zeros(total, **f32)
        self.grads = torch.zeros(total, **f32)
        self.mom = torch.zeros(total, **f32)
        self._p, self.g = {}, {}
        for name, (off, shape) in offs.items():
            n = math.prod(shape)
            self._p[name] = self._params[off:off + n].view(shape)
            self.g[name] = self.grads[off:off + n].view(shape)
        # Same init as the stock module under the same seed.
        torch.manual_seed(seed)
        ref = MnistNet()
        with torch.no_grad():
            for name, t in ref.state_dict().items():
                self._p[name].copy_(t.to(device))
        if self.world > 1:
            dist.broadcast(self._params, 0)  # DDP's ctor broadcast (COL1)

        B = self.B
        self.a1p = torch.empty(B * 2880, **f32)
        self.code1 = torch.empty(B * 2880, device=device, dtype=torch.uint8)
        self.a2p = torch.empty(B * 800, **f32)
        self.code2 = torch.empty(B * 800, device=device, dtype=torch.uint8)
        self.h1 = torch.empty(B * 500, **f32)
        self.loss_rows = torch.zeros(B, **f32)
        self.dlogits = torch.empty(B * 10, **f32)
        self.dh1 = torch.empty(B * 500, **f32)
        self.da2p = torch.empty(B * 800, **f32)
        self.da1p = torch.empty(B * 2880, **f32)

        if data is None:
            data, target = synthetic_mnist(dataset_size, device, seed=seed + 1000 * rank)
        self.n_batches = data.shape[0] // B
        self.data = data[: self.n_batches * B].reshape(self.n_batches, B * 784).contiguous()
        self.target = target[: self.n_batches * B].reshape(self.n_batches, B).contiguous()
        # device-side batch cursor: read by conv1 fwd/bwd and fc2_ce, advanced
        # by the optimizer launch (no per-step copy kernels, graph-safe)
        self.batch_idx = torch.zeros(1, device=device, dtype=torch.int64)
        # fused fc1+fc2/CE launch (PTO_FUSE_FC=0: the two-launch path) and its
        # per-16-row arrival counters (re-armed by the kernel itself)
        self.fuse_fc = os.environ.get("PTO_FUSE_FC", "0") == "1"  # measured: 1.06M vs 1.11M samples/s unfused
        self.fc_counters = torch.zeros(max(1, (self.B + 15) // 16), device=device, dtype=torch.int32)
        # Fused-optimizer schedule (no gradient all-reduce between backward and
        # the update, i.e. world size 1): no SGD launch; fc/conv2 are updated by
        # extra blocks of the conv1-backward launch, conv1's update is applied
        # on the fly by the next step's first launch and committed by its fc2
        # launch (mnist_kernels.hip, "Fused optimizer").  PTO_FUSED_OPT=0: the
        # separate multi-tensor SGD launch.
        if fused_opt is None:
            fused_opt = os.environ.get("PTO_FUSED_OPT", "1") == "1"
        self.fused_opt = bool(fused_opt) and not self.ddp and not self.fuse_fc
        self.pending = torch.zeros(1, device=device, dtype=torch.int32)  # conv1 update owed
        self.batch_snap = torch.zeros(1, device=device, dtype=torch.int64)  # cursor seen by this step's B1
        self._noops = int(os.environ.get("PTO_PROBE_NOOPS", "0"))
        self._probe_fork = torch.cuda.Stream(device) if os.environ.get("PTO_PROBE_FORK") == "1" else None
        self.conv12_version = int(os.environ.get("PTO_CONV12", "2"))  # 2: 512-thread F1+F2 launch
        # xGMI DDP step: SGD applied by the all-reduce kernels' epilogue
        self.ar_fused_sgd = os.environ.get("PTO_AR_FUSED_SGD", "1") == "1"
        # two-stream backward for the fused-optimizer schedule (PTO_SPLIT_BWD=1).
        # Off: a fork/join inside the replayed graph costs ~19 us on MI355X
        # (profiles/graph_fork_join_probe_r1.md), more than the overlap wins
        # (89.8 vs 54.5 us/step measured)
        self._bwd_side = (torch.cuda.Stream(device)
                          if self.fused_opt and os.environ.get("PTO_SPLIT_BWD", "0") == "1" else None)
        # fc1's weight gradient computed in B1 and consumed there by the SGD
        # epilogue (never stored), instead of stored by B3 and re-read by B1's
        # SGD blocks (PTO_DW1_SGD=0: the B3 path).  The fc1.weight slot of the
        # gradient buffer is then not maintained.
        self.dw1_sgd = (self.fused_opt and self._bwd_side is None
                        and os.environ.get("PTO_DW1_SGD", "1") == "1")
        # F1 copies the batch's images out for B1 (PTO_XCUR=0: B1 re-reads
        # them through the batch cursor)
        self.xcur = (torch.empty(self.B * 784, device=device)
                     if self.dw1_sgd and self.conv12_version == 2 and os.environ.get("PTO_XCUR", "1") == "1"
                     else None)
        # F4 and B3's d(a2p) in one launch (k_fc2_ce_dx), B3's all-row
        # reductions in B2, the batch-cursor advance in B1: 5 launches per
        # step (PTO_F4DX=0: the 6-launch schedule)
        self.merge_f4 = self.xcur is not None and os.environ.get("PTO_F4DX", "1") == "1"
        # the whole backward + optimizer as ONE launch (k_bwd_all): 4 launches
        # per step; conv2.weight is updated by the last-arriving wgrad chunk
        # of each tile, the dgrad blocks read F12's snapshot of it
        # (PTO_BWD_ALL=0: conv2 backward and B1 as two launches)
        self.bwd_all = self.merge_f4 and os.environ.get("PTO_BWD_ALL", "1") == "1"
        self.w2f = torch.empty(50 * 500, device=device) if self.bwd_all else None
        self.c2_ctr = torch.zeros(32, device=device, dtype=torch.int32) if self.bwd_all else None
        # deterministic mode (PTO_DETERMINISTIC=1): no floating-point atomics
        # in the backward -- conv2 wgrad chunks store partial tiles summed in
        # chunk order by the last arriver, conv1 grads one replica per
        # sample summed in replica order -- so B=64 steps are bitwise
        # reproducible run to run and across a checkpoint/resume
        self.deterministic = os.environ.get("PTO_DETERMINISTIC", "0") == "1"
        # multi-GPU step: the same single backward launch in grads-only mode
        # (every gradient into the flat buffer, no parameter touched) after
        # F12 / fc1 / F4dx -> 4 launches + the all-reduce (whose SGD
        # epilogue updates) instead of 6 (PTO_DDP_BWD_ALL=0: the old split)
        self.ddp_bwd_all = self.ddp and not self.fuse_fc and os.environ.get("PTO_DDP_BWD_ALL", "1") == "1"
        # conv1 gradient replicas of k_bwd_all (sample b adds into replica
        # b % R: B/R same-address atomics instead of B); summed by the lazy
        # apply and the commit (single GPU) or folded by the xGMI all-reduce
        # before its exchange (multi-GPU; RCCL: 1 replica, see ddp_nrep)
        self.c1_nrep = (min(16, max(1, int(os.environ.get("PTO_C1_REPLICAS", "8"))))
                        if (self.bwd_all or self.ddp_bwd_all) else 1)
        self.wpart = None
        if self.deterministic:
            if not (self.bwd_all or self.ddp_bwd_all) or self.B > 256:
                raise RuntimeError("PTO_DETERMINISTIC=1 needs the k_bwd_all schedule and batch <= 256")
            self.c1_nrep = self.B
            self.wpart = torch.empty(((self.B + 3) // 4) * 50 * 500, device=device)  # >= chunks x conv2.weight
            if self.c2_ctr is None:
                self.c2_ctr = torch.zeros(32, device=device, dtype=torch.int32)
        self.c1_stride = self.numel - offs["conv1.weight"][0]
        self.c1rep = torch.zeros(max(1, self.c1_nrep - 1) * self.c1_stride, **f32)
        self.ddp_nrep = 1
        if self.ddp_bwd_all and self.xcur is None:
            self.xcur = torch.empty(self.B * 784, device=device)
        # multi-GPU schedule: overlap the fc bucket's all-reduce with the conv
        # backward on a side stream (PTO_COMM_OVERLAP=1), or all-reduce the
        # whole flat buffer once after the backward on the compute stream
        # (=0: no fork/join in the graph, one collective).  Default "auto":
        # both whole-step graphs are captured and timed at startup (max over
        # ranks) and the faster is kept (_choose_schedule).
        self.comm_overlap = {"1": True, "0": False}.get(os.environ.get("PTO_COMM_OVERLAP", "auto"))
        if self.ddp and not self.fuse_fc and os.environ.get("PTO_DDP_BWD_ALL", "1") == "1":
            self.comm_overlap = False  # the fc gradients only exist after the single backward launch
        self._c1 = offs["conv1.weight"][0]
        self._c1_bias = offs["conv1.bias"][0] - self._c1

        # SGD launch table (one "tensor" = the whole flat buffer).
        from ..ops.optim import SgdTable

        self.sgd = SgdTable([(self._params, self.grads, self.mom)], device)
        self.lr_dev = torch.tensor([self.lr], **f32)
        self._graphs = None
        self._graph_unrolled = None
        self._graph_pow = {}
        self._graph_close = {}
        self._close_graphs = os.environ.get("PTO_CLOSE_GRAPHS", "1") == "1"
        self._owed = False  # host view: a conv1 update may be owed (fused_opt)
        self._static_ar = None
        self.steps_done = 0
        self._xgmi, self.comm_info = None, {"transport": "none" if self.world == 1 else "rccl"}
        if self.world > 1 and self.comm in ("xgmi", "auto"):
            self._setup_xgmi()
        self._side = torch.cuda.Stream(device) if self._xgmi is not None else None
        if self.ddp_bwd_all and self._xgmi is not None and self.ar_fused_sgd:
            self.ddp_nrep = self.c1_nrep  # the all-reduce's SGD launch folds them
        elif self.deterministic and self.ddp:
            raise RuntimeError("PTO_DETERMINISTIC=1 on several ranks needs the xGMI all-reduce with its SGD "
                               "epilogue (it folds the per-sample conv1 replicas in order)")
        # graph modes: "full" = the whole step (collectives included) is one
        # HIP graph; "split" = collectives issued eagerly between graphs;
        # "none" = eager launches.  The xGMI kernel and RCCL all-reduces are
        # captured into the graph by default (validated by
        # tests/test_graph_gpu.py); gloo collectives are host-side and cannot
        # be captured, so they use "split" (PTO_CAPTURE_COMM=0 forces it).
        capture_comm = os.environ.get("PTO_CAPTURE_COMM", "1") == "1"
        if (self.ddp and self._xgmi is None and dist.is_initialized() and dist.get_backend() != "nccl"):
            capture_comm = False
        self.graph_mode = graph or ("full" if (not self.ddp or capture_comm) else "split")
        if self._xgmi is not None and self.graph_mode == "split":
            self.graph_mode = "full"  # the xGMI kernel is plain stream work

    def _setup_xgmi(self):
        from ..parallel.xgmi import XgmiAllReduce

        try:
            ar = XgmiAllReduce(self.grads)
        except (RuntimeError, ValueError) as e:  # collective failure: every rank raises
            if self.comm == "xgmi":
                raise
            self.comm_info = {"transport": "rccl", "xgmi_error": str(e)}
            return
        split = self._split()
        ranges = [(0, split), (split, self.numel - split)] if self.comm_overlap else [(0, self.numel)]
        tune = ar.autotune(ranges)
        if self.comm == "xgmi" and not tune["correct"]:
            raise RuntimeError(f"xGMI all-reduce failed verification: {tune}")
        if self.comm == "xgmi" or tune["use_xgmi"]:
            self._xgmi = ar
            self.comm_info = dict(tune, transport="xgmi",
                                  optimizer="allreduce-epilogue" if self.ar_fused_sgd else "sgd-launch")
        else:
            ar.close()
            self.comm_info = dict(tune, transport="rccl")

    def _split(self) -> int:
        return param_offsets()[0]["conv2.weight"][0]

    # ------------------------------------------------------------------
    def _s(self):
        return _lib.stream_ptr(self.device)

    def forward_backward(self):
        self.forward_fc_backward()
        fork = self._probe_fork
        if fork is not None:  # PTO_PROBE_FORK=1: cost of one fork/join pair inside the graph
            cur = torch.cuda.current_stream(self.device)
            fork.wait_stream(cur)
            _lib.check(self.L.pto_noop(1, fork.cuda_stream), "noop")
        self.conv_backward()
        if fork is not None:
            torch.cuda.current_stream(self.device).wait_stream(fork)

    def forward_fc_backward(self):
        """Forward + loss + fc-layer backward: after this the fc grads
        (the first 405,632 elements of the flat buffer, 94% of the bytes)
        are final and their all-reduce can start."""
        L, s, B, P, G = self.L, self._s(), self.B, self._p, self.g
        c = self._check
        bi = self.batch_idx.data_ptr()
        if self.fused_opt:
            o = self._opt_args()
            f12 = (self.data.data_ptr(), P["conv1.weight"].data_ptr(), P["conv1.bias"].data_ptr(),
                   P["conv2.weight"].data_ptr(), P["conv2.bias"].data_ptr(), self.a1p.data_ptr(),
                   self.code1.data_ptr(), self.a2p.data_ptr(), self.code2.data_ptr(), B, bi,
                   self.grads[self._c1:].data_ptr(), self.mom[self._c1:].data_ptr(), self._c1_bias,
                   self.pending.data_ptr(), *o)
            if self.xcur is not None:
                c(L.pto_conv12_fwd_lazy_x(*f12, self.xcur.data_ptr(), _lib.ptr(self.w2f), self.c1rep.data_ptr(),
                                          self.c1_nrep, self.c1_stride, s), "conv12_fwd_lazy_x")
            else:
                c(L.pto_conv12_fwd_lazy(*f12, self.conv12_version, s), "conv12_fwd_lazy")
            c(L.pto_linear_fwd(self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(),
                               self.h1.data_ptr(), B, 500, 800, 1, s), "fc1_fwd")
            if self.merge_f4:  # F4 + d(a2p) + conv1 commit; dW2/db -> B2, cursor advance -> B1
                c(L.pto_fc2_ce_dx(self.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                                  self.target.data_ptr(), P["fc1.weight"].data_ptr(), self.loss_rows.data_ptr(),
                                  self.dlogits.data_ptr(), self.dh1.data_ptr(), self.da2p.data_ptr(), B, 1.0 / B, bi,
                                  self._params[self._c1:].data_ptr(), self.grads[self._c1:].data_ptr(),
                                  self.mom[self._c1:].data_ptr(), self.numel - self._c1, self.pending.data_ptr(),
                                  *o, self.c1rep.data_ptr(), self.c1_nrep, self.c1_stride, s), "fc2_ce_dx")
                return
            c(L.pto_fc2_ce_commit(self.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                                  self.target.data_ptr(), self.loss_rows.data_ptr(), self.dlogits.data_ptr(),
                                  self.dh1.data_ptr(), B, 1.0 / B, bi, self.batch_snap.data_ptr(),
                                  self._params[self._c1:].data_ptr(), self.grads[self._c1:].data_ptr(),
                                  self.mom[self._c1:].data_ptr(), self.numel - self._c1, self.pending.data_ptr(),
                                  *o, s), "fc2_ce_commit")
            fc_args = (self.dh1.data_ptr(), self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), self.h1.data_ptr(),
                       self.dlogits.data_ptr(), G["fc1.weight"].data_ptr(), G["fc1.bias"].data_ptr(),
                       G["fc2.weight"].data_ptr(), G["fc2.bias"].data_ptr(), self.da2p.data_ptr(), B)
            if self.dw1_sgd:
                c(L.pto_fc_bwd_adv_nodw1(fc_args[0], fc_args[1], fc_args[2], fc_args[3], fc_args[4], *fc_args[6:],
                                         bi, self.n_batches, self.pending.data_ptr(), s), "fc_bwd_adv_nodw1")
                return
            if self._bwd_side is None:
                c(L.pto_fc_bwd_adv(*fc_args, bi, self.n_batches, self.pending.data_ptr(), s), "fc_bwd_adv")
                return
            # two-stream backward: the fc weight gradients and the fc update
            # run on a side stream next to d(a2p) -> conv2 bwd -> conv1 bwd
            # (the update waits for d(a2p), the last reader of W1)
            cur, side = torch.cuda.current_stream(self.device), self._bwd_side
            side.wait_stream(cur)
            c(L.pto_fc_bwd_part(*fc_args, None, 1, None, 2, side.cuda_stream), "fc_bwd_wgrad")
            c(L.pto_fc_bwd_part(*fc_args, bi, self.n_batches, self.pending.data_ptr(), 1, s), "fc_bwd_dgrad")
            side.wait_stream(cur)
            split = self._split()
            c(L.pto_sgd_flat(self._params.data_ptr(), self.grads.data_ptr(), self.mom.data_ptr(), split, split, *o,
                             side.cuda_stream), "sgd_fc")
            return
        if self.ddp_bwd_all:  # F12 (copies the images out for the backward), fc1, F4 + d(a2p)
            c(L.pto_conv12_fwd_lazy_x(self.data.data_ptr(), P["conv1.weight"].data_ptr(),
                                      P["conv1.bias"].data_ptr(), P["conv2.weight"].data_ptr(),
                                      P["conv2.bias"].data_ptr(), self.a1p.data_ptr(), self.code1.data_ptr(),
                                      self.a2p.data_ptr(), self.code2.data_ptr(), B, bi, None, None, 0, None, None,
                                      0.0, 0.0, 1.0, 0, self.xcur.data_ptr(), None, None, 1, 0, s),
              "conv12_fwd_x")
            c(L.pto_linear_fwd(self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(),
                               self.h1.data_ptr(), B, 500, 800, 1, s), "fc1_fwd")
            c(L.pto_fc2_ce_dx(self.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                              self.target.data_ptr(), P["fc1.weight"].data_ptr(), self.loss_rows.data_ptr(),
                              self.dlogits.data_ptr(), self.dh1.data_ptr(), self.da2p.data_ptr(), B, 1.0 / B, bi,
                              self._params[self._c1:].data_ptr(), self.grads[self._c1:].data_ptr(),
                              self.mom[self._c1:].data_ptr(), self.numel - self._c1, None, *self._opt_args(),
                              None, 1, 0, s), "fc2_ce_dx")
            return
        # same F1+F2 launch without an owed update (pending = nullptr)
        c(L.pto_conv12_fwd_lazy(self.data.data_ptr(), P["conv1.weight"].data_ptr(), P["conv1.bias"].data_ptr(),
                                P["conv2.weight"].data_ptr(), P["conv2.bias"].data_ptr(), self.a1p.data_ptr(),
                                self.code1.data_ptr(), self.a2p.data_ptr(), self.code2.data_ptr(), B, bi, None, None,
                                0, None, None, 0.0, 0.0, 1.0, 0, self.conv12_version, s), "conv12_fwd")
        if self.fuse_fc:  # fc1 + (last block per 16 rows) fc2/CE/dlogits/dh1 in one launch
            c(L.pto_fc12_ce(self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(),
                            self.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                            self.target.data_ptr(), self.loss_rows.data_ptr(), self.dlogits.data_ptr(),
                            self.dh1.data_ptr(), B, 1.0 / B, bi, self.fc_counters.data_ptr(), s), "fc12_ce")
        else:
            c(L.pto_linear_fwd(self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(),
                               self.h1.data_ptr(), B, 500, 800, 1, s), "fc1_fwd")
            c(L.pto_fc2_ce(self.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                           self.target.data_ptr(), None, self.loss_rows.data_ptr(), self.dlogits.data_ptr(),
                           self.dh1.data_ptr(), B, 1.0 / B, bi, s), "fc2_ce")
        c(L.pto_fc_bwd(self.dh1.data_ptr(), self.a2p.data_ptr(), P["fc1.weight"].data_ptr(), self.h1.data_ptr(),
                       self.dlogits.data_ptr(), G["fc1.weight"].data_ptr(), G["fc1.bias"].data_ptr(),
                       G["fc2.weight"].data_ptr(), G["fc2.bias"].data_ptr(), self.da2p.data_ptr(), B, s), "fc_bwd")

    def conv_backward(self):
        L, s, B, P, G = self.L, self._s(), self.B, self._p, self.g
        c = self._check
        bi = self.batch_idx.data_ptr()
        # conv2 wgrad + dgrad(col2im) + bias in one launch.  (Folding conv1's
        # wgrad into the dgrad blocks is supported by the kernel — pass gw1 —
        # but measured break-even: every sample-block adds into the same 520
        # addresses, 64-way atomic contention.  The separate 320-block conv1
        # launch below adds each address only 16 times.)
        if self.bwd_all or self.ddp_bwd_all:  # the whole backward (+ every update when single-GPU) in one launch
            offs = param_offsets()[0]
            o = [offs[n][0] for n in ("fc2.weight", "fc2.bias", "fc1.weight", "fc1.bias", "conv2.weight",
                                      "conv2.bias", "conv1.weight", "conv1.bias")]
            go = not self.bwd_all  # grads-only (DDP): the all-reduce's epilogue updates
            c(L.pto_bwd_all(self.da2p.data_ptr(), self.code2.data_ptr(), self.a1p.data_ptr(), _lib.ptr(self.w2f),
                            self.xcur.data_ptr(), self.code1.data_ptr(), self.dh1.data_ptr(), self.a2p.data_ptr(),
                            self.h1.data_ptr(), self.dlogits.data_ptr(), self._params.data_ptr(),
                            self.grads.data_ptr(), self.mom.data_ptr(), *o, _lib.ptr(self.c2_ctr),
                            None if go else bi, self.n_batches, None if go else self.pending.data_ptr(), B,
                            *self._opt_args(), self.c1rep.data_ptr(), self.ddp_nrep if go else self.c1_nrep, self.c1_stride,
                            int(go), _lib.ptr(self.wpart), s), "bwd_all")
            return
        if self.merge_f4:  # + B3's all-row reductions (dW2, db1, db2)
            c(L.pto_conv2_bwd_fc(self.da2p.data_ptr(), self.code2.data_ptr(), self.a1p.data_ptr(),
                                 P["conv2.weight"].data_ptr(), G["conv2.weight"].data_ptr(),
                                 G["conv2.bias"].data_ptr(), self.da1p.data_ptr(), B, self.dh1.data_ptr(),
                                 self.h1.data_ptr(), self.dlogits.data_ptr(), G["fc2.weight"].data_ptr(),
                                 G["fc1.bias"].data_ptr(), G["fc2.bias"].data_ptr(), s), "conv2_bwd_fc")
        else:
            c(L.pto_conv2_bwd(self.da2p.data_ptr(), self.code2.data_ptr(), self.a1p.data_ptr(),
                              P["conv2.weight"].data_ptr(), G["conv2.weight"].data_ptr(), G["conv2.bias"].data_ptr(),
                              self.da1p.data_ptr(), B, 7, None, None, None, None, None, s), "conv2_bwd")
        if self.fused_opt:  # + the fc/conv2 update (grads final since B3/B2); B1 reads the cursor snapshot
            if self.dw1_sgd:
                xb = (self.xcur.data_ptr(), None) if self.xcur is not None else (self.data.data_ptr(),
                                                                                   self.batch_snap.data_ptr())
                c(L.pto_conv1_bwd_sgd_dw1(self.da1p.data_ptr(), self.code1.data_ptr(), xb[0],
                                          G["conv1.weight"].data_ptr(), G["conv1.bias"].data_ptr(), B,
                                          xb[1], self._params.data_ptr(), self.grads.data_ptr(),
                                          self.mom.data_ptr(), self._c1, self._split(), self.dh1.data_ptr(),
                                          self.a2p.data_ptr(), param_offsets()[0]["fc1.weight"][0],
                                          bi if self.merge_f4 else None, self.n_batches,
                                          self.pending.data_ptr() if self.merge_f4 else None,
                                          *self._opt_args(), s), "conv1_bwd_sgd_dw1")
                return
            if self._bwd_side is None:
                c(L.pto_conv1_bwd_sgd(self.da1p.data_ptr(), self.code1.data_ptr(), self.data.data_ptr(),
                                      G["conv1.weight"].data_ptr(), G["conv1.bias"].data_ptr(), B,
                                      self.batch_snap.data_ptr(), self._params.data_ptr(), self.grads.data_ptr(),
                                      self.mom.data_ptr(), self._c1, self._split(), *self._opt_args(), s),
                  "conv1_bwd_sgd")
                return
            split, esz = self._split(), self._params.element_size()
            c(L.pto_conv1_bwd_sgd(self.da1p.data_ptr(), self.code1.data_ptr(), self.data.data_ptr(),
                                  G["conv1.weight"].data_ptr(), G["conv1.bias"].data_ptr(), B,
                                  self.batch_snap.data_ptr(), self._params.data_ptr() + split * esz,
                                  self.grads.data_ptr() + split * esz, self.mom.data_ptr() + split * esz,
                                  self._c1 - split, 0, *self._opt_args(), s), "conv1_bwd_sgd")
            torch.cuda.current_stream(self.device).wait_stream(self._bwd_side)  # fc update joins the step
            return
        c(L.pto_conv1_bwd(self.da1p.data_ptr(), self.code1.data_ptr(), self.data.data_ptr(),
                          G["conv1.weight"].data_ptr(), G["conv1.bias"].data_ptr(), B, bi, s), "conv1_bwd")

    def allreduce(self):
        if self.world == 1:
            return
        if self._xgmi is not None:
            self._xgmi.allreduce_(0, self.numel)
        else:
            dist.all_reduce(self.grads)

    def _bucket_views(self):
        """Two DDP buckets in backward order: fc grads, conv grads."""
        if not hasattr(self, "_buckets"):
            split = self._split()
            self._buckets = (self.grads[:split], self.grads[split:])
        return self._buckets

    def _opt_args(self):
        """(lr device ptr, momentum, weight decay, grad scale, nesterov) for
        the fused-optimizer launchers."""
        return (self.lr_dev.data_ptr(), self.momentum, self.weight_decay, 1.0 / self.world, int(self.nesterov))

    def flush(self):
        """Commit an owed conv1 update (fused-optimizer schedule) so the flat
        buffers hold exactly the parameters/momentum an eager SGD step would
        have left.  Idempotent; a no-op for the other schedules and after a
        run() that ended on a closing graph."""
        if not self.fused_opt or self.steps_done == 0 or not self._owed:
            return
        self._commit_launch()
        self._owed = False

    def _commit_launch(self):
        _lib.check(self.L.pto_conv1_commit(self._params[self._c1:].data_ptr(), self.grads[self._c1:].data_ptr(),
                                           self.mom[self._c1:].data_ptr(), self.numel - self._c1,
                                           self.pending.data_ptr(), *self._opt_args(), self.c1rep.data_ptr(),
                                           self.c1_nrep, self.c1_stride, self._s()), "conv1_commit")

    @property
    def params(self):
        """Flat fp32 parameter buffer (owed updates committed first)."""
        self.flush()
        return self._params

    @property
    def p(self):
        """Parameter views by reference name (owed updates committed first)."""
        self.flush()
        return self._p

    def optimizer_step(self):
        if self.fused_opt:  # done inside the step's other launches
            return
        self.sgd.step(self.lr_dev, self.lr, self.momentum, self.weight_decay, 1.0 / self.world, self.nesterov,
                      zero_grad=True, stream=self._s(), batch_cursor=self.batch_idx, n_batches=self.n_batches)

    def _check(self, rc, name):
        _lib.check(rc, name)
        if self._noops:
            self._probe_noops()

    def _probe_noops(self):
        """PTO_PROBE_NOOPS=k: k empty launches after every phase launch
        (measures what one launch boundary costs inside the graph)."""
        import os

        k = int(os.environ.get("PTO_PROBE_NOOPS", "0"))
        for _ in range(k):
            _lib.check(self.L.pto_noop(int(os.environ.get("PTO_PROBE_BLOCKS", "1")), self._s()), "noop")

    def _eager_step(self):
        if self.ddp and self._xgmi is not None:
            self._xgmi_step()
            return
        if self.ddp:
            self._ddp_step()
            return
        self.forward_backward()
        self.optimizer_step()

    def _xgmi_step(self):
        """Default: forward + backward, then ONE xGMI all-reduce of the whole
        flat gradient buffer with the SGD epilogue (update, conv-grad
        zeroing, cursor advance) on the compute stream — no optimizer launch,
        no side stream.  ``comm_overlap``: the fc bucket is all-reduced on a
        side stream while the conv backward runs, the conv bucket after it
        (a graph fork/join costs ~19 us, more than the overlap hides at this
        size).  Pure stream work: capturable into one graph."""
        split = self._split()
        if not self.comm_overlap:
            self.forward_fc_backward()
            self.conv_backward()
            if self.ar_fused_sgd:
                lr, mom, wd, gs, nes = self._opt_args()
                self._xgmi.allreduce_sgd_(0, self.numel, params=self._params, mom=self.mom, lr_dev=self.lr_dev,
                                          momentum=mom, weight_decay=wd, gscale=gs, nesterov=bool(nes),
                                          zero_from=split, cursor=self.batch_idx, n_batches=self.n_batches,
                                          replicas=self.c1rep, n_replicas=self.ddp_nrep, rep_from=self._c1)
                return
            self._xgmi.allreduce_(0, self.numel)
            self.optimizer_step()
            return
        cur = torch.cuda.current_stream(self.device)
        self.forward_fc_backward()
        self._side.wait_stream(cur)
        if self.ar_fused_sgd:  # the update rides in the all-reduce launches: no optimizer launch
            lr, mom, wd, gs, nes = self._opt_args()
            kw = dict(params=self._params, mom=self.mom, lr_dev=self.lr_dev, momentum=mom, weight_decay=wd,
                      gscale=gs, nesterov=bool(nes), zero_from=split)
            self._xgmi.allreduce_sgd_(0, split, chan=0, stream=self._side, **kw)
            self.conv_backward()
            self._xgmi.allreduce_sgd_(split, self.numel - split, chan=1, cursor=self.batch_idx,
                                      n_batches=self.n_batches, **kw)
            cur.wait_stream(self._side)
            return
        self._xgmi.allreduce_(0, split, chan=0, stream=self._side)
        self.conv_backward()
        self._xgmi.allreduce_(split, self.numel - split, chan=1)
        cur.wait_stream(self._side)
        self.optimizer_step()

    def _ddp_step(self):
        """RCCL: one all-reduce of the whole flat buffer after the backward
        (default), or (``comm_overlap``) bucket 0 (fc grads, 94% of the
        bytes) on RCCL's stream while the conv backward runs, then bucket 1;
        the optimizer waits for both.  Valid eagerly and under graph
        capture."""
        if not self.comm_overlap:
            self.forward_fc_backward()
            self.conv_backward()
            dist.all_reduce(self.grads)
            self.optimizer_step()
            return
        fc_b, conv_b = self._bucket_views()
        self.forward_fc_backward()
        w0 = dist.all_reduce(fc_b, async_op=True)
        self.conv_backward()
        w1 = dist.all_reduce(conv_b, async_op=True)
        w0.wait()
        w1.wait()
        self.optimizer_step()

    def _capture(self):
        # Warm up on a side stream (lazy library/allocator init must not
        # happen under capture), then roll the state back so capture does
        # not change the training trajectory, then capture.
        state = (self._params, self.mom, self.grads, self.batch_idx, self.pending, self.batch_snap, self.c1rep)
        snap = [t.clone() for t in state]
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        # the xGMI barriers spin for PTO_XGMI_TIMEOUT_MS only: every rank
        # arrives here after its own checkpoint load / earlier captures, so
        # they line up on the host first (skew > 500 ms tripped it)
        self._align_ranks("warmup")
        with torch.cuda.stream(s):
            self._eager_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for dst, src in zip(state, snap):
            dst.copy_(src)
        torch.cuda.synchronize(self.device)
        graphs = []
        if self.graph_mode == "full":
            # k consecutive steps per graph for k = 1, 2, 4, ..., unroll (the
            # device batch cursor walks the data inside the graph): run(n)
            # then needs n // unroll + popcount(n % unroll) replays, so a
            # 20-step run costs 2 replays, not 20 (profiles/graph_unroll_sweep_r1.md)
            self._graph_pow = {}
            for k in self._graph_sizes():
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk):
                    for _ in range(k):
                        self._eager_step()
                self._graph_pow[k] = gk
            # fused-optimizer schedule: a "closing" graph per run length
            # 1..unroll whose last node commits the owed conv1 update, so
            # run(n) is n // unroll replays + ONE closing replay and needs
            # no separate flush launch afterwards
            self._graph_close = {}
            if self.fused_opt and self._close_graphs:
                for k in range(1, self.unroll + 1):
                    gk = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gk):
                        for _ in range(k):
                            self._eager_step()
                        self._commit_launch()
                    self._graph_close[k] = gk
            graphs = [self._graph_pow[1]]
            self._graph_unrolled = self._graph_pow[max(self._graph_pow)]
            # replay every graph once now and roll the training state back:
            # a graph's first launch pays a one-time upload (measured +80 us
            # on the first 16-step replay of a 20-step timed run); xGMI
            # epochs are NOT rolled back (they must stay in step with the
            # peers, which replay the same graphs)
            torch.cuda.synchronize(self.device)
            snap = [t.clone() for t in state]
            self._align_ranks("warm-replay")
            for g in list(self._graph_pow.values()) + list(self._graph_close.values()):
                g.replay()
            torch.cuda.synchronize(self.device)
            for dst, src in zip(state, snap):
                dst.copy_(src)
            torch.cuda.synchronize(self.device)
            self._align_ranks("captured")
        else:  # split: collectives outside the graphs, overlapped with conv bwd
            ga, gb, gc = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                self.forward_fc_backward()
            with torch.cuda.graph(gb):
                self.conv_backward()
            with torch.cuda.graph(gc):
                self.optimizer_step()
            graphs = [ga, gb, gc]
        self._graphs = graphs

    def _align_ranks(self, tag: str):
        """Host-side barrier before device work whose cross-rank spins are
        short-bounded (the xGMI all-reduce); a no-op otherwise."""
        if self._xgmi is not None:
            from ..utils import dist as pdist

            pdist.host_barrier(tag=f"xgmi-{tag}")

    def _graph_sizes(self) -> list[int]:
        if self.fused_opt and self._close_graphs:
            return sorted({1, max(1, self.unroll)})  # run() ends on a closing graph
        sizes, k = [], 1
        while k < self.unroll:
            sizes.append(k)
            k *= 2
        return sizes + [max(1, self.unroll)]

    def _choose_schedule(self, reps: int = 8):
        """Capture the step both ways (one whole-buffer all-reduce after the
        backward / fc bucket overlapped on a side stream), time ``reps``
        replays of each unrolled graph (max over ranks, same decision on
        every rank), roll the training state back, keep the faster."""
        import time

        from ..utils import dist as pdist

        state = (self._params, self.mom, self.grads, self.batch_idx, self.pending, self.batch_snap, self.c1rep)
        snap = [t.clone() for t in state]
        res = {}
        for ov in (False, True):
            self.comm_overlap = ov
            self._graphs, self._graph_unrolled = None, None
            self._capture()
            self._graph_unrolled.replay()  # warm
            torch.cuda.synchronize(self.device)
            pdist.barrier(self.device)
            torch.cuda.synchronize(self.device)
            t0 = time.perf_counter()
            for _ in range(reps):
                self._graph_unrolled.replay()
            torch.cuda.synchronize(self.device)
            t = pdist.all_reduce_max(time.perf_counter() - t0, self.device) / (reps * self.unroll)
            res[ov] = (t, self._graphs, self._graph_unrolled, self._graph_pow)
            for dst, src in zip(state, snap):
                dst.copy_(src)
            torch.cuda.synchronize(self.device)
        best = min(res, key=lambda k: res[k][0])
        self.comm_overlap = best
        _, self._graphs, self._graph_unrolled, self._graph_pow = res[best]
        self.comm_info["schedule"] = {"chosen": "overlap" if best else "sequential",
                                      "sequential_us": round(res[False][0] * 1e6, 2),
                                      "overlap_us": round(res[True][0] * 1e6, 2)}

    def _ensure_captured(self):
        if self._graphs is not None:
            return
        if self.ddp and self.graph_mode == "full" and self.comm_overlap is None and self.unroll > 1:
            try:
                self._choose_schedule()
                return
            except Exception as e:  # noqa: BLE001 - fall back to the fixed schedule below
                import warnings

                warnings.warn(f"schedule autotune failed ({e}); using the sequential schedule")
                torch.cuda.synchronize(self.device)
                self.comm_overlap = False
                self._graphs, self._graph_unrolled = None, None
        try:
            self._capture()
        except Exception as e:  # noqa: BLE001 - capture of collectives unsupported
            if self.graph_mode != "full" or not self.ddp:
                raise
            import warnings

            warnings.warn(f"HIP-graph capture of the DDP step failed ({e}); using split graphs")
            torch.cuda.synchronize(self.device)
            self.graph_mode = "split"
            self._capture()

    def run(self, n: int, blocking_check: bool = True):
        """Run exactly ``n`` training steps: the largest captured multi-step
        graphs first (n // unroll replays of the unroll-step graph, then one
        replay per set bit of the remainder), then check the gradient
        transport's error word (a dead or stalled xGMI peer raises
        :class:`~pytorch_operator_1_amd.parallel.xgmi.XgmiTimeout` here, at
        most one chunk after it happened).  ``blocking_check=False``: the
        check does not wait for this chunk (it reads the word captured after
        the previous chunk), so a training loop keeps the device busy while
        it logs."""
        if n <= 0:
            return
        if self.graph_mode == "full":
            self._ensure_captured()
            if self._graph_close:
                U = max(self._graph_close)
                g = self._graph_pow[U]
                while n > U:
                    g.replay()
                    self.steps_done += U
                    n -= U
                self._graph_close[n].replay()
                self.steps_done += n
                self._owed = False
                n = 0
            for k in sorted(self._graph_pow, reverse=True):
                g = self._graph_pow[k]
                while n >= k:
                    g.replay()
                    self.steps_done += k
                    self._owed = self.fused_opt
                    n -= k
        for _ in range(n):
            self.step()
        self.check_comm(blocking_check)

    def check_comm(self, blocking: bool = True):
        """Raise if the xGMI all-reduce reported a barrier timeout (no-op for
        RCCL/gloo, whose failures raise from the collective itself).
        Synchronises with the device when xGMI is in use, unless
        ``blocking=False`` (then the word of the previous call is checked)."""
        if self._xgmi is not None:
            if blocking:
                self._xgmi.check()
            else:
                self._xgmi.poll()

    def loss_async(self):
        """Mean loss of the last step, copied into pinned host memory without
        waiting: returns ``(host_tensor, event)``; read the tensor after
        ``event.synchronize()``."""
        if getattr(self, "_loss_host", None) is None:
            self._loss_host = torch.zeros(2, dtype=torch.float32, pin_memory=True)
            self._loss_i = 0
        buf = self._loss_host[self._loss_i:self._loss_i + 1]
        self._loss_i ^= 1
        buf.copy_(self.loss_rows.mean().view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return buf, ev

    @property
    def needs_host_barrier(self) -> bool:
        """True if peers' queued collectives time out when this rank spends
        long on host work (checkpoint, evaluation): the caller must then
        re-align the ranks (utils.dist.host_barrier) before the next run()."""
        return self._xgmi is not None

    def step(self):
        if self.graph_mode == "none":
            self._eager_step()
        else:
            self._ensure_captured()
            if self.graph_mode == "full":
                self._graphs[0].replay()
            elif not self.ddp:
                for g in self._graphs:
                    g.replay()
            else:
                # bucket 0 (fc grads) all-reduces on RCCL's stream while the
                # conv backward graph runs; bucket 1 follows; the optimizer
                # graph waits for both (DDP-style overlap)
                fc_b, conv_b = self._bucket_views()
                self._graphs[0].replay()
                if self.ddp_bwd_all:  # the fc grads are produced by the backward launch
                    self._graphs[1].replay()
                    dist.all_reduce(self.grads)
                else:
                    w0 = dist.all_reduce(fc_b, async_op=True)
                    self._graphs[1].replay()
                    w1 = dist.all_reduce(conv_b, async_op=True)
                    w0.wait()
                    w1.wait()
                self._graphs[2].replay()
        self.steps_done += 1
        self._owed = self.fused_opt

    def last_loss(self):
        return float(self.loss_rows.mean().item())

    @torch.no_grad()
    def evaluate(self, data: torch.Tensor, target: torch.Tensor, batch_size: int = 1000):
        """Test pass with the same kernels (forward + fused argmax/NLL-sum
        eval head, K11).  Returns ``(mean_loss, accuracy)`` like the
        reference's ``test()`` (examples/mnist/mnist.py:51-65)."""
        self.flush()
        L, s, P = self.L, self._s(), self._p
        n = data.shape[0]
        Bm = min(batch_size, n)
        f32 = dict(device=self.device, dtype=torch.float32)
        a1p = torch.empty(Bm * 2880, **f32)
        c1 = torch.empty(Bm * 2880, device=self.device, dtype=torch.uint8)
        a2p = torch.empty(Bm * 800, **f32)
        c2 = torch.empty(Bm * 800, device=self.device, dtype=torch.uint8)
        h1 = torch.empty(Bm * 500, **f32)
        logp = torch.empty(Bm * 10, **f32)
        stats = torch.zeros(2, **f32)
        x = data.reshape(n, 784).contiguous()
        y = target.to(torch.int64).contiguous()
        c = _lib.check
        for i in range(0, n, Bm):
            B = min(Bm, n - i)
            xb, yb = x[i:i + B], y[i:i + B]
            c(L.pto_conv1_fwd(xb.data_ptr(), P["conv1.weight"].data_ptr(), P["conv1.bias"].data_ptr(),
                              a1p.data_ptr(), c1.data_ptr(), B, None, s), "conv1_fwd")
            c(L.pto_conv2_fwd(a1p.data_ptr(), P["conv2.weight"].data_ptr(), P["conv2.bias"].data_ptr(),
                              a2p.data_ptr(), c2.data_ptr(), B, s), "conv2_fwd")
            c(L.pto_linear_fwd(a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(), h1.data_ptr(),
                               B, 500, 800, 1, s), "fc1_fwd")
            c(L.pto_fc2_ce(h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(), yb.data_ptr(),
                           logp.data_ptr(), None, None, None, B, 1.0, None, s), "fc2_ce")
            c(L.pto_eval_head(logp.data_ptr(), yb.data_ptr(), stats.data_ptr(), B, s), "eval_head")
        loss_sum, correct = stats.tolist()
        return loss_sum / n, correct / n

    def set_lr(self, lr: float):
        self.flush()  # an owed update uses the lr of the step that produced it
        self.lr = float(lr)
        self.lr_dev.fill_(self.lr)

    # ------------------------------------------------------------------
    def state_dict(self):
        """Module-style state (same keys as the reference ``Net``) plus the
        optimizer momentum in torch.optim.SGD layout."""
        self.flush()
        model = {k: v.detach().clone() for k, v in self._p.items()}
        offs, _ = param_offsets()
        order = [n for n, _ in PARAM_SHAPES]
        mom = {}
        for name in order:
            off, shape = offs[name]
            mom[name] = self.mom[off:off + math.prod(shape)].view(shape).clone()
        return {"model": model, "momentum": mom, "lr": self.lr, "momentum_coef": self.momentum,
                "batch_idx": int(self.batch_idx.item()), "steps_done": self.steps_done}

    def load_state_dict(self, sd):
        self.flush()  # nothing owed afterwards: the loaded state is complete
        offs, _ = param_offsets()
        with torch.no_grad():
            for name, t in sd["model"].items():
                self._p[name].copy_(t.to(self.device))
            for name, t in sd.get("momentum", {}).items():
                off, shape = offs[name]
                self.mom[off:off + math.prod(shape)].copy_(t.reshape(-1).to(self.device))
        self.batch_idx.fill_(int(sd.get("batch_idx", 0)) % self.n_batches)
        self.steps_done = int(sd.get("steps_done", 0))
        self.set_lr(float(sd.get("lr", self.lr)))
