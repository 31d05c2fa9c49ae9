"""Build and load the package's gfx950 HIP kernel library.

All device code is compiled by ``hipcc --offload-arch=gfx950`` into ONE
in-tree shared object, ``pytorch_operator_1_amd/_lib/libpto_hip.so``, that
exposes a plain C ABI (``extern "C" pto_*`` launchers taking raw device
pointers and a ``hipStream_t``).  It is loaded with ``ctypes`` — no torch
C++ headers in the kernel build, so a rebuild takes seconds and the object
works with any torch-ROCm of the same HIP major version.

On a GPU box the library is REQUIRED: :func:`lib` raises if it cannot be
built or loaded (no silent eager fallback).  On a CPU-only host it is only
needed by the ``build()`` check.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os
import shutil
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libpto_hip.so")
ARCH = os.environ.get("PTO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

HIP_SOURCES = ("kernels/mnist_kernels.hip", "kernels/common_kernels.hip", "kernels/optim_kernels.hip",
               "kernels/llm_kernels.hip", "kernels/attention.hip", "kernels/bn_kernels.hip", "kernels/conv3x3.hip",
               "comm/xgmi_allreduce.hip")

_lock = threading.Lock()
# launchers return an int hipError; these few return something else
_RESTYPES = {"pto_ar_timeout_ticks": ctypes.c_longlong}
_lib = None


def _sources():
    return [os.path.join(CSRC, s) for s in HIP_SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _digest() -> str:
    h = hashlib.sha256()
    h.update(ARCH.encode())
    for p in sorted(_sources() + glob.glob(os.path.join(CSRC, "kernels", "*.h")) +
                    glob.glob(os.path.join(CSRC, "comm", "*.h"))):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def is_current() -> bool:
    """True if the in-tree library was built from the current sources."""
    stamp = LIB_PATH + ".stamp"
    if not (os.path.exists(LIB_PATH) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == _digest()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every HIP source for gfx950 into the in-tree library."""
    os.makedirs(LIB_DIR, exist_ok=True)
    stamp = LIB_PATH + ".stamp"
    dig = _digest()
    if not force and os.path.exists(LIB_PATH) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == dig:
                return LIB_PATH
    tmp = LIB_PATH + f".tmp{os.getpid()}"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(CSRC, "kernels"), "-I", os.path.join(CSRC, "comm"), "-o", tmp] + _sources()
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    with open(stamp, "w") as f:
        f.write(dig)
    return LIB_PATH


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_L = ctypes.c_longlong

_SIGS = {
    "pto_conv1_fwd": [_P, _P, _P, _P, _P, _I, _P, _P],
    "pto_conv2_fwd": [_P, _P, _P, _P, _P, _I, _P],
    "pto_linear_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "pto_linear_bwd": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "pto_relu_bwd": [_P, _P, _P, _I, _P],
    "pto_fc2_ce": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _P, _P],
    "pto_conv2_bwd": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P],
    "pto_conv1_bwd": [_P, _P, _P, _P, _P, _I, _P, _P],
    "pto_conv1_bwd_data": [_P, _P, _P, _P, _I, _P],
    # fused-optimizer schedule of the single-process MNIST step
    "pto_conv12_fwd_lazy_x": [_P] * 9 + [_I, _P, _P, _P, _I, _P, _P, _F, _F, _F, _I, _P, _P, _P, _I, _I, _P],
    "pto_conv12_fwd_ar": [_P] * 9 + [_I, _P, _P, _P, _I, _I, _P, _P, _I, _P, _P, _P, _F, _F, _F, _I,
                                     _L, _L, _I, _L, _L, _L, _I, _L, _I, _I, _L, _P, _P],
    "pto_synth_mnist": [_P, _P, _L, ctypes.c_ulonglong, _P],
    "pto_bwd_all": [_P] * 13 + [_L] * 8 + [_P, _P, _L, _P, _I, _P, _F, _F, _F, _I, _P, _I, _I, _I, _P, _P, _I,
                                          _P],
    "pto_conv1_commit": [_P, _P, _P, _I, _P, _P, _F, _F, _F, _I, _P, _I, _I, _P],
    "pto_mnist_ddp_sgd": [_P, _P, _P, _I, _I, _I, _P, _I, _P, _F, _F, _F, _I, _P, _L, _P],
    "pto_fc2_ce_dx": [_P] * 9 + [_I, _F, _P, _P, _P, _P, _I, _P, _P, _F, _F, _F, _I, _P, _I, _I, _P, _P, _P, _L,
                                  _P, _P, _P],
    "pto_fc1_fwd_split": [_P, _P, _P, _I, _P],
    "pto_eval_head": [_P, _P, _P, _I, _P],
    "pto_sgd_block_count": [_L],
    "pto_sgd_multi": [_P, _P, _I, _I, _P, _F, _F, _F, _F, _I, _I, _P, _L, _P],
    "pto_log_softmax_fwd": [_P, _P, _I, _I, _P],
    "pto_log_softmax_bwd": [_P, _P, _P, _I, _I, _P],
    "pto_cross_entropy_fwd": [_P, _P, _P, _P, _I, _I, _F, _P],
    "pto_scale": [_P, _P, _F, _L, _P],
    "pto_sum": [_P, _P, _L, _F, _P],
    "pto_adamw_block_count": [_L],
    "pto_adamw_multi": [_P, _P, _I, _I, _I, _P, _F, _F, _F, _F, _F, _I, _F, _I, _P],
    "pto_bf16_to_f32": [_P, _P, _L, _P],
    # LLM memory-bound kernels (csrc/kernels/llm_kernels.hip)
    "pto_add_rmsnorm_fwd": [_P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
    "pto_rmsnorm_bwd_groups": [_L],
    "pto_rmsnorm_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "pto_swiglu_fwd": [_P, _P, _L, _I, _P],
    "pto_swiglu_bwd": [_P, _P, _P, _L, _I, _P],
    "pto_swiglu_bwd_t": [_P, _P, _P, _P, _L, _I, _P],
    "pto_rope": [_P, _P, _P, _P, _L, _I, _I, _I, _I, _L, _I, _P],
    "pto_ce_fwd": [_P, _P, _P, _P, _L, _I, _L, _P],
    "pto_ce_bwd": [_P, _P, _P, _P, _L, _I, _L, _P],
    "pto_transpose_bf16": [_P, _P, _L, _L, _L, _L, _P],
    "pto_noop": [_I, _P],
    "pto_graph_upload": [_P, _P],
    "pto_lane_ops_selftest": [_P, _P, _P, _P],
    "pto_probe_kernel": [_I, _I, _P, _I, _I, _P],
    "pto_gridbar_probe": [_I, _I, _P, _I, _I, _P],
    "pto_cu_id_probe": [_I, _P, _I, _P],
    "pto_stream_create_cu_mask": [ctypes.c_uint, _P, ctypes.POINTER(ctypes.c_void_p)],
    "pto_stream_get_cu_mask": [_P, ctypes.c_uint, _P],
    "pto_stream_destroy": [_P],
    # fused BatchNorm(+add)(+ReLU), channels-last bf16 (csrc/kernels/bn_kernels.hip)
    "pto_bn_scratch_floats": [_L, _I],
    "pto_bn_fwd": [_P, _P, _P, _L, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _I, _P, _P],
    "pto_bn_bwd": [_P, _P, _P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _I, _P],
    "pto_bn_fwd_part": [_P, _I, _P, _P, _P, _L, _I, _P, _P, _F, _F, _P, _P, _P, _P, _I, _P, _P],
    # ResNet-50 3x3 convs (csrc/kernels/conv3x3.hip)
    "pto_conv3x3_tile_m": [_I],
    "pto_conv3x3_set_variant": [_I, _I],
    "pto_conv3x3_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "pto_conv1x1_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "pto_conv1x1_set_variant": [_I],
    "pto_conv3x3_wcast": [_P, _P, _L, _P],
    "pto_conv3x3_wflip": [_P, _P, _P, _I, _I, _P],
    "pto_maxpool_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "pto_stem_fwd": [_P, _P, _L, _L, _L, _L, _P, _P, _I, _P],
    "pto_maxpool_bwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    # causal GQA flash attention, head_dim 128 (csrc/kernels/attention.hip)
    "pto_attn_fwd": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _L, _L, _L, _L, _F, _P],
    "pto_attn_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _L, _L, _L, _L, _F, _P],
    # xGMI peer all-reduce (csrc/comm/xgmi_allreduce.hip)
    "pto_ar_ipc_handle_size": [],
    "pto_ar_flag_bytes": [_I],
    "pto_ar_max_ranks": [],
    "pto_ar_peers_bytes": [],
    "pto_ar_epoch_words": [],
    "pto_ar_set_timeout_ms": [_I],
    "pto_ar_set_protocol": [_I],
    "pto_ar_get_protocol": [],
    "pto_ar_alloc_flags": [ctypes.POINTER(ctypes.c_void_p)],
    "pto_ar_free": [_P],
    "pto_ar_get_ipc_handle": [_P, _P, ctypes.POINTER(ctypes.c_longlong)],
    "pto_ar_open_ipc_handle": [_P, ctypes.POINTER(ctypes.c_void_p)],
    "pto_ar_close_ipc_handle": [_P],
    "pto_ar_blocks": [_L, _I],
    "pto_ar_hash_offset_words": [],
    "pto_ar_hash_ring": [],
    "pto_ar_param_hash": [_P, _P, _L, _I, _I, _P, _P],
    "pto_ar_read_words": [_P, _P, _L],
    "pto_ar_read_words_async": [_P, _P, _L, _P],
    "pto_ar_allreduce": [_P, _L, _L, _I, _I, _I, _P, _P, _P],
    "pto_ar_timeout_ticks": [],
    "pto_ar_allreduce_bf16": [_P, _L, _L, _I, _I, _I, _P, _P, _P],
    "pto_ar_role_sgd": [_P, _L, _L, _I, _I, _I, _P, _P, _I, _P, _P, _P, _F, _F, _F, _I, _L, _P],
    "pto_ar_oneshot_role_sgd": [_P, _L, _L, _I, _I, _I, _P, _P, _I, _P, _P, _P, _F, _F, _F, _I, _L, _I, _I, _L, _P,
                                _P],
    "pto_ar_oneshot_role_blocks": [_L, _I],
    "pto_ar_allreduce_sgd": [_P, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _F, _I, _L, _P, _L, _P, _I, _I, _L,
                             _P],
}


def _current_library() -> str:
    # build() is a no-op when the stamp matches the current sources, and
    # recompiles a stale library (e.g. sources edited after a build).
    try:
        return build(force=os.environ.get("PTO_REBUILD") == "1")
    except (OSError, subprocess.CalledProcessError):
        # Only a library built from exactly these sources may stand in
        # (e.g. hipcc missing on a run host): a stale one has launchers
        # whose argument lists no longer match _SIGS.
        if not is_current():
            raise
        return LIB_PATH


def lib():
    """Return the loaded ctypes library, building it on first use."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # PTO_HIP_LIB: load a library built from OTHER sources (A/B runs of
        # a kernel change in one GPU call: the baseline build sits next to
        # the current one); its launchers must match _SIGS.
        path = os.environ.get("PTO_HIP_LIB") or _current_library()
        L = ctypes.CDLL(path)
        for name, args in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
        return _lib


def loaded_path() -> str | None:
    return getattr(_lib, "_name", None) if _lib is not None else None


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
