"""Loader for the native HIP kernel library (``trustworthy_dl/_native/libtdl_kernels.so``).

The kernels are plain HIP C++ (csrc/*.hip) compiled for gfx950 by ``build_native.py`` and
exported through a C ABI: every entry point takes device pointers, sizes and the HIP
stream to launch on, and returns a ``hipError_t``.  Using a C ABI (instead of a torch C++
extension) keeps the build to seconds per file and makes every launch capturable in a
HIP graph (the caller passes the capturing stream).

Policy: a CUDA(HIP) tensor ALWAYS goes to the native kernel.  If the library is missing
on a machine with a GPU the op raises — there is no silent eager fallback.  CPU tensors
use the PyTorch reference implementations in the op modules (used by the CPU/gloo tests).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_LIB_NAME = "libtdl_kernels.so"
_HERE = os.path.dirname(os.path.abspath(__file__))
# TDL_NATIVE_LIB: another build of the same library (interleaved A/B runs of a kernel change on one
# box, scripts/gpu_*_ab.sh); the in-tree build otherwise
LIB_PATH = os.environ.get("TDL_NATIVE_LIB") or os.path.normpath(os.path.join(_HERE, "..", "_native", _LIB_NAME))

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


class NativeLibraryMissing(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load (once) and return the native kernel library; raise loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryMissing(
                    f"{LIB_PATH} not found: run `python build_native.py` (hipcc --offload-arch=gfx950)")
            _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(_lib)
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (NativeLibraryMissing, OSError):
        return False


def stream_ptr(device: Optional[torch.device] = None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def check(err: int, name: str):
    if err != 0:
        raise RuntimeError(f"native kernel {name} failed with hipError {err}")


_P, _I, _L, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

class LayoutBatch(ctypes.Structure):
    """csrc/conv.hip LayoutBatch (passed by value): up to 32 conv weights' layout jobs."""
    MAX = 32
    _fields_ = [("w", ctypes.c_void_p * 32), ("krsc", ctypes.c_void_p * 32), ("crsk", ctypes.c_void_p * 32),
                ("Cout", ctypes.c_int * 32), ("C", ctypes.c_int * 32), ("Cp", ctypes.c_int * 32),
                ("RS", ctypes.c_int * 32), ("n", ctypes.c_int)]


class TransposeBatch(ctypes.Structure):
    """csrc/norm_act.hip TransposeBatch (passed by value): up to 64 bf16 [R, C] -> [C, R] jobs;
    ``first[j]`` = first 64 x 64 tile of job j, ``first[n]`` = total tiles."""
    MAX = 64
    _fields_ = [("inp", ctypes.c_void_p * 64), ("out", ctypes.c_void_p * 64), ("R", ctypes.c_int * 64),
                ("C", ctypes.c_int * 64), ("first", ctypes.c_int * 65), ("n", ctypes.c_int)]


class BnFin(ctypes.Structure):
    """csrc/conv.hip BnFin: a folded BatchNorm finalized by the producing convolution's kernels."""
    _fields_ = [("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("save_mean", ctypes.c_void_p),
                ("save_rstd", ctypes.c_void_p), ("upd_mean", ctypes.c_void_p), ("upd_var", ctypes.c_void_p),
                ("pro", ctypes.c_void_p), ("zero_sums", ctypes.c_void_p), ("count", ctypes.c_int64),
                ("eps", ctypes.c_float), ("momentum", ctypes.c_float)]


# name -> argtypes (restype is int for all)
_SIGNATURES = {
    # norm_act.hip
    "tdl_layernorm_fwd": [_P, _P, _P, _P, _P, _P, _I, _I, _F, _P],
    "tdl_layernorm_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P],
    "tdl_layernorm_bwd_ws_floats": [_I, _I],
    "tdl_layernorm_bwd_res": [_P] * 11 + [_I, _I, _P, _P],
    "tdl_add_bias_ln_fwd": [_P] * 11 + [_I, _I, _F, _P],
    "tdl_bias_gelu_fwd": [_P, _P, _P, _I, _I, _P],
    "tdl_bias_gelu_bwd": [_P, _P, _P, _P, _P, _I, _I, _P, _P],
    "tdl_embedding_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "tdl_embedding_bwd": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "tdl_add_into_f32": [_P, _P, _L, _I, _P],
    "tdl_conv_weight_layouts": [_P, _P, _P, _I, _I, _I, _I, _P],
    "tdl_conv_dgrad_bnsums": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "tdl_bn_act_bwd_pro_summed": [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "tdl_global_avgpool_fwd": [_P, _P, _I, _I, _I, _P],
    "tdl_global_avgpool_bwd": [_P, _P, _I, _I, _I, _P],
    "tdl_maxpool_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "tdl_maxpool_bwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "tdl_colsum_f32": [_P, _I, _I, _I, _P, _P],
    "tdl_colsum_bf16": [_P, _P, _I, _I, _P, _P],
    "tdl_transpose_bf16": [_P, _P, _I, _I, _P],
    "tdl_transpose_bf16_batch": [TransposeBatch, _P],
    # xent.hip
    "tdl_xent_fwd": [_P, _P, _P, _P, _I, _I, _I, _P],
    "tdl_xent_bwd": [_P, _P, _P, _P, _P, _I, _I, _I, _F, _P],
    "tdl_xent_fused": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    "tdl_scale_bf16": [_P, _P, _P, _L, _P],
    # optim.hip
    "tdl_adamw_flat": [_P, _P, _P, _P, _P, _L, _F, _F, _F, _F, _F, _F, _F, _P, _I, _P],
    "tdl_fill_f32": [_P, _L, _F, _P],
    "tdl_copy_if": [_P, _P, _P, _L, _P],
    "tdl_splitk_reduce_add": [_P, _P, _I, _L, _P],
    # stats.hip
    "tdl_tensor_stats": [_P, _I, _L, _P, _P, _I, _P],
    "tdl_grad_stats": [_P, _P, _P, _I, _P, _L, _F, _I, _P, _I, _I, _P],
    "tdl_grad_stats_ws_bytes": [_I, _I],
    "tdl_grad_stats_partial": [_P, _P, _P, _I, _I, _I, _I, _F, _P, _I, _P],
    "tdl_grad_stats_reduce_partial": [_P, _P, _I, _L, _L, _P, _P, _I, _I, _I, _I, _F, _P, _I, _P],
    "tdl_grad_stats_final": [_P, _P, _I, _P, _L, _I, _P, _I, _I, _P],
    "tdl_grad_sumsq": [_P, _P, _I, _P, _P, _P, _P],
    "tdl_gram_ws_bytes": [],
    "tdl_cosine_gram": [_P, _I, _L, _I, _P, _P, _P],
    "tdl_zscore_detect": [_P, _P, _P, _I, _I, _I, _F, _I, _I, _I, _I, _F, _F, _P, _P],
    "tdl_trust_update": [_P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _P],
    "tdl_kl_div_softmax": [_P, _P, _I, _I, _P, _P],
    "tdl_stats_workspace_bytes": [],
    "tdl_checksum_bf16": [_P, _L, _P, _P, _P],
    "tdl_verify_features": [_P, _P, _P, _P, _P],
    "tdl_verify_finish": [_P, _P],
    "tdl_verify_args_bytes": [],
    # attack.hip
    "tdl_attack_inject": [_P, _I, _L, _I, _F, ctypes.c_uint64, ctypes.c_uint64, _P],
    # attention.hip
    "tdl_attn_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _P],
    "tdl_attn_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _P],
    # gemm.hip
    "tdl_gemm": [_P] * 6 + [_I] * 10 + [_L, _P],
    "tdl_gemm_wgrad_grouped": [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "tdl_gemm_set_timestamps": [_P],
    # audit.hip
    "tdl_b2s_nodes": [_P, _L, _L, _I, _I, _I, _I, _P, _L, _P],
    "tdl_b2s_leaves_l1": [_P, _L, _I, _L, _L, _P, _L, _P],
    "tdl_b2s_top_max_in": [],
    "tdl_b2s_top": [_P, _L, _I, _I, _I, _I, _P, _L, _P],
    "tdl_keyed_sketch_ws_floats": [_L],
    "tdl_keyed_sketch": [_P, _L, _I, _P, _L, _L, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _I, _P],
    "tdl_contrib_snap": [_P, _P, _P, _L, _P],
    "tdl_absdiff_max": [_P, _P, _L, _L, _P, _P],
    # conv.hip / bn.hip
    "tdl_conv_nt": [_P] * 5 + [_I] * 12 + [_P],
    "tdl_conv_stats_ws_floats": [_I, _I],
    "tdl_conv_ws_floats": [_I, _I, _I, _I],
    "tdl_conv_wgrad": [_P] * 4 + [_I] * 12 + [_P],
    "tdl_bn_act_fwd": [_P] * 13 + [_L, _I, _F, _F, _I, _P],
    "tdl_bn_bwd_ws_floats": [_I],
    "tdl_bn_act_bwd": [_P] * 12 + [_L, _I, _I, _P],
    "tdl_bn_bwd_part_floats": [_I],
    "tdl_bn_finalize": [_P] * 9 + [_L, _I, _F, _F, _P],
    "tdl_bn_act_bwd_pro": [_P] * 11 + [_L, _I, _I, _P],
    "tdl_conv_nt_pro": [_P] * 5 + [_I] * 11 + [_P, _P],
    "tdl_conv_wgrad_pro": [_P] * 4 + [_I] * 12 + [_P, _P],
    "tdl_conv_weight_layouts_batch": [LayoutBatch, _P],
    "tdl_conv_fwd_bn": [_P] * 5 + [_I] * 11 + [_P, ctypes.POINTER(BnFin), ctypes.POINTER(ctypes.c_int), _P],
}


def _declare(l: ctypes.CDLL):
    for name, argtypes in _SIGNATURES.items():
        fn = getattr(l, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int64 if name.endswith(("_bytes", "_floats")) else ctypes.c_int


# Debug mode (race detection): ``TDL_SYNC_LAUNCH=1`` synchronises the device after every
# native launch and checks the sticky HIP error, so an asynchronous fault is reported at the kernel
# that caused it (the HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL=3 idea, for our own entry points).
SYNC_LAUNCH = os.environ.get("TDL_SYNC_LAUNCH", "0") not in ("", "0")


def set_sync_launch(on: bool) -> None:
    global SYNC_LAUNCH
    SYNC_LAUNCH = bool(on)


def call(name: str, *args):
    fn = getattr(lib(), name)
    check(fn(*args), name)
    if SYNC_LAUNCH:
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # pragma: no cover - device fault path
            raise RuntimeError(f"native kernel {name} faulted: {e}") from e


DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
