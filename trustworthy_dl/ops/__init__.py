"""Compute ops: native gfx950 HIP kernels for GPU tensors, PyTorch references for CPU tensors."""
from ._lib import available as native_available, lib as native_lib, LIB_PATH  # noqa: F401
from .layers import layer_norm, linear, causal_attention, embedding, cross_entropy  # noqa: F401
from .block import gpt2_block, fused_block_enabled  # noqa: F401
from .conv import conv_bn_act, conv_bn_chain, conv2d, global_avg_pool, max_pool2d  # noqa: F401
from .attack import AttackMode, inject_  # noqa: F401
from . import stats  # noqa: F401
