"""GPT-2 built from the native ops, laid out as a flat list of pipeline-partitionable layers.

The reference asks ``ModelFactory.create_model('gpt2')`` for a HuggingFace-style model and
partitions ``model.transformer.h`` (distributed_trainer.py:118-135) — dropping embeddings,
final LayerNorm and LM head and any remainder layers.  This model keeps the HF
parameter names (``transformer.wte/wpe/h.N.{ln_1,attn.c_attn,attn.c_proj,ln_2,mlp.c_fc,mlp.c_proj}
/ln_f``; Conv1D weights stored [in, out]) and exposes ``pipeline_layers()``:
``[Embedding, Block x n_layer, Head]`` so a partitioner can place *every* layer, with the
embedding on the first stage and ``ln_f`` + tied LM head + cross-entropy on the last.

Vocabulary rows are padded to a multiple of 64 (50257 -> 50304) so logits rows are 16-byte
aligned and the LM-head GEMM tiles evenly; padded logits are masked out of the softmax, so the
function computed is exactly GPT-2's.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from .. import ops

GPT2_SIZES = {
    "tiny": dict(n_layer=2, n_embd=128, n_head=2),
    "mini": dict(n_layer=4, n_embd=256, n_head=4),
    "small": dict(n_layer=12, n_embd=768, n_head=12),
    "medium": dict(n_layer=24, n_embd=1024, n_head=16),
    "large": dict(n_layer=36, n_embd=1280, n_head=20),
    "xl": dict(n_layer=48, n_embd=1600, n_head=25),
}


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    pad_vocab_multiple: int = 64
    fused_block: bool = True  # ops/block.py single-node block; False = op-by-op autograd

    @classmethod
    def from_size(cls, size: str = "small", **kw) -> "GPT2Config":
        base = dict(GPT2_SIZES[size])
        base.update(kw)
        return cls(**base)

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return (self.vocab_size + m - 1) // m * m

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head


class Conv1D(nn.Module):
    """HF GPT-2 Conv1D: y = x @ weight + bias, weight stored [in, out]."""

    def __init__(self, nx: int, nf: int, act: Optional[str] = None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(nx, nf))
        self.bias = nn.Parameter(torch.zeros(nf))
        self.act = act

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, self.act)


class LayerNorm(nn.Module):
    def __init__(self, n: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.bias = nn.Parameter(torch.zeros(n))
        self.eps = eps

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.eps)


class GPT2Attention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        self.c_attn = Conv1D(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = Conv1D(cfg.n_embd, cfg.n_embd)

    def forward(self, x):
        return self.c_proj(ops.causal_attention(self.c_attn(x), self.n_head, causal=True))


class GPT2MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = Conv1D(cfg.n_embd, 4 * cfg.n_embd, act="gelu")
        self.c_proj = Conv1D(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x):
        return self.c_proj(self.c_fc(x))


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon)
        self.attn = GPT2Attention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon)
        self.mlp = GPT2MLP(cfg)
        self.fused = cfg.fused_block

    def forward(self, x):
        if self.fused and ops.fused_block_enabled(x.shape[-1], x.device):
            return ops.gpt2_block(x, self)  # one autograd node, residual adds fused (ops/block.py)
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class GPT2HalfBlock(nn.Module):
    """One residual half of a GPT2Block as its own pipeline unit: ``x + attn(ln_1(x))`` (part
    "attn") or ``x + mlp(ln_2(x))`` (part "mlp").  Shares the block's submodules, so parameter
    names inside the unit are the block's own (``ln_1.weight``, ``mlp.c_fc.weight`` ...).

    With half-block granularity a stage boundary may fall between a block's attention and MLP,
    which halves the partition granule (an MLP is ~0.6 of a block): an 8-stage GPT-2-medium split
    otherwise leaves whole-block stages of 4 against an ideal of ~3.5.  Both halves of a block on
    one stage still run as the single fused block op (parallel/stage.py pairs them)."""

    def __init__(self, block: GPT2Block, part: str, index: int):
        super().__init__()
        if part not in ("attn", "mlp"):
            raise ValueError(part)
        self.part = part
        self.block_index = index
        self.fused = block.fused
        if part == "attn":
            self.ln_1, self.attn = block.ln_1, block.attn
        else:
            self.ln_2, self.mlp = block.ln_2, block.mlp

    def forward(self, x):
        if self.part == "attn":
            return x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class FusedHalfPair:
    """Runs an (attn, mlp) pair of GPT2HalfBlock units of the same block as one fused block op.
    Not an nn.Module: it only borrows the two units' submodules (no parameter is registered twice)."""

    def __init__(self, attn_half: GPT2HalfBlock, mlp_half: GPT2HalfBlock):
        self.ln_1, self.attn = attn_half.ln_1, attn_half.attn
        self.ln_2, self.mlp = mlp_half.ln_2, mlp_half.mlp
        self._halves = (attn_half, mlp_half)
        self.fused = attn_half.fused

    def __call__(self, x):
        if self.fused and ops.fused_block_enabled(x.shape[-1], x.device):
            return ops.gpt2_block(x, self)
        return self._halves[1](self._halves[0](x))


class GPT2Embedding(nn.Module):
    """wte (padded vocab) + wpe; first pipeline layer. Input: token ids [B, T]."""
    takes_tokens = True

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd))

    def forward(self, ids):
        return ops.embedding(ids, self.wte, self.wpe)


class GPT2Head(nn.Module):
    """ln_f + tied LM head + softmax cross-entropy; last pipeline layer."""
    computes_loss = True

    def __init__(self, cfg: GPT2Config, wte: Optional[nn.Parameter] = None):
        super().__init__()
        self.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon)
        self.wte = wte if wte is not None else nn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd))
        self.vocab_size = cfg.vocab_size

    def logits(self, h):
        return ops.layers.linear_t(self.ln_f(h), self.wte)

    accepts_observer = True  # Stage passes its output monitor in (the logits buffer is reused)

    def forward(self, h, labels=None):
        observe = getattr(self, "_observe", None)
        if labels is None:
            logits = self.logits(h)
            self._last_logits = logits  # monitored output when the head is a stage on its own
            return logits
        # fused head: the logits buffer becomes dlogits inside the forward, so the monitor (if
        # any) is handed the logits before that and there is no _last_logits afterwards
        self._last_logits = None
        return ops.layers.lm_head_cross_entropy(self.ln_f(h), self.wte, labels, self.vocab_size, observe=observe)


class _Transformer(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.embed = GPT2Embedding(cfg)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])

    @property
    def wte(self):
        return self.embed.wte

    @property
    def wpe(self):
        return self.embed.wpe


class GPT2LMHeadModel(nn.Module):
    """Full model (single device / local simulation). ``forward(ids, labels)`` -> loss."""

    family = "gpt2"

    def __init__(self, cfg: GPT2Config, seed: Optional[int] = 0):
        super().__init__()
        self.config = cfg
        self.transformer = _Transformer(cfg)
        self.head = GPT2Head(cfg, wte=self.transformer.embed.wte)
        self.granularity = "block"
        self._halves: Optional[List[GPT2HalfBlock]] = None  # plain list: not registered twice
        self.reset_parameters(seed)

    def set_pipeline_granularity(self, granularity: str) -> None:
        """``"block"``: pipeline units are whole blocks; ``"half"``: attention and MLP halves."""
        if granularity not in ("block", "half"):
            raise ValueError(f"granularity must be 'block' or 'half', got {granularity!r}")
        self.granularity = granularity

    def reset_parameters(self, seed: Optional[int] = 0):
        """GPT-2 init (normal 0.02; residual projections scaled by 1/sqrt(2L)); deterministic per seed."""
        g = torch.Generator().manual_seed(seed if seed is not None else 0)
        std = self.config.initializer_range
        with torch.no_grad():
            for name, p in self.named_parameters():
                if name.endswith("ln_1.weight") or name.endswith("ln_2.weight") or name.endswith("ln_f.weight"):
                    p.fill_(1.0)
                elif name.endswith("bias"):
                    p.zero_()
                else:
                    s = std / math.sqrt(2 * self.config.n_layer) if name.endswith("c_proj.weight") else std
                    p.copy_(torch.randn(p.shape, generator=g) * s)
            self.transformer.embed.wte[self.config.vocab_size:].zero_()

    def pipeline_layers(self) -> List[nn.Module]:
        if self.granularity == "half":
            if self._halves is None:
                self._halves = [GPT2HalfBlock(b, part, i) for i, b in enumerate(self.transformer.h)
                                for part in ("attn", "mlp")]
            return [self.transformer.embed, *self._halves, self.head]
        return [self.transformer.embed, *self.transformer.h, self.head]

    # time per token of each unit relative to 24 n^2 dense-GEMM FLOPs: the attention core and the
    # pointwise kernels run far from the GEMM rate, the LM head GEMMs close to it.  Calibrated on
    # MI355X from per-unit fwd+bwd timings of GPT-2-medium at T=1024, micro-batch 16
    # (scripts/time_units.py, profiles/r1_gpt2m_unit_times.jsonl): attention half 0.50, MLP half
    # 0.57, LM head 2.9 and embedding 0.14 block-times.
    _ATTN_CORE_WEIGHT = 1.64     # causal attention FLOPs (4 T n) relative to GEMM FLOPs
    _POINTWISE_PER_BLOCK = 0.12  # LayerNorms, bias-GELU, residual adds: fraction of the block GEMMs
    _EMBED_PER_BLOCK = 0.14      # gather fwd + wte/wpe scatter-add bwd

    def layer_costs(self, seq_len: int) -> List[float]:
        """Relative fwd+bwd time per pipeline unit (per token)."""
        c = self.config
        n, T = c.n_embd, seq_len
        pw = self._POINTWISE_PER_BLOCK * 24 * n * n
        attn = 8 * n * n + self._ATTN_CORE_WEIGHT * 4 * T * n + 0.4 * pw  # qkv + proj GEMMs + core
        mlp = 16 * n * n + 0.6 * pw                                         # fc + proj GEMMs + GELU
        head = 2 * n * c.padded_vocab + 10 * c.padded_vocab  # LM head GEMM + softmax/CE passes
        embed = self._EMBED_PER_BLOCK * (attn + mlp)
        units = [attn, mlp] if self.granularity == "half" else [attn + mlp]
        return [embed] + [float(u) for u in units] * c.n_layer + [float(head)]

    def forward(self, ids, labels=None):
        h = self.transformer.embed(ids)
        for blk in self.transformer.h:
            h = blk(h)
        return self.head(h, labels)

    def num_parameters(self, exclude_padding: bool = True) -> int:
        n = sum(p.numel() for p in self.parameters())
        if exclude_padding:
            n -= (self.config.padded_vocab - self.config.vocab_size) * self.config.n_embd
        return n
