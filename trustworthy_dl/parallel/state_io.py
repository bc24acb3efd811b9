"""Checkpoint state of ``PipelineEngine`` (utils/checkpoint.py): stage-local state dicts in the
reference's ``model_partitions[node]`` layout (distributed_trainer.py:448-463), optimizer and
verifier state, trust state, and layer-wise loading across plans.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ..ops.layers import bump_weight_generation


class StateIOMixin:
    """Checkpoint state (mixed into ``PipelineEngine``)."""

    # ================================================================== checkpoint state
    def stage_state_dicts(self) -> Dict[int, Dict[str, torch.Tensor]]:
        """model_partitions[node] = stage-local state dict (fp32 master weights + buffers)."""
        out = {}
        for node, st in self.stages.items():
            sd = {}
            for i, n in enumerate(st.flat.names):
                sd[n] = st.flat.view(st.flat.master, i).detach().cpu().clone()
            for n, b in st.module.named_buffers():
                sd[n] = b.detach().cpu().clone()
            out[node] = sd
        return out

    def optimizer_state_dicts(self) -> Dict[int, Dict]:
        return {node: st.flat.state_dict() for node, st in self.stages.items()}

    def verifier_state_dicts(self) -> Dict[int, Dict]:
        return {node: st.verifier.state_dict() for node, st in self.stages.items()}

    def trust_state(self) -> Dict[str, torch.Tensor]:
        return {"values": self.t_values.cpu(), "counts": self.t_counts.cpu(), "status": self.t_status.cpu()}

    def load_trust_state(self, sd, partial: bool = False):
        """``partial``: the saved job had a different node count; the first ``len`` entries are
        restored, the rest keep their initial values."""
        for dst, key in ((self.t_values, "values"), (self.t_counts, "counts"), (self.t_status, "status")):
            src = sd[key]
            if partial:
                k = min(dst.numel(), src.numel())
                dst[:k].copy_(src[:k])
            else:
                dst.copy_(src)

    def load_layer_states(self, layers: Dict[int, Dict], step: int):
        """Fill the local stages layer by layer (fp32 master + AdamW moments + buffers) from a saved
        job whose plan differs from this one (utils/checkpoint.load_checkpoint).  Tied parameters
        that the saved stage stored under another layer of their tie group are found there."""
        alias: Dict[Tuple[int, str], List[Tuple[int, str]]] = {}
        for grp in self.ties:
            for m in grp:
                alias[m] = [o for o in grp if o != m]

        def find(kind, li, attr):
            ent = layers.get(li, {}).get(kind, {})
            if attr in ent:
                return ent[attr]
            for lj, aj in alias.get((li, attr), []):
                ent = layers.get(lj, {}).get(kind, {})
                if aj in ent:
                    return ent[aj]
            raise KeyError(f"checkpoint holds no {kind[:-1]} '{attr}' of layer {li}")

        self.t_taint.zero_()      # weights replaced from a checkpoint
        for node, st in self.stages.items():
            a, _ = st.layer_range
            for i, name in enumerate(st.flat.names):
                k, attr = name.split(".", 1)
                m, ea, eas = find("params", a + int(k), attr)
                st.flat.view(st.flat.master, i).copy_(m)
                st.flat.view(st.flat.exp_avg, i).copy_(ea)
                st.flat.view(st.flat.exp_avg_sq, i).copy_(eas)
            for name, b in st.module.named_buffers():
                k, attr = name.split(".", 1)
                b.copy_(find("buffers", a + int(k), attr))
            st.flat.step_count = int(step)
            if st.flat.data is not st.flat.master:
                st.flat.data.copy_(st.flat.master)
            st.param_checksum = None
        bump_weight_generation()
        self._invalidate_mirrors()   # every rank loads: mirrors are re-seeded from the loaded state
        self.refresh_shadows()    # the loaded weights are the new trusted copy

    def load_stage_states(self, model_sd: Dict[int, Dict], optim_sd: Dict[int, Dict],
                          verifier_sd: Optional[Dict[int, Dict]] = None):
        self.t_taint.zero_()      # weights replaced from a checkpoint
        missing = [n for n in self.stages if n not in optim_sd and n not in model_sd]
        if missing:
            raise KeyError(f"checkpoint holds no state for local stage node(s) {missing}")
        for node, st in self.stages.items():
            if node in optim_sd:
                st.flat.load_state_dict(optim_sd[node])
            elif node in model_sd:
                for i, n in enumerate(st.flat.names):
                    if n in model_sd[node]:
                        st.flat.view(st.flat.master, i).copy_(model_sd[node][n])
                if st.flat.data is not st.flat.master:
                    st.flat.data.copy_(st.flat.master)
            if node in model_sd:
                for n, b in st.module.named_buffers():
                    if n in model_sd[node]:
                        b.copy_(model_sd[node][n])
            if verifier_sd and node in verifier_sd:
                st.verifier.load_state_dict(verifier_sd[node])
            st.param_checksum = None  # weights legitimately replaced
        self._invalidate_mirrors()
        self.refresh_shadows()        # the loaded weights are the new trusted copy
