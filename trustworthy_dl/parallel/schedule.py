"""Pipeline schedules of ``PipelineEngine`` (parallel/pipeline.py): the local in-process schedule
(every stage in one process, the deterministic simulation backend) and the distributed 1F1B
schedules (grouped exchanges, or latency-hiding async P2P on per-direction communicators), plus
the attacker's stage hooks they call.

The reference runs its "nodes" sequentially inside one process with no micro-batching and no
P2P (distributed_trainer.py:148-207); here they are real pipeline stages.
"""
from __future__ import annotations

import time
from collections import deque
from typing import Dict, List, Optional

import torch

from . import comm as p2p
from ..ops import stats as dstats
from ..ops.layers import defer_weight_grads
from ..runtime import progress
from ..runtime.commcheck import note_host_sync
from .stage import Stage


class ScheduleMixin:
    """Forward / backward schedules over M micro-batches (mixed into ``PipelineEngine``)."""

    def _pre_micro(self, node: int, st: Stage, i: int):
        if self.attacker is not None and hasattr(self.attacker, "before_micro_backward"):
            self.attacker.before_micro_backward(node, st.flat.grad, self.global_step, i, len(self._audit_batch))

    def _tamper_dx(self, node: int, dx: torch.Tensor, i: int) -> torch.Tensor:
        """The input gradient ``node`` sends upstream for micro-batch ``i`` (Byzantine backward hook)."""
        if self.attacker is not None and hasattr(self.attacker, "on_input_grad"):
            d2 = self.attacker.on_input_grad(node, dx, self.global_step, i, len(self._audit_batch))
            if d2 is not None:
                self._truth_now[node] = True
                return d2
        return dx

    # ------------------------------------------------------------------ attacks on a stage
    def _attack_params(self, node: int, st: Stage, truth: Dict[int, bool]):
        if self.attacker is not None and hasattr(self.attacker, "on_parameters"):
            if self.attacker.on_parameters(node, st.flat, self.global_step):
                truth[node] = True
        self._commit_master(node, st)   # the weights this step runs with (side stream)
        # the stage's weights are final for this step from here on: take the integrity checksum now,
        # on the verifier's side stream, overlapped with the forward / backward instead of serially
        # on the step's tail (_integrity_flag picks it up after finish_step joined the side stream)
        side = getattr(st.verifier, "side", None)
        if self.cfg.param_integrity and side is not None and st.flat.data.is_cuda:
            cur = torch.cuda.current_stream(st.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                st._early_checksum = dstats.checksum(st.flat.data)
            st._early_checksum.record_stream(cur)

    def _attack_output(self, node: int, y: torch.Tensor, truth: Dict[int, bool], micro: Optional[int] = None,
                       num_micro: Optional[int] = None) -> torch.Tensor:
        if self.attacker is not None and hasattr(self.attacker, "on_output"):
            y2 = self.attacker.on_output(node, y, self.global_step, micro, num_micro)
            if y2 is not None:
                truth[node] = True
                return y2
        return y

    def _attack_grads(self, node: int, st: Stage, truth: Dict[int, bool]):
        if self.attacker is not None and hasattr(self.attacker, "on_gradients"):
            if self.attacker.on_gradients(node, st.flat.grad, self.global_step):
                truth[node] = True

    # ------------------------------------------------------------------ local (in-process) schedule
    def _run_local(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        order = list(zip(self.plan.ranks, self.plan.ranges))
        M = len(inputs)
        for node, _ in order:
            self._attack_params(node, self.stages[node], truth)
        total = None
        bwd_audit = self._audit_now and self.cfg.audit_backward
        for i in range(M):
            x = inputs[i]
            watch = i == self._mon_idx
            y_copy = None   # the previous stage's recorded output: the next stage's recorded input when
            #                 it arrives unchanged (same device), kept once instead of twice
            for sidx, (node, _) in enumerate(order):
                st = self.stages[node]
                x = self._stage_input(x, st) if sidx == 0 else x.to(st.device, non_blocking=True)
                labels = targets[i].to(st.device, non_blocking=True) if st.computes_loss else None
                obs = st.output_observer() if watch else None
                rec = self._audit_rec.setdefault(node, {}).setdefault(i, {}) \
                    if self._audit_now and (i in self._audit_ms or self._targeted) else None
                if rec is not None:
                    rec["x"] = y_copy if y_copy is not None and y_copy.device == x.device else x.detach().clone()
                    if st.computes_loss:
                        rec["labels"] = labels
                if sidx > 0 and x.requires_grad:
                    # the input gradient this stage sends upstream (Byzantine-backward hook first, then
                    # the audit's copy of what was sent); registered before the previous stage's
                    # output-gradient capture below, so that capture sees the gradient as sent
                    def _dx_hook(g, node=node, i=i, rec=rec):
                        g2 = self._tamper_dx(node, g, i)
                        if rec is not None and bwd_audit:
                            rec["dx"] = g2.detach().clone()
                        return g2 if g2 is not g else None
                    x.register_hook(_dx_hook)
                    prec = self._audit_rec.get(order[sidx - 1][0], {}).get(i) if rec is not None and bwd_audit else None
                    if prec is not None:
                        def _dy_hook(g, prec=prec, rec=rec):
                            # runs after _dx_hook: the gradient as sent, already copied there
                            dx = rec.get("dx") if rec is not None else None
                            prec["dy"] = dx if dx is not None and dx.device == g.device else g.detach().clone()
                        x.register_hook(_dy_hook)
                with self.tracer.phase("fwd"):
                    y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1)
                if not st.computes_loss:
                    y = self._attack_output(node, y, truth, i, M)
                    if watch:
                        mon = y
                    y_copy = None
                    if rec is not None:
                        rec["y"] = y_copy = y.detach().clone()
                        if self._targeted:
                            rec["ystat"] = self._output_stat(rec["y"])
                if watch and mon is not None:
                    st.verifier.observe_output(mon)
                    if st.computes_loss and st.verifier.side is not None:
                        torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
                x = y
            loss = x / M
            for node, _ in order:
                self._pre_micro(node, self.stages[node], i)
            with self.tracer.phase("bwd_input"):
                loss.backward()
            for node, _ in order:
                self._commit_micro(node, self.stages[node], i)
            total = loss.detach() if total is None else total + loss.detach()
        return total

    # ------------------------------------------------------------------ distributed 1F1B schedule
    def _run_1f1b(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        if self.p2p_mode == "async":
            return self._run_1f1b_async(inputs, targets, truth)
        st = self.my_stage()
        if st is None:
            return None
        node = self.rank
        comm = self.comm
        M = len(inputs)
        S = self.plan.num_stages
        s = st.stage_id
        first, last = s == 0, s == S - 1
        self._attack_params(node, st, truth)
        self._audit_early_ship(st)
        in_shape, out_shape = self._boundary_shapes(st, inputs[0])
        act_dtype = self.dtype
        defer_w = self.cfg.defer_wgrad and not first
        warm = min(S - s - 1, M)
        rem = M - warm
        in_q: deque = deque()
        out_q: deque = deque()
        total = [None]
        waited0 = comm.wait_seconds
        keep_out = self._audit_now and self.cfg.audit_backward and not last   # loss-stage inputs + x cross-check
        self._audit_outputs: Dict[int, torch.Tensor] = {}

        def get_input(i):
            if first:
                return self._stage_input(inputs[i], st)
            progress.mark(f"step {self.global_step}: stage {s} grouped exchange with rank {comm.prev}")
            x, _ = comm.exchange(recv_prev=(in_shape, act_dtype))
            return x

        def fwd(i, x):
            if not first:
                x.requires_grad_(True)
            labels = targets[i].to(st.device, non_blocking=True) if last else None
            watch = i == self._mon_idx
            obs = st.output_observer() if watch else None
            if self._audit_now and not first:
                # every received input stays referenced until the audit (no copy): it is the previous
                # stage's output as seen here (audited here) and my input (the next stage audits me)
                self._audit_inputs[i] = x.detach()
            y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1 and not defer_w)
            if last:
                y = y / M
                total[0] = y.detach() if total[0] is None else total[0] + y.detach()
            else:
                y = self._attack_output(node, y, truth, i, M)
                if watch:
                    mon = y
                if keep_out:
                    self._audit_outputs[i] = y.detach()
            if watch and mon is not None:
                st.verifier.observe_output(mon)
                if last and st.verifier.side is not None:
                    # the CE backward rewrites the logits buffer in place
                    torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
            return y

        def bwd(bi, x, y, dy):
            """Input-gradient backward; the weight-gradient GEMMs are queued (ops.layers
            .defer_weight_grads) and run by the caller AFTER dx has been posted upstream."""
            self._pre_micro(node, st, bi)
            if dy is not None and self._audit_now:
                self._audit_recv_dy[bi] = dy
            with defer_weight_grads(defer_w) as dw:
                if last:
                    y.backward()
                else:
                    torch.autograd.backward(y, dy)
            dx = None
            if not first:
                dx = self._tamper_dx(node, x.grad, bi)
                if self._audit_now:
                    self._audit_sent_dx[bi] = dx
            dw.bi = bi
            return dx, dw

        def wgrad(dw):
            dw.run()
            self._commit_micro(node, st, dw.bi)

        def send_dx_then_w(dx, dw, recv_prev=None):
            h = comm.post(send_prev=dx, recv_prev=recv_prev)
            wgrad(dw)  # overlaps the transfer and the upstream stage's backward
            return comm.wait(h)[0]

        for i in range(warm):
            x = get_input(i)
            y = fwd(i, x)
            comm.exchange(send_next=y)
            in_q.append((i, x))
            out_q.append(y)
        x = get_input(warm) if rem > 0 else None
        for j in range(rem):
            i = warm + j
            y = fwd(i, x)
            if last:
                dy = None
            else:
                _, dy = comm.exchange(send_next=y, recv_next=(out_shape, act_dtype))
            in_q.append((i, x))
            out_q.append(y)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dx, dw = bwd(bi, x0, y0, dy)
            if j == rem - 1:
                if not first:
                    send_dx_then_w(dx, dw)
                else:
                    wgrad(dw)
            else:
                if first:
                    wgrad(dw)
                    x = get_input(i + 1)
                else:
                    x = send_dx_then_w(dx, dw, recv_prev=(in_shape, act_dtype))
        for _ in range(warm):
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dy = None
            if not last:
                _, dy = comm.exchange(recv_next=(out_shape, act_dtype))
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send_dx_then_w(dx, dw)
            else:
                wgrad(dw)
        self._comm_wait = comm.wait_seconds - waited0
        return total[0]

    def _run_1f1b_async(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        """1F1B with latency-hiding point-to-point transfers.

        Activations travel on one process group and activation gradients on another, so every
        communicator carries one-way traffic per neighbour pair in issue order (deadlock-free for
        any interleaving of the two directions).  Each receive is posted one compute phase ahead
        of its use — the next input before this stage's backward, the next output gradient before
        its forward — so the xGMI transfer overlaps compute instead of adding a full transfer
        latency to every pipeline hop (the grouped exchange serialises send and receive behind
        both neighbours' compute).  On each direction's stream a send is always issued before the
        next receive, so a ready send never queues behind a pending receive.  The compute stream
        never waits for a send; all sends are drained at the end of the step.  Weight gradients
        (B/W split) run after the input gradient is posted."""
        st = self.my_stage()
        if st is None:
            return None
        node = self.rank
        M = len(inputs)
        S = self.plan.num_stages
        s = st.stage_id
        first, last = s == 0, s == S - 1
        self._attack_params(node, st, truth)
        self._audit_early_ship(st)
        in_shape, out_shape = self._boundary_shapes(st, inputs[0])
        act_pg, grad_pg = self._dir_groups
        prev, nxt = self.comm.prev, self.comm.next
        dt = self.dtype
        warm = min(S - s - 1, M)
        rem = M - warm
        in_q: deque = deque()
        out_q: deque = deque()
        sends: List = []
        total = [None]
        waited = [0.0]
        defer_w = self.cfg.defer_wgrad and not first
        # my outputs stay referenced until the audit: the loss stage's inputs (I audit it) and the next
        # stage's inputs (its auditor compares the copies it receives with what I sent)
        keep_out = self._audit_now and self.cfg.audit_backward and not last   # loss-stage inputs + x cross-check
        self._audit_outputs: Dict[int, torch.Tensor] = {}

        step = self.global_step

        def post_recv(shape, src, group):
            buf = torch.empty(shape, dtype=dt, device=st.device)
            return p2p.irecv(buf, src, group=group), buf, src

        def take(h):
            progress.mark(f"step {step}: stage {s} waits for a P2P receive from rank {h[2]}")
            t0 = time.perf_counter()
            h[0].wait()
            waited[0] += time.perf_counter() - t0
            progress.mark(f"step {step}: stage {s} compute")
            return h[1]

        def post_x(i):
            return None if first or i >= M else post_recv(in_shape, prev, act_pg)

        def post_dy(i):
            return None if last or i >= M else post_recv(out_shape, nxt, grad_pg)

        def send(t, dst, group):
            sends.append(p2p.isend(t.contiguous(), dst, group=group))
            if len(sends) > 8:  # drop finished sends (their tensors are released)
                sends[:] = [w for w in sends if not w.is_completed()]

        def fwd(i, x):
            if not first:
                x.requires_grad_(True)
            labels = targets[i].to(st.device, non_blocking=True) if last else None
            watch = i == self._mon_idx
            obs = st.output_observer() if watch else None
            if self._audit_now and not first:
                # every received input stays referenced until the audit (no copy): it is the previous
                # stage's output as seen here (audited here) and my input (the next stage audits me)
                self._audit_inputs[i] = x.detach()
            y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1 and not defer_w)
            if last:
                y = y / M
                total[0] = y.detach() if total[0] is None else total[0] + y.detach()
            else:
                y = self._attack_output(node, y, truth, i, M)
                if watch:
                    mon = y
                if keep_out:
                    self._audit_outputs[i] = y.detach()
            if watch and mon is not None:
                st.verifier.observe_output(mon)
                if last and st.verifier.side is not None:
                    torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
            return y

        def bwd(bi, x, y, dy):
            self._pre_micro(node, st, bi)
            if dy is not None and self._audit_now:
                self._audit_recv_dy[bi] = dy
            with defer_weight_grads(defer_w) as dw:
                if last:
                    y.backward()
                else:
                    torch.autograd.backward(y, dy)
            dx = None
            if not first:
                dx = self._tamper_dx(node, x.grad, bi)
                if self._audit_now:
                    self._audit_sent_dx[bi] = dx
            return dx, dw

        def wgrad(bi, dw):
            dw.run()
            self._commit_micro(node, st, bi)

        def input_of(i, h):
            return self._stage_input(inputs[i], st) if first else take(h)

        tr = self.tracer
        if tr.enabled:
            fwd, bwd, take = tr.wrap("fwd", fwd), tr.wrap("bwd_input", bwd), tr.wrap("p2p_wait", take)

        x_h = post_x(0)
        for i in range(warm):                      # warm > 0 implies not last
            x = input_of(i, x_h)
            y = fwd(i, x)
            send(y, nxt, act_pg)
            x_h = post_x(i + 1)
            in_q.append((i, x))
            out_q.append(y)
        for j in range(rem):
            i = warm + j
            x = input_of(i, x_h)
            dy_h = post_dy(j)                      # arrives while this forward runs
            y = fwd(i, x)
            if not last:
                send(y, nxt, act_pg)
            x_h = post_x(i + 1)                    # arrives while the backward below runs
            in_q.append((i, x))
            out_q.append(y)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dy = None if last else take(dy_h)
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send(dx, prev, grad_pg)
            with tr.phase("bwd_weight"):
                wgrad(bi, dw)
        dy_h = post_dy(rem) if warm > 0 else None
        for c in range(warm):
            b = rem + c
            dy = take(dy_h)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send(dx, prev, grad_pg)
            dy_h = post_dy(b + 1)                  # after the send: no send queues behind it
            with tr.phase("bwd_weight"):
                wgrad(bi, dw)
        progress.mark(f"step {step}: stage {s} drains its P2P sends")
        t0 = time.perf_counter()
        for w in sends:
            w.wait()
        waited[0] += time.perf_counter() - t0
        self._comm_wait = waited[0]
        return total[0]

    def _boundary_shapes(self, st: Stage, sample_in: torch.Tensor):
        """Activation shapes entering / leaving this stage (exchanged once, then cached)."""
        key = (self.plan.version, tuple(sample_in.shape))
        cached = self._shape_cache.get(key)
        if cached is not None:
            return cached
        S = self.plan.num_stages
        s = st.stage_id
        hdr = torch.zeros(8, dtype=torch.int64, device=st.device)
        in_shape = None
        if s > 0:
            h, _ = self.comm.exchange(recv_prev=((8,), torch.int64))
            note_host_sync()
            in_shape = torch.Size([int(v) for v in h[1:1 + int(h[0])].tolist()])
            probe = torch.zeros(in_shape, dtype=self.dtype, device=st.device)
        else:
            probe = sample_in.to(st.device)
        out_shape = None
        if s < S - 1:
            was_training = st.module.training
            st.module.eval()  # shape probe must not touch BatchNorm running statistics
            with torch.no_grad():
                y, _ = st.forward(probe, None)
            st.module.train(was_training)
            out_shape = y.shape
            hdr[0] = len(out_shape)
            hdr[1:1 + len(out_shape)] = torch.tensor(list(out_shape), dtype=torch.int64)
            self.comm.exchange(send_next=hdr)
        self._shape_cache[key] = (in_shape, out_shape)
        return in_shape, out_shape
