"""Fused training step: step_begin -> forward -> ELBO -> backward -> [grad all-reduce] -> Adam.

Replaces Lightning's loop around experiment.VAEXperiment.training_step (experiment.py:45-86)
plus torch.optim.Adam (experiment.py:308-311) for the hot path.  One step is a fixed launch
sequence on one stream; `TrainStep(graph=True)` captures it into HIP graphs so a step costs
one or two graph launches from the host.  Data parallelism (DDP semantics of run.py:86:
per-rank BatchNorm statistics, gradient mean over ranks) all-reduces the flat gradient
buffer with RCCL between the backward graph and the optimizer graph.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib as L
from .dp import BucketedAllReduce, broadcast_buffers, final_prefix, plan_buckets
from .net import BATCH_FN, VAENet, call_one


class FusedAdam:
    """torch.optim.Adam semantics (lerp first moment, bias-corrected) over the flat buffer;
    also refreshes the bf16 weight copy in the same pass.  step and lr are device scalars."""

    def __init__(self, net: VAENet, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 m: Optional[torch.Tensor] = None, v: Optional[torch.Tensor] = None):
        self.net = net
        # m / v may be given: a torch.optim.Adam's exp_avg / exp_avg_sq of the same flat
        # parameter, so that optimizer's state (checkpoints) IS this one (experiment.GraphedSteps)
        self.m = m if m is not None else torch.zeros_like(net.params)
        self.v = v if v is not None else torch.zeros_like(net.params)
        self.step = torch.zeros(1, dtype=torch.int32, device=net.device)
        self.lr = torch.full((1,), float(lr), dtype=torch.float32, device=net.device)
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay

    def set_lr(self, lr: float):
        self.lr.fill_(float(lr))

    def apply_deferred(self, grads: torch.Tensor, slabs, elbo, stream=None, lo: int = 0, hi: Optional[int] = None):
        """apply() with the weight-gradient reductions the backward deferred (L.deferred_take) done in
        the same launch (vae_adam_step_ex): each reduced gradient is written into `grads` before its
        elements' update, and a deferred loss is evaluated by one extra workgroup.  [lo, hi): the
        elements this launch updates (a multiple of 4 apart from 0; the descriptors must lie inside)."""
        net = self.net
        if len(slabs) > L.SLAB_MAX:
            raise ValueError(f"{len(slabs)} deferred reductions > {L.SLAB_MAX}")
        hi = net.params.numel() if hi is None else hi
        if lo % 4 or not 0 <= lo < hi <= net.params.numel():
            raise ValueError(f"apply_deferred range [{lo}, {hi})")
        ex = self.__dict__.setdefault("_ex", {})
        a = ex.get(lo) or ex.setdefault(lo, L.AdamArgs())
        a.n, a.p, a.g = hi - lo, net.params.data_ptr() + 4 * lo, grads.data_ptr() + 4 * lo
        a.m, a.v = self.m.data_ptr() + 4 * lo, self.v.data_ptr() + 4 * lo
        a.step, a.lr = self.step.data_ptr(), self.lr.data_ptr()
        a.beta1, a.beta2, a.eps, a.weight_decay = self.betas[0], self.betas[1], self.eps, self.weight_decay
        a.p_lowp = net.lowp.data_ptr() + 2 * lo if net.lowp is not None else None
        a.nslab = len(slabs)
        for i, sl in enumerate(slabs):
            a.slab[i] = sl
        a.has_elbo = 1 if elbo is not None else 0
        if elbo is not None:
            a.elbo = elbo
        L.call("vae_adam_step_ex", ctypes.byref(a), stream if stream is not None else L.stream_ptr())

    def apply(self, grads: torch.Tensor, stream=None, refresh_swaps: bool = True):
        """One Adam step over the flat parameters (writes the bf16 copy).  refresh_swaps=False leaves
        the swapped-axes weight copies stale (net.swaps_stale) for a caller that refreshes them at the
        start of its next step (TrainStep: inside vae_step_begin_ex)."""
        net = self.net
        L.call("vae_adam_step", net.params.numel(), net.params.data_ptr(), grads.data_ptr(), self.m.data_ptr(),
               self.v.data_ptr(), self.step.data_ptr(), self.lr.data_ptr(), self.betas[0], self.betas[1], self.eps,
               self.weight_decay, net.lowp.data_ptr() if net.lowp is not None else None,
               stream if stream is not None else L.stream_ptr())
        if getattr(net, "swap_descs", None) is not None:
            if refresh_swaps:
                net.refresh_swaps(stream)
            else:
                net.swaps_stale = True


PAD_FNS = ("vae_nchw_to_nhwc_pad", "vae_pad_channels")


def begin_args(plan, step: torch.Tensor):
    """vae_step_begin_ex arguments for a plan: its zero region and the step counter, plus the image
    and weight padding calls that head its forward list (they run inside the same launch).
    Returns (args, number of leading forward calls it replaces)."""
    a = L.StepBeginArgs(zero=plan.zero.data_ptr(), bytes=plan.zero.numel() * 4, step=step.data_ptr(),
                        dtype=plan.net.dcode)
    k = npad = 0
    for fn, arg in plan.fwd_calls:
        if fn == "vae_nchw_to_nhwc_pad" and not a.x:
            a.dtype, a.n, a.c, a.h, a.w, a.cp, a.x, a.y = arg
        elif fn == "vae_pad_channels" and npad < L.PAD_MAX and arg[0] == a.dtype:
            _, rows, c, cp, src, dst = arg
            a.pad[npad] = L.PadDesc(rows=rows, c=c, cp=cp, src=src, dst=dst)
            npad += 1
        else:
            break
        k += 1
    a.npad = npad
    # the swapped-axes weight copies the bf16 GEMMs read (net.swap_descs), refreshed in the same
    # launch from the weights the previous step's optimizer wrote
    sw = getattr(plan.net, "swap_descs", None)
    if isinstance(sw, ctypes.Array) and 0 < len(sw) <= L.SWAP_MAX:      # (VQNet: several arrays)
        a.nswap = len(sw)
        for i in range(len(sw)):
            a.swap[i] = sw[i]
    return a, k


class TrainStep:
    """One full training step of a plan (VanillaVAE family: net.StepPlan; VQ-VAE: vq.VQStepPlan)
    on fixed-shape device buffers.

    Inputs live in `plan.x` (NCHW fp32 images) and `plan.eps` (N(0,1) noise, the reference's
    torch.randn_like at vanilla_vae.py:116); write them before calling, or pass tensors — or let the
    step draw eps on the device (device_eps=seed: Philox in the fused bottleneck kernel).
    With more than one rank the backward is cut into segments at gradient-bucket boundaries
    (dp.plan_buckets); each bucket's RCCL all-reduce is launched as soon as its segment is
    queued, so it runs on the communication stream while the rest of the backward computes."""

    def __init__(self, net, plan, opt: FusedAdam, *, graph: bool = True, process_group=None,
                 nbuckets: int = 2, device_eps: Optional[int] = None, force_buckets: bool = False,
                 graph_comm: bool = True, begin_ex: bool = True, defer_reductions: bool = True,
                 overlap: bool = True, comm_dtype: torch.dtype = torch.float32, split_adam: bool = True):
        self.net, self.plan, self.opt = net, plan, opt
        # device_eps = seed: the forward draws eps itself every step (StepPlan.use_device_eps, keyed
        # by the optimizer's step counter) — the reference's per-step randn_like inside the step
        self.device_eps = (device_eps is not None and hasattr(plan, "use_device_eps")
                           and plan.use_device_eps(opt.step, device_eps))
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.use_graph = graph
        self.segments = []                      # (call range) of the backward per bucket
        # force_buckets: the bucketed path (segment graphs, one all-reduce per bucket, the buffer
        # broadcast) at world size 1 too — how the one-GPU tests run the RCCL branch
        if self.world > 1 or (force_buckets and self.world == 1 and dist.is_available() and dist.is_initialized()):
            raw = getattr(plan, "bwd_calls_raw", plan.bwd_calls)
            self.buckets = plan_buckets(raw, plan.grads, net.layout, nbuckets)
            if hasattr(plan, "batch_wgrads"):
                # the weight gradients of each bucket's segment as one batch at its end
                ends = plan.batch_wgrads([b[0] for b in self.buckets])
                self.buckets = [(e, s, t) for e, (_, s, t) in zip(ends, self.buckets)]
            # the last bucket also carries the loss terms (plan.metrics sits right after the
            # gradients): their rank mean is the reference's log_dict(sync_dist=True) at no extra
            # collective (experiment.py:55)
            e, s, _ = self.buckets[-1]
            mo = plan.metrics.data_ptr() - plan.zero.data_ptr()
            self.buckets[-1] = (e, s, mo // 4 + plan.metrics.numel())
            self.comm = BucketedAllReduce(plan.zero, self.buckets, process_group)
        else:
            self.buckets = [(len(plan.bwd_calls), 0, plan.grads.numel())]
            self.comm = None
        # graph_comm: the bucket all-reduces (RCCL) and the buffer broadcast captured into ONE graph
        # with the backward segments and the optimizer — each all-reduce on a communication stream
        # forked after its segment and joined before Adam — so a step is one replay, with no host
        # round trip per bucket.  Needs the "nccl" (RCCL) backend (gloo: host-issued); checked bit for
        # bit against the host-issued path at world size 1 (tests/test_gpu_zz_rccl.py).
        # nbuckets = 2 by default (round 6): the first bucket's weight gradients run on the overlap
        # stream (below), so its all-reduce hides behind the encoder's backward.  Round 5, without
        # that stream, measured one bucket best at one rank (0.483 ms in-graph vs 0.542 with two:
        # the second grouped weight-gradient launch sat on the critical path, profiles/r5_notes.md).
        self.graph_comm = (graph_comm and graph and self.comm is not None
                           and dist.get_backend(process_group) == "nccl")
        self.comm_stream = torch.cuda.Stream(device=net.device) if self.graph_comm else None
        # overlap (in-graph exchange, two or more buckets): the weight-gradient batch that closes a
        # bucket's backward segment runs on a stream of its own, forked from the segment's data-
        # gradient chain; the bucket's all-reduce waits for it there, while the next segment's data
        # gradients go on — the exchange of the decoder's gradients overlaps the encoder's backward
        # (DDP's hook-driven overlap, run.py:86), and the batch itself is off the critical path.
        # Each overlapped batch gets a workspace of its own (the main chain's is reused meanwhile).
        self.overlap = bool(overlap and self.graph_comm and len(self.buckets) > 1)
        # comm_dtype=torch.bfloat16 (in-graph exchange only; opt-in): each bucket is rounded to bf16,
        # all-reduced (AVG) in bf16 and widened back into the fp32 gradients Adam reads — half the
        # bytes over xGMI; the parity mode keeps fp32 (the reference's DDP all-reduces fp32)
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"comm_dtype {comm_dtype}")
        self.comm_dtype = comm_dtype if self.graph_comm else torch.float32
        self._comm_bufs = ([torch.empty(b1 - b0, dtype=torch.bfloat16, device=net.device) for _, b0, b1 in self.buckets]
                           if self.comm_dtype == torch.bfloat16 else None)
        self.wg_stream = torch.cuda.Stream(device=net.device) if self.overlap else None
        self._wg_ws = []
        self._wg_forked = False
        if self.overlap:
            lo = 0
            for end, _, _ in self.buckets[:-1]:
                seg = plan.bwd_calls[lo:end]
                if seg and seg[-1][0] == BATCH_FN:
                    b = seg[-1][1]
                    need = b.workspace_size()
                    ws = torch.empty(max(1, (need + 3) // 4), dtype=torch.float32, device=net.device)
                    b.workspace, b.workspace_bytes = (ws.data_ptr(), ws.numel() * 4) if need > 0 else (None, 0)
                    self._wg_ws.append(ws)
                lo = end
        self.graphs = []
        self.g_opt: Optional[torch.cuda.CUDAGraph] = None
        self.stream = torch.cuda.Stream(device=net.device)
        # the step's head (zeroing, step count, image and weight padding) as one launch;
        # begin_ex=False keeps vae_step_begin + the padding calls (tests/test_gpu_routes.py)
        self._begin = begin_args(plan, opt.step) if begin_ex else None
        self._begin_swaps = self._begin is not None and self._begin[0].nswap > 0
        # one rank: the backward's weight-gradient slab reductions (and the loss fused into the head
        # backward) run inside the optimizer launch (StepPlan.defer_reductions, vae_adam_step_ex);
        # with more ranks the gradients must be complete before their all-reduce
        self.deferred = (self.comm is None and defer_reductions and hasattr(plan, "defer_reductions")
                         and plan.defer_reductions())
        self._slabs, self._elbo = [], None
        # one rank, the decoder's weight gradients on the plan's side stream (StepPlan(wg_overlap=True)):
        # the optimizer splits at the gradients final once that batch has run (their prefix of the
        # buffer, ordered by backward completion) — Adam over the prefix runs on the side stream right
        # behind the batch, beside the encoder's backward; Adam over the rest on the main stream
        self._adam_split = 0
        if self.deferred and split_adam and getattr(plan, "wg_overlap", False) and getattr(plan, "side", None) is not None:
            si = next((i for i, (fn, ref) in enumerate(plan.bwd_calls)
                       if fn == BATCH_FN and getattr(ref, "side", False)), None)
            if si is not None:
                t = final_prefix(plan.bwd_calls, si, plan.grads, net.layout)
                if 0 < t < plan.grads.numel() and t % 4 == 0:
                    self._adam_split = t

    # -------------------------------------------------------------- eager pieces
    def _segment(self, k: int):
        """Segment k of the step: k == 0 also runs step_begin and the forward."""
        p = self.plan
        st = L.stream_ptr()
        if k == 0:
            skip = 0
            if self._begin is not None:
                args, skip = self._begin
                L.call("vae_step_begin_ex", args, st)
                if self._begin_swaps:
                    self.net.swaps_stale = False        # (refreshed by that launch)
            else:
                L.call("vae_step_begin", p.zero.data_ptr(), p.zero.numel() * 4, self.opt.step.data_ptr(), st)
            if p.loss_kind == L.LOSS_BETA_B:
                p.num_iter.add_(1.0)
            p._run(p.fwd_calls[skip:], st)
            if self.comm is not None and not getattr(p, "elbo_in_head", False):
                p.metrics.copy_(p.out)
        lo = 0 if k == 0 else self.buckets[k - 1][0]
        if self.deferred:
            L.call("vae_deferred_reset")
        seg = p.bwd_calls[lo:self.buckets[k][0]]
        self._wg_forked = False
        if self.overlap and k < len(self.buckets) - 1 and seg and seg[-1][0] == BATCH_FN:
            # the segment's weight gradients on the overlap stream, behind its data gradients
            p._run(seg[:-1], st)
            ws = self.wg_stream
            ws.wait_stream(torch.cuda.current_stream())
            call_one(BATCH_FN, seg[-1][1], ws.cuda_stream)
            self._wg_forked = True
        else:
            p._run(seg, st)
        if self.deferred:
            # (the same pointers at every run: each deferring call has a workspace of its own)
            self._slabs, self._elbo = L.deferred_take()
            self._keep_written(p)
        if k == 0 and self.comm is not None and getattr(p, "elbo_in_head", False):
            # the loss terms come from the head backward (vae_head_args.elbo), the first call of
            # segment 0's backward: copied behind it, reduced with the last bucket as before
            p.metrics.copy_(p.out)

    def _keep_written(self, p):
        """The gradients the deferred calls write whole (their reductions' destinations and the
        single-slice weight gradients: every descriptor) need no zeroing at the step head
        (vae_step_begin_args.keep): the step-begin launch leaves them out from the next step on."""
        if self._begin is None:
            return
        a = self._begin[0]
        base, end = p.zero.data_ptr(), p.zero.data_ptr() + p.zero.numel() * 4
        n = 0
        for sl in self._slabs:
            if sl.dst is None or not base <= sl.dst < end or n >= len(a.keep):
                continue
            a.keep[n] = L.KeepRange(off=sl.dst - base, bytes=sl.count * 4)
            n += 1
        a.nkeep = n

    def _opt(self):
        # with the swapped copies refreshed by the next step's head, the optimizer skips its own pass
        if self.deferred and self._adam_split:
            t, g = self._adam_split, self.plan.grads
            end = g.data_ptr() + 4 * t
            head = [sl for sl in self._slabs if sl.dst < end]
            tail = [sl for sl in self._slabs if sl.dst >= end]
            if any(sl.dst + 4 * sl.count > end for sl in head):
                raise RuntimeError("deferred reduction across the optimizer split")
            side, main = self.plan.side, torch.cuda.current_stream()
            # (the side stream's last work is the decoder's weight-gradient batch; the forward and the
            # backward calls before it were queued behind the fork)
            self.opt.apply_deferred(g, head, self._elbo, side.cuda_stream, 0, t)
            self.opt.apply_deferred(g, tail, None, main.cuda_stream, t)
            main.wait_stream(side)
        elif self.deferred:
            self.opt.apply_deferred(self.plan.grads, self._slabs, self._elbo, L.stream_ptr())
        if self.deferred:
            if getattr(self.net, "swap_descs", None) is not None:
                if self._begin_swaps:
                    self.net.swaps_stale = True
                else:
                    self.net.refresh_swaps(L.stream_ptr())
            return
        self.opt.apply(self.plan.grads, L.stream_ptr(), refresh_swaps=not self._begin_swaps)

    def _capture(self):
        # warm up on a side stream (allocations, lazy init), then capture
        s = self.stream
        s.wait_stream(torch.cuda.current_stream())
        state = (self.net.params.clone(), self.net.running.clone(), self.opt.m.clone(), self.opt.v.clone(),
                 self.opt.step.clone(), self.plan.num_iter.clone())
        with torch.cuda.stream(s):
            for k in range(len(self.buckets)):
                self._segment(k)
            if self.overlap:
                s.wait_stream(self.wg_stream)
            self._opt()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # restore what the warm-up step changed
        self.net.params.copy_(state[0]); self.net.running.copy_(state[1]); self.opt.m.copy_(state[2])
        self.opt.v.copy_(state[3]); self.opt.step.copy_(state[4]); self.plan.num_iter.copy_(state[5])
        self.net.sync_lowp()
        self.graphs = []
        if self.graph_comm:
            cs = self.comm_stream
            with torch.cuda.stream(cs):         # communicators up before the capture records them
                dist.all_reduce(torch.zeros(1, device=self.net.device), group=self.pg)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for k in range(len(self.buckets)):
                    self._segment(k)
                    _, b0, b1 = self.buckets[k]
                    cs.wait_stream(s)                   # this segment's gradients are complete
                    if self._wg_forked:
                        cs.wait_stream(self.wg_stream)  # (its weight gradients: the overlap stream)
                    with torch.cuda.stream(cs):
                        grad = self.plan.zero[b0:b1]
                        if self._comm_bufs is not None:
                            buf = self._comm_bufs[k]
                            buf.copy_(grad)
                            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.pg)
                            grad.copy_(buf)
                        else:
                            dist.all_reduce(grad, op=dist.ReduceOp.AVG, group=self.pg)
                with torch.cuda.stream(cs):
                    broadcast_buffers(self.net.running, self.pg)
                s.wait_stream(cs)
                if self.overlap:
                    s.wait_stream(self.wg_stream)
                self._opt()
            self.graphs.append(g)
            self.g_opt = None
            torch.cuda.synchronize()
            return
        if self.comm is None:
            # one rank: the whole step (forward, backward and the optimizer) is one graph, one
            # launch from the host — two graphs per step left an ~8.7 us gap between them
            # (profiles/r3a: the replay of the optimizer graph behind the backward graph)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._segment(0)
                self._opt()
            self.graphs.append(g)
            self.g_opt = None
            torch.cuda.synchronize()
            return
        for k in range(len(self.buckets)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._segment(k)
            self.graphs.append(g)
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, stream=s):
            self._opt()
        torch.cuda.synchronize()

    def __call__(self, x: Optional[torch.Tensor] = None, eps: Optional[torch.Tensor] = None):
        if x is not None:
            self.plan.x.copy_(x)
        if eps is not None:
            if self.device_eps:
                raise ValueError("this step draws eps on the device (device_eps); do not pass eps")
            self.plan.eps.copy_(eps.reshape(self.plan.eps.shape))
        if self.use_graph and not self.graphs:
            self._capture()
        if self.graph_comm:
            self.graphs[0].replay()                     # segments, all-reduces, broadcast, Adam
            if self._begin_swaps:
                self.net.swaps_stale = True
            self.net.num_batches_tracked += 1
            return
        for k in range(len(self.buckets)):
            if self.use_graph:
                self.graphs[k].replay()
            else:
                self._segment(k)
            if self.comm is not None:
                self.comm.launch(k)
        bcast = None
        if self.comm is not None:
            self.comm.wait()
            # rank 0's BatchNorm running statistics, off the critical path: the broadcast runs on
            # the communication stream while the optimizer step (which does not read them) runs
            bcast = broadcast_buffers(self.net.running, self.pg, async_op=True)
        if self.use_graph:
            if self.g_opt is not None:
                self.g_opt.replay()
        else:
            self._opt()
        if bcast is not None:
            bcast.wait()                 # before the next step's forward updates them
        if self._begin_swaps:
            self.net.swaps_stale = True  # the swapped copies follow at the next step's head
        self.net.num_batches_tracked += 1

    def loss_terms(self):
        """[loss, Reconstruction_Loss, KLD|VQ_Loss] of the last step: the mean over ranks with more
        than one (what the reference logs, experiment.py:55), else this rank's."""
        return (self.plan.metrics if self.comm is not None else self.plan.out)[:3].tolist()
