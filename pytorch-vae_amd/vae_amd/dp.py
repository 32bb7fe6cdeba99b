"""Data parallelism of the training step: DDP semantics of the reference's Lightning DDPPlugin
(run.py:86, trainer gpus from configs/vae/vae.yaml:23) on one process per GPU.

  * every rank runs forward/backward on its own shard of the global batch, BatchNorm statistics
    per rank (no SyncBatchNorm — DDP's default);
  * gradients are averaged over ranks (DDP all-reduce mean) — here the flat fp32 gradient
    buffer, in buckets that are launched as soon as the backward has finished them, so RCCL
    over xGMI runs on its own stream while the rest of the backward continues (the layout
    orders parameters by backward completion, decoder output layer first: layout.py);
  * BatchNorm running statistics follow rank 0 (DDP broadcast_buffers=True).

Buckets are planned from the step's launch list: a parameter is final after the last call that
writes its gradient (dw / db / BatchNorm affine outputs), so the flat prefix that is complete
after call i is known on the host before anything runs.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

# fields of the argument structs that point into the gradient buffer
_GRAD_FIELDS = ("dw", "db", "dcodebook", "dw1", "db1", "dw2", "db2")
_XF_GRAD_FIELDS = ("dgamma_out", "dbeta_out")


def _written_grad_ptrs(arg) -> List[int]:
    out = []
    for f in _GRAD_FIELDS:
        if hasattr(arg, f):
            v = getattr(arg, f)
            if v:
                out.append(int(v))
    for name in ("xf", "dy_xf"):             # vae_bn_args (mode 1) / a weight-gradient call's
        xf = getattr(arg, name, None)        # BN_DY transform: dγ, dβ outputs
        if xf is not None:
            for f in _XF_GRAD_FIELDS:
                v = getattr(xf, f)
                if v:
                    out.append(int(v))
    fin = getattr(arg, "bn_finalize", None)  # a BatchNorm finalisation fused into this call
    if fin:
        out += _written_grad_ptrs(fin.contents)
    return out


def last_writers(calls: Sequence, grads: torch.Tensor, layout):
    """The parameters in buffer order and, for each, the index of the last call of `calls` that
    writes its gradient (-1: none) — read from the gradient pointers of every call's arguments."""
    base = grads.data_ptr()
    params = sorted(layout.params, key=lambda p: p.offset)
    starts = [p.offset for p in params]
    last = [-1] * len(params)
    for i, (fn, ref) in enumerate(calls):
        if ref is None:
            continue
        if hasattr(ref, "args"):                # a batch of weight-gradient calls (net.FilterBatch)
            ptrs = [p for a in ref.args for p in _written_grad_ptrs(a)]
            ptrs += [r[4] for f, r in getattr(ref, "after", []) if f == "vae_unpad_accumulate"]
        elif isinstance(ref, tuple):            # scalar-argument entry points
            ptrs = [ref[4]] if fn == "vae_unpad_accumulate" else []
        else:
            ptrs = _written_grad_ptrs(ref._obj if hasattr(ref, "_obj") else ref)
        for ptr in ptrs:
            off = (ptr - base) // 4
            if not 0 <= off < layout.total:
                continue
            # parameter containing this offset
            lo, hi = 0, len(params) - 1
            while lo < hi:
                mid = (lo + hi + 1) // 2
                if starts[mid] <= off:
                    lo = mid
                else:
                    hi = mid - 1
            last[lo] = max(last[lo], i)
    return params, last


def final_prefix(calls: Sequence, upto: int, grads: torch.Tensor, layout) -> int:
    """Elements of the leading run of parameters whose gradients are final once calls[:upto + 1]
    have run (no later call writes them)."""
    params, last = last_writers(calls, grads, layout)
    t = 0
    for k, p in enumerate(params):
        if last[k] > upto:
            break
        t = params[k + 1].offset if k + 1 < len(params) else layout.total
    return t


def plan_buckets(calls: Sequence, grads: torch.Tensor, layout, nbuckets: int = 4,
                 min_bucket_bytes: int = 1 << 20) -> List[Tuple[int, int, int]]:
    """Split the backward launch list into segments whose completion finishes a flat prefix of
    the gradient buffer.  Returns [(end_call, start_elem, end_elem)]: after calls[:end_call]
    have run, grads[start_elem:end_elem] is final.  The last bucket ends at len(calls) and
    covers the rest of the buffer."""
    params, last = last_writers(calls, grads, layout)
    # complete[i] = number of leading params final after call i
    total = layout.total
    target = max(min_bucket_bytes // 4, total // max(1, nbuckets))
    buckets, start = [], 0
    prefix_last = -1
    order_last = []
    for k in range(len(params)):
        prefix_last = max(prefix_last, last[k])
        order_last.append(prefix_last)          # call index after which params[:k+1] are final
    for k in range(len(params)):
        end_elem = params[k + 1].offset if k + 1 < len(params) else total
        if end_elem - start >= target and k + 1 < len(params) and order_last[k] + 1 < len(calls):
            buckets.append((order_last[k] + 1, start, end_elem))
            start = end_elem
    buckets.append((len(calls), start, total))
    # segments must be non-decreasing in end_call; merge any that are not
    merged: List[Tuple[int, int, int]] = []
    for b in buckets:
        if merged and b[0] <= merged[-1][0]:
            merged[-1] = (merged[-1][0], merged[-1][1], b[2])
        else:
            merged.append(b)
    return merged


class _MeanWork:
    """A gloo SUM all-reduce still in flight, whose wait() also applies the 1/world scale (gloo has
    no AVG): the caller keeps queueing work (the next backward segments) until it waits, as with
    RCCL's AVG handle."""

    def __init__(self, work, t: torch.Tensor, world: int):
        self.work, self.t, self.world = work, t, world
        self.scaled = False

    def wait(self):
        if not self.scaled:
            self.work.wait()
            self.t.div_(self.world)
            self.scaled = True
        return True

    def is_completed(self):
        """torch Work semantics: True once the all-reduce has finished (a poller never needs wait()).
        The 1/world scale is applied here on the first True, so whenever this returns True the
        tensor holds the rank mean, as with RCCL's AVG handle."""
        if not self.scaled and self.work.is_completed():
            self.wait()
        return self.scaled


def allreduce_mean(t: torch.Tensor, group=None, async_op: bool = False):
    """DDP gradient averaging of one bucket: RCCL AVG on GPU, gloo SUM then 1/world.  async_op:
    returns a handle to wait on (for gloo the scaling happens in its wait()), None otherwise."""
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group, async_op=async_op)
    work = dist.all_reduce(t, group=group, async_op=async_op)
    if async_op:
        return _MeanWork(work, t, world)
    t.div_(world)
    return None


def broadcast_buffers(running: torch.Tensor, group=None, async_op: bool = False):
    """DDP broadcast_buffers=True: every rank takes rank 0's BatchNorm running statistics.
    async_op: returns the work handle (the caller waits before the next forward reads them —
    on RCCL a stream-ordered wait, so the optimizer step runs meanwhile)."""
    src = dist.get_global_rank(group, 0) if group is not None else 0
    return dist.broadcast(running, src=src, group=group, async_op=async_op)


class BucketedAllReduce:
    """Launches the bucket all-reduces of one step as the backward segments complete and waits
    for them before the optimizer."""

    def __init__(self, grads: torch.Tensor, buckets: List[Tuple[int, int, int]], group=None):
        self.grads, self.buckets, self.group = grads, buckets, group
        self.works = []

    def launch(self, k: int):
        _, s, e = self.buckets[k]
        w = allreduce_mean(self.grads[s:e], self.group, async_op=True)
        if w is not None:
            self.works.append(w)

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
