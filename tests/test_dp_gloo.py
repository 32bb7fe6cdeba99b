"""Data-parallel exchange (vae_amd/dp.py) on CPU with gloo, world_size 2.

Each rank runs the oracle's VanillaVAE step on its shard of the batch (per-rank BatchNorm, as
DDP), writes the gradients into the native flat buffer, and averages them with the product's
bucketed all-reduce; the result must equal the mean of both shards' gradients (DDP semantics,
run.py:86), and the BatchNorm running statistics must follow rank 0 (broadcast_buffers)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(O, sd, x, eps, layout, r, world):
    B = x.shape[0] // world
    o = O.train_step("VanillaVAE", sd, x[r * B:(r + 1) * B], eps[r * B:(r + 1) * B], M_N=0.5, do_adam=False)
    full = dict(sd)
    full.update(o["grads"])
    full.update({k: v for k, v in o["running"].items()})
    flat = torch.zeros(layout.total)
    run = torch.zeros(layout.bn_total)
    layout.load_reference(flat, run, full)
    return flat, run


def _fake_bwd_calls(layout, flat):
    """Backward launch list stand-in: one call per parameter in layout (= backward) order, its
    gradient pointer into `flat` (what plan_buckets reads from the real argument structs)."""
    from vae_amd import _lib as L
    import ctypes
    calls = []
    for p in sorted(layout.params, key=lambda q: q.offset):
        a = L.ConvArgs()
        a.dw = flat.data_ptr() + 4 * p.offset
        calls.append(("vae_conv2d_bwd_filter", ctypes.byref(a)))
    return calls


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(2)
        from oracle import vae_oracle as O
        from vae_amd.dp import BucketedAllReduce, broadcast_buffers, plan_buckets
        from vae_amd.layout import vanilla_layout
        layout = vanilla_layout(3, 128, [32, 64, 128, 256, 512])
        sd = O.make_params(O.vanilla_param_spec(), 1265)
        x, eps = O.make_inputs(4 * world, 128, 1265)
        mine, run = _shard_grads(O, sd, x, eps, layout, rank, world)
        want = sum(_shard_grads(O, sd, x, eps, layout, r, world)[0] for r in range(world)) / world
        run0 = _shard_grads(O, sd, x, eps, layout, 0, world)[1]
        calls = _fake_bwd_calls(layout, mine)
        buckets = plan_buckets(calls, mine, layout, nbuckets=4)
        assert len(buckets) >= 2 and buckets[0][1] == 0 and buckets[-1][2] == layout.total
        for a, b in zip(buckets, buckets[1:]):
            assert a[2] == b[1] and a[0] < b[0]
        comm = BucketedAllReduce(mine, buckets)
        for k in range(len(buckets)):
            comm.launch(k)
            # the launch returns at once with a handle (the step queues its next backward segment
            # here): a bucket is never scaled before its wait — never already the mean
            assert len(comm.works) == k + 1
        comm.wait()
        # allreduce_mean on gloo: an in-flight handle, mean only after wait()
        from vae_amd.dp import allreduce_mean
        t = torch.full((1 << 16,), float(rank + 1))
        h = allreduce_mean(t, async_op=True)
        assert h is not None
        before = float(t[0])
        assert before in (float(rank + 1), float(sum(range(1, world + 1))))   # not yet scaled
        #  torch Work semantics: a poller sees completion without calling wait(), and
        # whenever is_completed() is True the tensor already holds the mean
        import time
        t0 = time.time()
        while not h.is_completed():
            assert time.time() - t0 < 60, "is_completed() never turned True without wait()"
            time.sleep(0.001)
        assert torch.equal(t, torch.full_like(t, sum(range(1, world + 1)) / world))
        h.wait()                             # idempotent: no second scale
        assert h.is_completed()
        assert torch.equal(t, torch.full_like(t, sum(range(1, world + 1)) / world))
        broadcast_buffers(run)
        err = float((mine - want).abs().max() / want.abs().max())
        assert err < 1e-6, err
        assert torch.equal(run, run0)
        # the step's asynchronous form (engine.TrainStep): each rank's forward moved its own
        # statistics, the broadcast runs beside other work, and after the wait every rank holds
        # rank 0's — two steps in a row
        for step in range(2):
            run.add_(float(rank + 1) * (step + 1))
            ref = run.clone()
            dist.broadcast(ref, src=0)                 # what rank 0 holds now
            work = broadcast_buffers(run, async_op=True)
            other = torch.ones(1000).cumsum(0)         # the optimizer step's stand-in
            work.wait()
            assert torch.equal(run, ref), step
            assert float(other[-1]) == 1000.0
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bucketed_gradient_mean_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
