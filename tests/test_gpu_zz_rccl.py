"""The RCCL branch of the data-parallel step (dp.allreduce_mean's ReduceOp.AVG, dp.py; run.py:86
DDP) on the one GPU a test box has: a world of one rank over the "nccl" backend (RCCL), with the
step forced onto its bucketed path (engine.TrainStep(force_buckets=True): backward HIP-graph
segments per gradient bucket, one RCCL all-reduce launched after each, the loss terms riding in
the last bucket, rank 0's BatchNorm buffers broadcast).  Two ranks cannot share a device under
RCCL, so the multi-rank arithmetic is covered by the gloo tests (test_gpu_dp.py, test_dp_gloo.py; this file
sorts last so that its RCCL process group initialises after every single-process test has run);
this one checks that the RCCL calls run inside the step's stream order and leave the step's
result unchanged: against the one-graph, collective-free path (fp32 parity mode, VanillaVAE B=16)
the first step's gradients within 1e-3 relative norm + 1e-6 (the bucketed plan batches its weight
gradients per segment and the weight-gradient atomics add in run-dependent order: measured 3.2e-5 to
1.2e-4 between runs, decoder.1.0.weight / decoder.3.0.weight;
a second step's gradients differ by up to 1.2e-4 as Adam amplifies that noise on near-zero
gradients), the Adam update of every element whose gradient is clear of that noise within 1e-5
(measured 1.2e-6 at a 1e-3 x max cut, decoder.1.0.weight; the step is lr = 5e-3), the
BatchNorm buffers within 1e-4, the loss terms of two steps within 1e-4 — a
broken exchange (a bucket missed, summed twice or raced by the next segment) is an O(1) error."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, SEED, M_N, LR = 16, 1265, 2.5e-4, 0.005


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(force, x, eps):
    from oracle import vae_oracle as O
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet
    net = VAENet(latent_dim=128, dtype=torch.float32, device="cuda:0")
    net.load_reference_state_dict(O.make_params(O.vanilla_param_spec(), SEED))
    plan = StepPlan(net, B, kld_weight=M_N)
    step = TrainStep(net, plan, FusedAdam(net, lr=LR), graph=True, nbuckets=4, force_buckets=force)
    if force:
        assert step.comm is not None and len(step.buckets) >= 2, step.buckets
    else:
        assert step.comm is None
    step(x, eps)
    torch.cuda.synchronize()
    terms = [step.loss_terms()]
    grads = {k: v.cpu().numpy() for k, v in net.layout.export_reference(plan.grads).items()}
    state = {k: v.cpu().numpy() for k, v in net.reference_state_dict().items()}
    step(x, eps)                          # a second step from the updated parameters and Adam state
    torch.cuda.synchronize()
    terms.append(step.loss_terms())
    return grads, state, terms, len(step.buckets)


def _worker(port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
        assert dist.get_backend() == "nccl"
        from oracle import vae_oracle as O
        x, eps = O.make_inputs(B, 128, 7)
        x, eps = x.cuda(), eps.cuda()
        ga, sa, ta, nb = _run(True, x, eps)
        gb, sb, tb, _ = _run(False, x, eps)
        dist.barrier()
        dist.destroy_process_group()
        q.put((ga, sa, ta, gb, sb, tb, nb))
    except Exception:
        import traceback
        q.put((traceback.format_exc(),) + (None,) * 6)


def _err(a, b, rel):
    """norm(a - b) against rel * norm(b) + 1e-6: the absolute term covers gradients that are zero in
    exact arithmetic (a conv bias in front of a BatchNorm: 1e-8-sized rounding either way, their
    difference norm ~1e-7 between the two summation orders); returns (error, bound)."""
    d = float(np.linalg.norm((a.astype(np.float64) - b.astype(np.float64)).ravel()))
    n = float(np.linalg.norm(b.astype(np.float64).ravel()))
    return d, rel * n + 1e-6


def test_rccl_bucketed_step_matches_one_graph_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    ga, sa, ta, gb, sb, tb, nb = q.get(timeout=240)
    p.join(timeout=60)
    assert not isinstance(ga, str), ga
    assert nb >= 2
    for k in gb:                          # the first step's gradients
        d, bound = _err(ga[k], gb[k], 1e-3)
        assert d <= bound, (k, d, bound)
    # parameters after it: Adam's first step moves every element by lr * g / (|g| + eps), i.e. by
    # lr * sign(g) wherever |g| >> eps, so the two runs must agree exactly on every element whose
    # gradient is clear of the summation-order noise (elements near zero may take the step with
    # the other sign; parameters whose gradient is zero in exact arithmetic — the conv biases in
    # front of a BatchNorm — are all noise and not compared)
    for k in gb:
        g = np.abs(gb[k].astype(np.float64))
        if g.max() < 1e-6:
            continue
        clear = g > 1e-2 * g.max()
        assert clear.mean() > 0.1, (k, clear.mean())
        dmax = float(np.abs(sa[k].astype(np.float64) - sb[k].astype(np.float64))[clear].max())
        assert dmax <= 1e-5, (k, dmax)    # (lr = 5e-3 per element: a wrong exchange moves lr-sized)
    # buffers (BatchNorm running statistics): the same batch statistics either way
    for k in sb:
        if k not in gb and sb[k].dtype.kind == "f":
            d, bound = _err(sa[k], sb[k], 1e-4)
            assert d <= bound, (k, d, bound)
    np.testing.assert_allclose(np.array(ta), np.array(tb), rtol=1e-4, atol=0)
