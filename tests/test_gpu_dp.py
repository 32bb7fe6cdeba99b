"""The data-parallel training step (engine.TrainStep with more than one rank) on a real GPU, at
BASELINE.json configs[2]'s per-GPU shape: BetaVAE-H (beta 4, models/beta_vae.py:129-152), 32
images per rank.  Two ranks share cuda:0 over gloo (one box has one GPU; RCCL needs distinct
devices); the backward runs as HIP-graph segments per gradient bucket with each bucket's
all-reduce launched between them, and the loss terms ride in the last bucket.

Checked against the CPU oracle, not against another HIP run: each rank's shard through
oracle.train_step, the shard gradients averaged (DDP semantics, run.py:86), one Adam step.  Bars
are the single-GPU parity bars (test_gpu_parity_shapes.py): averaged gradients within max(1e-3,
3 x the oracle's own thread-count spread) relative norm per parameter (3e-3 floor BatchNorm affine), loss terms (the rank mean the reference logs
with sync_dist, experiment.py:55) within 1e-4, BatchNorm buffers = rank 0's shard statistics
(DDP broadcast_buffers), and the Adam update equal to the oracle's on every element whose
averaged gradient is not within noise of zero."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, WORLD, SEED, M_N, LR = 32, 2, 1265, 2.5e-4, 0.005


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank):
    from oracle import vae_oracle as O
    return O.make_inputs(B, 128, 100 + rank)


def _worker(rank, port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from oracle import vae_oracle as O
        from vae_amd.engine import FusedAdam, TrainStep
        from vae_amd.net import StepPlan, VAENet
        net = VAENet(latent_dim=128, dtype=torch.float32, device="cuda:0")
        net.load_reference_state_dict(O.make_params(O.vanilla_param_spec(), SEED))
        plan = StepPlan(net, B, loss="betaH", kld_weight=M_N, beta=4.0)
        step = TrainStep(net, plan, FusedAdam(net, lr=LR), graph=True, nbuckets=4)
        assert len(step.buckets) >= 2, step.buckets
        x, eps = _shard(rank)
        step(x.cuda(), eps.cuda())
        torch.cuda.synchronize()
        # numpy, not torch tensors: a torch CPU tensor crosses the queue as a shared-memory file
        # descriptor that dies with this process
        grads = {k: v.cpu().numpy() for k, v in net.layout.export_reference(plan.grads).items()}
        state = {k: v.cpu().numpy() for k, v in net.reference_state_dict().items()}
        q.put((rank, state, grads, step.loss_terms(), plan.out[:3].tolist()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None))


def test_data_parallel_betaH_matches_oracle_shard_mean():
    from oracle import vae_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, state, grads, terms, local = q.get(timeout=240)
        assert not isinstance(state, str), state
        state = {k: torch.from_numpy(v) for k, v in state.items()}
        grads = {k: torch.from_numpy(v) for k, v in grads.items()}
        res[r] = (state, grads, terms, local)
    for p in procs:
        p.join(timeout=60)
    from parity_util import grad_bar, oracle_with_spread
    sd = O.make_params(O.vanilla_param_spec(), SEED)
    shards, spreads = zip(*[oracle_with_spread("BetaVAE", sd, *_shard(r), M_N=M_N, lr=LR, loss_type="H", beta=4.0)
                            for r in range(WORLD)])
    spread = {k: max(sp[k] for sp in spreads) for k in spreads[0]}
    # both ranks hold the same averaged gradient, parameters and (broadcast) buffers
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k]), k
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    state, grads, terms, _ = res[0]
    # loss terms: rank mean (sync_dist) on both ranks; each rank's own terms match its shard
    for r in range(WORLD):
        for i, t in enumerate(("loss", "Reconstruction_Loss", "KLD")):
            want = sum(s["loss"][t] for s in shards) / WORLD
            assert abs(res[r][2][i] - want) <= 1e-4 * abs(want), (r, t, res[r][2][i], want)
            assert abs(res[r][3][i] - shards[r]["loss"][t]) <= 1e-4 * abs(shards[r]["loss"][t]), (r, t)
    gmean = {k: sum(s["grads"][k] for s in shards) / WORLD for k in shards[0]["grads"]}
    worst = 0.0
    for name, gr in gmean.items():
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue                                    # analytically zero under train-mode BN
        err = float((grads[name].double() - gr.double()).norm() / gr.double().norm())
        worst = max(worst, err)
        bound = grad_bar(name, spread)
        assert err < bound, (name, err, bound)
    print(f"DP betaH 2x{B}: worst averaged-gradient rel-norm {worst:.2e}")
    # one Adam step from zero state on the averaged gradient: lr * g / (|g| + eps) elementwise —
    # compared where the oracle's averaged gradient is clear of the noise floor (sign-stable) and
    # of Adam's eps: d/dg [g / (|g| + eps)] = eps / (|g| + eps)^2, so at |g| >= 1e-5 a relative
    # gradient error e moves the update by at most lr * 1e-3 * e
    for name, gr in gmean.items():
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue
        p0 = sd[name].double()
        want = p0 - LR * gr.double() / (gr.double().abs() + 1e-8)
        ok = (gr.abs() > 1e-2 * gr.abs().max()) & (gr.abs() > 1e-5)
        np.testing.assert_allclose(state[name].double()[ok].numpy(), want[ok].numpy(), rtol=0,
                                   atol=1e-6 + 1e-3 * LR, err_msg=name)
    for k, v in shards[0]["running"].items():           # rank 0's statistics (broadcast_buffers)
        np.testing.assert_allclose(state[k].numpy(), v.numpy(), rtol=1e-4, atol=1e-6, err_msg=k)
