"""The data-parallel VQ-VAE training step (engine.TrainStep over vq.VQStepPlan with more than one
rank) on a real GPU: two ranks share cuda:0 over gloo, each with its own shard; the backward runs
as HIP-graph segments per gradient bucket (38.85 MB of fp32 gradients, codebook included), each
bucket's all-reduce launched (waitable) between them — with the weight gradients on the plan's
side stream (concurrent=True) and without.

Checked against the CPU oracle teacher-forced with each rank's own code indices (the VQ index
rule, tests/test_gpu_vq.py): shard gradients averaged (DDP, run.py:86), loss terms the rank mean
(sync_dist, experiment.py:55), every rank holding the same averaged gradient and parameters, and
the one Adam step equal to the oracle's where the gradient is clear of noise.  fp32 parity mode;
bars as the single-GPU VQ test (gradients within 1e-3 relative norm)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, WORLD, SEED, LR = 8, 2, 1265, 0.005


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank):
    return torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(300 + rank))


def _worker(rank, port, concurrent, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from oracle import vae_oracle as O
        from vae_amd.engine import FusedAdam, TrainStep
        from vae_amd.vq import VQNet, VQStepPlan
        net = VQNet(dtype=torch.float32, device="cuda:0")
        net.load_reference_state_dict(O.make_params(O.vq_param_spec(), SEED))
        plan = VQStepPlan(net, B, beta=0.25, concurrent=concurrent)
        step = TrainStep(net, plan, FusedAdam(net, lr=LR), graph=True, nbuckets=4)
        assert len(step.buckets) >= 2, step.buckets
        step(_shard(rank).cuda())
        torch.cuda.synchronize()
        grads = {k: v.cpu().numpy() for k, v in net.layout.export_reference(plan.grads).items()}
        state = {k: v.cpu().numpy() for k, v in net.reference_state_dict().items()}
        q.put((rank, state, grads, step.loss_terms(), plan.out[:3].tolist(), plan.indices.cpu().numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None, None))


@pytest.mark.parametrize("concurrent", [False, True])
def test_data_parallel_vq_matches_oracle_shard_mean(concurrent):
    from oracle import vae_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, concurrent, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, state, grads, terms, local, idx = q.get(timeout=240)
        assert not isinstance(state, str), state
        res[r] = ({k: torch.from_numpy(v) for k, v in state.items()}, {k: torch.from_numpy(v) for k, v in grads.items()},
                  terms, local, torch.from_numpy(idx))
    for p in procs:
        p.join(timeout=60)
    sd = O.make_params(O.vq_param_spec(), SEED)
    shards = [O.train_step("VQVAE", sd, _shard(r), M_N=0.0, lr=LR, vq_beta=0.25, vq_indices=res[r][4], do_adam=False)
              for r in range(WORLD)]
    for k in res[0][0]:
        assert torch.equal(res[0][0][k], res[1][0][k]), k
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    state, grads = res[0][0], res[0][1]
    for r in range(WORLD):
        for i, t in enumerate(("loss", "Reconstruction_Loss", "VQ_Loss")):
            want = sum(float(s["loss"][t]) for s in shards) / WORLD
            assert abs(res[r][2][i] - want) <= 1e-4 * abs(want), (r, t, res[r][2][i], want)
            own = float(shards[r]["loss"][t])
            assert abs(res[r][3][i] - own) <= 1e-4 * abs(own), (r, t)
    gmean = {k: sum(s["grads"][k] for s in shards) / WORLD for k in shards[0]["grads"]}
    worst = 0.0
    for name, gr in gmean.items():
        err = float((grads[name].double() - gr.double()).norm() / gr.double().norm())
        worst = max(worst, err)
        assert err < 1e-3, (name, err)
    print(f"DP VQ 2x{B} concurrent={concurrent}: worst averaged-gradient rel-norm {worst:.2e}")
    for name, gr in gmean.items():
        p0 = sd[name].double()
        want = p0 - LR * gr.double() / (gr.double().abs() + 1e-8)
        ok = (gr.abs() > 1e-2 * gr.abs().max()) & (gr.abs() > 1e-5)
        np.testing.assert_allclose(state[name].double()[ok].numpy(), want[ok].numpy(), rtol=0,
                                   atol=1e-6 + 1e-3 * LR, err_msg=name)
