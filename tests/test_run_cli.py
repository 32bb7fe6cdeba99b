"""run.py counterpart (vae_amd/run.py) host logic on CPU: flags and YAML overrides as the
reference's run.py:18-51, per-rank batch shards, Lightning-format checkpoints."""
import os

import torch
import yaml

from vae_amd import run as R


def _cfg(tmp_path, **over):
    cfg = {"model_params": {"name": "VanillaVAE", "in_channels": 3, "latent_dim": 128},
           "data_params": {"data_path": "Data/", "train_batch_size": 8, "val_batch_size": 8, "patch_size": 64,
                           "num_workers": 0},
           "exp_params": {"LR": 0.005, "weight_decay": 0.0, "scheduler_gamma": 0.95, "kld_weight": 1e-8,
                          "manual_seed": 1265},
           "trainer_params": {"gpus": [0], "max_epochs": 3},
           "logging_params": {"save_dir": str(tmp_path / "logs"), "name": "VanillaVAE"}}
    cfg.update(over)
    p = tmp_path / "vae.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p)


def test_config_overrides_and_experiment_name(tmp_path):
    args = R.build_parser().parse_args(["-c", _cfg(tmp_path), "-r", "coinrun", "-t", "maze", "-d", "64", "-k", "0.5",
                                        "--max_epochs", "1"])
    c = R.load_config(args)
    assert c["model_params"]["latent_dim"] == 64 and c["exp_params"]["kld_weight"] == 0.5
    assert c["trainer_params"]["max_epochs"] == 1
    assert c["exp_name"] == "VanillaVAE-64-kl_0.5-train_coinrun-test_maze"
    assert c["exp_params"]["test_output_dir"].endswith(c["exp_name"])


def test_batches_shard_per_rank():
    imgs = torch.arange(20, dtype=torch.float32).view(20, 1, 1, 1)
    names = [str(i) for i in range(20)]
    b0 = R.batches(imgs, names, 4, False, 0, rank=0, world=2)
    b1 = R.batches(imgs, names, 4, False, 0, rank=1, world=2)
    assert len(b0) == len(b1) == 2
    seen = sorted(int(n) for bl in (b0, b1) for _, _, ns in bl for n in ns)
    assert seen == list(range(16))                       # disjoint shards, last partial global batch dropped
    single = R.batches(imgs, names, 6, False, 0)
    assert sum(len(ns) for _, _, ns in single) == 20


def test_lightning_checkpoint_roundtrip(tmp_path):
    m = torch.nn.Linear(4, 3)
    path = str(tmp_path / "ck" / "last.ckpt")
    R.save_checkpoint(path, m, epoch=2, global_step=10)
    ck = torch.load(path, weights_only=True)
    assert set(ck["state_dict"]) == {"model.weight", "model.bias"} and ck["epoch"] == 2
    m2 = torch.nn.Linear(4, 3)
    R.load_checkpoint(path, m2)
    assert torch.equal(m2.weight, m.weight) and torch.equal(m2.bias, m.bias)
