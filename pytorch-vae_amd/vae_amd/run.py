"""run.py counterpart (reference run.py:18-107) on the MI355X path, without PyTorch Lightning.

    python -m vae_amd.run -c configs/vae/vae.yaml -r <train_dataset> [-t <test_dataset>] ...
    python -m torch.distributed.run --nproc-per-node N -m vae_amd.run -c ... (one rank per GPU)

Same flags and YAML keys as the reference (model_params -> the vae_models registry, exp_params ->
VAEXperiment, data_params, trainer_params.max_epochs, logging_params); the experiment name and
the -d / -k overrides follow run.py:39-51.  What differs, on purpose:
  * the model is the libvaehip drop-in (vae_amd.models) — add `--dtype bf16` for the throughput
    mode; `--synthetic N` trains on N synthetic U[0,1) images instead of a PNG folder;
  * data parallelism is the reference's DDPPlugin semantics done directly: per-rank shards of
    each batch list, flat-gradient all-reduce (mean) after backward, rank-0 BatchNorm buffers;
  * checkpoints are Lightning-format dicts (`state_dict` with `model.`-prefixed reference keys,
    run.py:80-84 `best.ckpt` by val_loss and `last.ckpt`), loadable by the reference and back;
  * image outputs of test (draw.py / make_tex.py) are out of scope: test reports loss terms.
"""
from __future__ import annotations

import argparse
import os
import random
from typing import Dict, List, Optional

import numpy as np
import torch

LIGHTNING_VERSION = "1.5.6"          # the reference's pin (requirements.txt:1), recorded in checkpoints


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description='Generic runner for VAE models (MI355X path)')
    p.add_argument('--config', '-c', dest="filename", metavar='FILE', help='path to the config file',
                   default='configs/vae.yaml')
    p.add_argument('-r', '--train_dataset', type=str, help='Dataset to use for training')
    p.add_argument('-t', '--test_dataset', type=str, help='Dataset to use for testing')
    p.add_argument('-d', '--latent_dim', type=int, help='Latent dimension override')
    p.add_argument('-p', '--trained_model_path', type=str, help='Checkpoint to test (skips training)')
    p.add_argument('-k', '--kl_penalty', type=float, help='KL penalty override')
    p.add_argument('-o', '--test_output_dir', type=str, default='full_test_output')
    p.add_argument('-e', '--extra_image_outputs', action='store_true', default=False)
    p.add_argument('-a', '--dont_annotate_loss', action='store_true', default=False)
    p.add_argument('--histogram_only', action='store_true', default=False)
    # MI355X-path options
    p.add_argument('--dtype', choices=['f32', 'bf16'], default='f32')
    p.add_argument('--synthetic', type=int, default=0, help='train/test on N synthetic U[0,1) images')
    p.add_argument('--engine', choices=['graph', 'eager'], default='graph',
                   help='graph: each training step is one replay of the fused HIP-graph step '
                        '(experiment.GraphedSteps); eager: training_step + loss.backward() + optimizer.step()')
    p.add_argument('--max_epochs', type=int, help='override trainer_params.max_epochs')
    return p


def load_config(args) -> dict:
    """run.py:30-51: YAML + command-line overrides + experiment name."""
    import yaml
    with open(args.filename) as f:
        config = yaml.safe_load(f)
    if args.train_dataset is None and args.test_dataset is None and not args.synthetic:
        raise ValueError("At least one of train_dataset and test_dataset must be provided")
    ep = config['exp_params']
    ep['extra_image_outputs'] = args.extra_image_outputs
    ep['dont_annotate_loss'] = args.dont_annotate_loss
    ep['histogram_only'] = args.histogram_only
    if args.latent_dim is not None:
        config['model_params']['latent_dim'] = args.latent_dim
    if args.kl_penalty is not None:
        ep['kld_weight'] = args.kl_penalty
    if args.max_epochs is not None:
        config['trainer_params']['max_epochs'] = args.max_epochs
    name = f"{config['logging_params']['name']}-{config['model_params'].get('latent_dim', '')}-kl_{ep['kld_weight']}"
    if args.trained_model_path is None:
        name += f"-train_{args.train_dataset or 'synthetic'}"
    if args.test_dataset is not None:
        name += f"-test_{args.test_dataset}"
    config['exp_name'] = name
    ep['test_output_dir'] = os.path.join(args.test_output_dir, name)
    return config


# ----------------------------------------------------------------------------- data
def _load_png(path: str, size: int) -> torch.Tensor:
    """default_loader + Resize(patch_size) + ToTensor (dataset.py:78-79): RGB, [0,1], CHW."""
    from PIL import Image
    img = Image.open(path).convert("RGB").resize((size, size), Image.BILINEAR)
    t = torch.frombuffer(bytearray(img.tobytes()), dtype=torch.uint8).view(size, size, 3)
    return t.permute(2, 0, 1).float() / 255.0


def folder_split(data_dir: str, train_ratio: float, seed: int):
    """dataset.py split_images for plain '<n>.png' names: shuffled split, test part sorted."""
    files = sorted(f for f in os.listdir(data_dir) if f.endswith('.png'))
    rng = random.Random(seed)
    rng.shuffle(files)
    cut = int(train_ratio * len(files))
    key = lambda f: (0, int(f[:-4])) if f[:-4].isdigit() else (1, f)
    return [os.path.join(data_dir, f) for f in files[:cut]], sorted((os.path.join(data_dir, f) for f in files[cut:]),
                                                                     key=lambda p: key(os.path.basename(p)))


def batches(images: torch.Tensor, names: List[str], bs: int, shuffle: bool, seed: int, rank: int = 0, world: int = 1):
    """(imgs, labels, names) batches; with world > 1 each rank takes its contiguous shard of every
    global batch (the DistributedSampler role)."""
    idx = list(range(images.shape[0]))
    if shuffle:
        random.Random(seed).shuffle(idx)
    out = []
    gbs = bs * world
    for s in range(0, len(idx) - gbs + 1 if world > 1 else len(idx), gbs):
        sel = idx[s + rank * bs:s + (rank + 1) * bs]
        if not sel:
            continue
        out.append((images[sel], torch.zeros(len(sel), dtype=torch.float64), [names[i] for i in sel]))
    return out


# ----------------------------------------------------------------------------- checkpoints
def save_checkpoint(path: str, model, epoch: int, global_step: int, optimizer=None, extra: Optional[Dict] = None):
    """Lightning-format checkpoint: state_dict keys 'model.<reference key>' (run.py:80-84)."""
    ck = {"epoch": epoch, "global_step": global_step, "pytorch-lightning_version": LIGHTNING_VERSION,
          "state_dict": {"model." + k: v.detach().cpu() for k, v in model.state_dict().items()},
          "optimizer_states": [optimizer.state_dict()] if optimizer is not None else [], "lr_schedulers": []}
    if extra:
        ck.update(extra)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save(ck, path)


def load_checkpoint(path: str, model, strict: bool = True):
    """Load a Lightning checkpoint of VAEXperiment (ours or the reference's) into a drop-in model.
    Only tensors are read (weights_only=True)."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck.get("state_dict", ck)
    sd = {k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")} or sd
    return model.load_state_dict(sd, strict=strict)


# ----------------------------------------------------------------------------- main
def main(argv=None) -> Dict[str, float]:
    args = build_parser().parse_args(argv)
    config = load_config(args)
    import torch.distributed as dist
    from .dp import allreduce_mean, broadcast_buffers
    from .data import ImageSet, ImgDifficultySampler, VAEDataset
    from .experiment import GraphedSteps, VAEXperiment, _fusable
    from .models import vae_models

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    seed = config['exp_params'].get('manual_seed', 1265)
    torch.manual_seed(seed)                                       # seed_everything (run.py:66):
    random.seed(seed)                                             # torch, Python and numpy
    np.random.seed(seed)                                          # (the difficulty sampler's draws)
    mp = dict(config['model_params'])
    name = mp.pop('name')
    dtype = torch.bfloat16 if args.dtype == 'bf16' else torch.float32
    model = vae_models[name](**mp, dtype=dtype, device=f"cuda:{local}", seed=seed)
    experiment = VAEXperiment(model, config['exp_params'])
    dpar = dict(config['data_params'])
    size = dpar.get('patch_size', 64)
    size = size if isinstance(size, int) else size[0]
    dev = torch.device("cuda", local)
    if args.synthetic:
        g = torch.Generator().manual_seed(seed)
        imgs = torch.rand(args.synthetic, 3, size, size, generator=g)
        names = [f"{i}.png" for i in range(args.synthetic)]
        cut = int(0.9 * args.synthetic)
        dm = VAEDataset("", **{k: v for k, v in dpar.items() if k not in ("data_path", "train_dataset", "test_dataset")},
                        train_dataset=None, test_dataset=None, device=dev, rank=rank, world=world)
        dm.train_set = ImageSet(imgs[:cut].to(dev), names[:cut])
        dm.val_set = dm.test_set = ImageSet(imgs[cut:].to(dev), names[cut:])
        if dpar.get('use_difficulty_sampling'):
            dm.difficulty_sampler = ImgDifficultySampler(names[:cut], dm.train_batch_size)
    else:
        # dataset.py VAEDataset(**data_params) with the -r / -t folders (run.py:71-76), resident on
        # the device; split_images uses Python's `random`, seeded above like seed_everything
        dm = VAEDataset(**{k: v for k, v in dpar.items() if k not in ("train_dataset", "test_dataset")},
                        train_dataset=args.train_dataset, test_dataset=args.test_dataset, device=dev,
                        rank=rank, world=world)
        dm.setup()
    experiment.datamodule = dm
    train = dm.train_set
    log_dir = os.path.join(config['logging_params']['save_dir'], config['exp_name'], "version_0")
    ck_dir = os.path.join(log_dir, "checkpoints")
    result: Dict[str, float] = {}
    if args.trained_model_path is None and train is not None:
        opt_cfg = experiment.configure_optimizers()
        plateau = None
        if isinstance(opt_cfg, tuple):
            optims, scheds = opt_cfg
        elif isinstance(opt_cfg, dict):
            optims, scheds, plateau = [opt_cfg["optimizer"]], [], opt_cfg["lr_scheduler"]["scheduler"]
        else:
            optims, scheds = opt_cfg, []
        best, step = float("inf"), 0
        epochs = config['trainer_params'].get('max_epochs', 1)
        graphed = None
        if args.engine == 'graph' and hasattr(model, 'fused_train_step') and len(optims) == 1 and _fusable(model):
            # the fused step replayed from HIP graphs (DDP gradient mean and rank-0 buffers inside
            # the TrainStep); no host synchronisation inside the epoch
            graphed = GraphedSteps(experiment, optims[0])
        for epoch in range(epochs):
            model.train()
            sums: Dict[str, float] = {}
            for i, batch in enumerate(dm.train_dataloader()):
                if graphed is not None:
                    graphed(batch, i)
                    step += 1
                    continue
                optims[0].zero_grad(set_to_none=True)
                loss = experiment.training_step(batch, i)
                loss.backward()
                if world > 1:                                   # DDP: gradient mean, rank-0 buffers
                    allreduce_mean(model.flat.grad)
                    broadcast_buffers(model.net.running)
                optims[0].step()
                step += 1
            if graphed is not None:
                graphed.flush()                                 # per-image losses, extreme images
            dm.on_epoch_end()                                   # difficulty sampler update
            for k, v in experiment.logged.items():
                sums[k] = float(v)
            model.eval()
            vals = [experiment.validation_step(b, i) for i, b in enumerate(dm.val_dataloader())]
            if vals:
                for k in vals[0]:
                    sums[f"val_{k}"] = sum(float(v[k]) for v in vals) / len(vals)
            for s in scheds:
                s["scheduler"].step()
            if plateau is not None and "val_loss" in sums:
                plateau.step(sums["val_loss"])
            experiment.reset_extreme_image_tracking()
            if rank == 0:
                save_checkpoint(os.path.join(ck_dir, "last.ckpt"), model, epoch, step, optims[0])
                if sums.get("val_loss", float("inf")) < best:
                    best = sums["val_loss"]
                    save_checkpoint(os.path.join(ck_dir, "best.ckpt"), model, epoch, step, optims[0])
                print(f"epoch {epoch}: " + ", ".join(f"{k}={v:.5f}" for k, v in sorted(sums.items())), flush=True)
            result = sums
        checkpoint_path = os.path.join(ck_dir, "last.ckpt")
    else:
        checkpoint_path = args.trained_model_path
    if (args.test_dataset is not None or args.synthetic) and checkpoint_path and os.path.exists(checkpoint_path):
        load_checkpoint(checkpoint_path, model)
        model.eval()
        outs = [experiment.test_step(b, i) for i, b in enumerate(dm.test_dataloader())]
        if outs and rank == 0:
            result.update({f"test_{k}": sum(float(o[k]) for o in outs) / len(outs) for k in outs[0]})
            st = experiment.loss_stats['total_loss']
            print("test: " + ", ".join(f"{k}={v:.5f}" for k, v in sorted(result.items()) if k.startswith("test_"))
                  + f"; per-image total loss x1000 in [{st['min']:.3f}, {st['max']:.3f}] over "
                  f"{len(experiment.test_data)} images")
    if world > 1 and dist.is_initialized():
        dist.destroy_process_group()
    if rank == 0:
        print(f"----\nSuccessfully completed {config['exp_name']}\n----")
    return result


if __name__ == "__main__":
    main()
