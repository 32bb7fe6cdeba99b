"""Data path of the reference's training loop, GPU-resident: VAEDataset (dataset.py:32-216) and
ImgDifficultySampler (difficulty_sampler.py:6-46) without Lightning or torchvision.

  split_images / sort_images   dataset.py:148-216 — the same file-name rules (plain '<n>.png' and
                               'iter..env..step..run-id..' names, run-ids kept whole on one side of
                               the split), the same use of Python's global `random` state
  ImgDifficultySampler         difficulty_sampler.py:6-46 — importance sampling with replacement by
                               per-image running-mean loss, numpy's global RNG, the mean/5 floor
  VAEDataset                   dataset.py:32-147 — setup (0.9 split, optional separate test set,
                               sampler), train/val/test batches, record_img_losses, on_epoch_end

What differs, for the GPU: images are decoded once (default_loader + Resize(patch_size) +
ToTensor semantics, RGB in [0, 1]) into one uint8 tensor [N, 3, H, W] that lives on the device; a
batch is an index gather plus a uint8 -> fp32 scale on the device, so the training loop never
waits on host decoding or a host->device copy.  Batches are the reference's DataLoader tuples
(imgs [B, 3, H, W] fp32, labels [B] float64 zeros — MyDataset's dummy 0.0 — and file names)."""
from __future__ import annotations

import os
import random
import re
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

_SIMPLE = re.compile(r'^(\d+)\.png$')
_COMPLEX = re.compile(r'iter(\d+).*?env(\d+).*?step(\d+).*?run-id(\d+)')


def sort_images(img_paths: Sequence[str]) -> List[str]:
    """dataset.py:187-216: '<n>.png' by n; complex names by (run-id, iter, env, step); anything
    else is an error."""
    def key(path):
        name = os.path.basename(path)
        s, c = _SIMPLE.match(name), _COMPLEX.search(name)
        if s:
            return (0, int(s.group(1)))
        if c:
            return (1, int(c.group(4)), int(c.group(1)), int(c.group(2)), int(c.group(3)))
        raise ValueError(f"Filename {name} is in the wrong format")
    return sorted(img_paths, key=key)


def split_images(data_dir: str, train_ratio: float, verbose: bool = False) -> Tuple[List[str], List[str]]:
    """dataset.py:148-185.  Consumes Python's global `random` state exactly as the reference does
    (one shuffle of the run-ids, one of the plain names), so `random.seed(s)` reproduces its split."""
    image_files = [f for f in os.listdir(data_dir) if f.endswith('.png')]
    run_ids = set()
    for f in image_files:
        m = _COMPLEX.search(f)
        if m:
            run_ids.add(int(m.group(4)))
    run_ids = list(run_ids)
    random.shuffle(run_ids)
    train_ids = run_ids[:int(train_ratio * len(run_ids))]
    simple, train_c, test_c = [], [], []
    for f in image_files:
        s, c = _SIMPLE.match(f), _COMPLEX.search(f)
        if s:
            simple.append(os.path.join(data_dir, f))
        elif c:
            (train_c if int(c.group(4)) in train_ids else test_c).append(os.path.join(data_dir, f))
    random.shuffle(simple)
    cut = int(train_ratio * len(simple))
    train_all = simple[:cut] + train_c
    test_all = sort_images(simple[cut:] + test_c)
    if verbose:
        print(f"Loaded {len(train_all)} training images and {len(test_all)} test images")
    return train_all, test_all


class ImgDifficultySampler:
    """difficulty_sampler.py:6-46: each epoch draws len(dataset) indices with replacement, with
    probability proportional to the image's weight (its running-mean loss, floored at mean/5)."""

    def __init__(self, image_paths: Sequence[str], batch_size: int):
        self.dataset_size = len(image_paths)
        self.batch_size = batch_size
        self.img_weights = np.ones(self.dataset_size)
        self.image_paths = list(image_paths)
        self.imgname_to_idx = {os.path.basename(p): i for i, p in enumerate(self.image_paths)}
        self.indices = None

    def __iter__(self):
        probs = self.img_weights / np.sum(self.img_weights)
        self.indices = np.random.choice(self.dataset_size, size=self.dataset_size, replace=True, p=probs)
        return iter(self.indices.tolist())

    def __len__(self):
        return self.dataset_size

    def update_img_difficulties(self, img_names: Sequence[str], losses: Sequence[float]):
        indices = [self.imgname_to_idx[n] for n in img_names]
        counts = np.zeros(self.dataset_size, dtype=np.int32)
        for idx, loss in zip(indices, losses):
            counts[idx] += 1
            self.img_weights[idx] = (self.img_weights[idx] * (counts[idx] - 1) + loss) / counts[idx]
        floor = np.mean(self.img_weights) / 5
        self.img_weights = np.maximum(self.img_weights, floor)


def resized_size(w: int, h: int, size: int):
    """torchvision transforms.Resize(int) output (w, h): the SHORTER edge becomes `size`, the longer
    one int(size * long / short) (torchvision _compute_resized_output_size; dataset.py:78)."""
    short, long_ = (w, h) if w <= h else (h, w)
    if short == size:
        return w, h
    new_long = int(size * long_ / short)
    return (size, new_long) if w <= h else (new_long, size)


def load_images(paths: Sequence[str], size: int, device=None) -> torch.Tensor:
    """default_loader (RGB) + Resize(size) + ToTensor (dataset.py:78-79), kept as uint8
    [N, 3, size, size] (the ToTensor scale 1/255 is applied per batch on the device).  Resize(int)
    scales the shorter edge to `size` with PIL's bilinear filter (torchvision's default for PIL
    inputs) and keeps the aspect ratio; a non-square image therefore comes out non-square, which the
    reference's models cannot take (their flatten sizes assume size x size, vanilla_vae.py:36) — such
    an image is rejected here with its name instead of failing later inside the model."""
    from PIL import Image
    out = torch.empty(len(paths), 3, size, size, dtype=torch.uint8)
    for i, p in enumerate(paths):
        with Image.open(p) as im:
            im = im.convert("RGB")
            tgt = resized_size(im.size[0], im.size[1], size)
            if tgt != (size, size):
                raise ValueError(f"{p}: {im.size[0]}x{im.size[1]} resizes to {tgt[0]}x{tgt[1]} under "
                                 f"Resize({size}) (shorter edge to {size}); the models take {size}x{size} images")
            if im.size != tgt:
                im = im.resize(tgt, Image.BILINEAR)
            a = np.asarray(im, dtype=np.uint8)
        out[i] = torch.from_numpy(a.copy()).permute(2, 0, 1)
    return out.to(device) if device is not None else out


class ImageSet:
    """A device-resident image set: uint8 pixels + file names."""

    def __init__(self, pixels: torch.Tensor, names: Sequence[str]):
        self.pixels, self.names = pixels, list(names)

    def __len__(self):
        return len(self.names)

    def batch(self, idx: Sequence[int]):
        it = torch.as_tensor(list(idx), dtype=torch.long, device=self.pixels.device)
        imgs = self.pixels.index_select(0, it)
        imgs = imgs.float().div_(255.0) if imgs.dtype == torch.uint8 else imgs.float()
        return imgs, torch.zeros(len(idx), dtype=torch.float64), [self.names[i] for i in idx]


class VAEDataset:
    """dataset.py:32-147 (LightningDataModule) with device-resident data.

    data_path/train_dataset/test_dataset, batch sizes, patch_size and use_difficulty_sampling
    have the reference's meaning; num_workers/pin_memory are accepted and unused (nothing is
    decoded inside the loop).  rank/world shard every global batch (DistributedSampler's role)."""

    def __init__(self, data_path: str, train_batch_size: int = 8, val_batch_size: int = 8,
                 test_batch_size: int = 8, patch_size=(256, 256), num_workers: int = 0, pin_memory: bool = False,
                 train_dataset='coinrun', test_dataset=None, use_difficulty_sampling=False, device=None,
                 rank: int = 0, world: int = 1, **kwargs):
        self.train_data_dir = os.path.join(data_path, train_dataset) if train_dataset is not None else None
        self.test_data_dir = os.path.join(data_path, test_dataset) if test_dataset is not None else None
        self.train_batch_size, self.val_batch_size, self.test_batch_size = train_batch_size, val_batch_size, test_batch_size
        self.patch_size = patch_size if isinstance(patch_size, int) else patch_size[0]
        self.train_dataset_name, self.test_dataset_name = train_dataset, test_dataset
        self.use_difficulty_sampling = use_difficulty_sampling
        self.device, self.rank, self.world = device, rank, world
        self.sampled_img_names: List[str] = []
        self.sampled_img_losses: List[float] = []
        self.train_set = self.val_set = self.test_set = None
        self.difficulty_sampler: Optional[ImgDifficultySampler] = None

    def setup(self, stage: Optional[str] = None) -> None:
        """dataset.py:78-103."""
        sz = self.patch_size
        if self.train_dataset_name is not None:
            tr, va = split_images(self.train_data_dir, 0.9)
            self.train_set = ImageSet(load_images(tr, sz, self.device), [os.path.basename(p) for p in tr])
            self.val_set = ImageSet(load_images(va, sz, self.device), [os.path.basename(p) for p in va])
            if self.use_difficulty_sampling:
                self.difficulty_sampler = ImgDifficultySampler(tr, self.train_batch_size)
        if self.test_dataset_name is not None:
            _, te = split_images(self.test_data_dir, 0.0)
            self.test_set = ImageSet(load_images(te, sz, self.device), [os.path.basename(p) for p in te])
        else:
            self.test_set = self.val_set

    def _eval_batches(self, s: ImageSet, bs: int) -> Iterable:
        """val / test loaders: every image is evaluated.  One rank: in order, the last batch
        partial.  Several ranks: DistributedSampler(shuffle=False) semantics — the index list
        padded by wrap-around to a multiple of world, rank r taking r, r+world, ... — so every rank
        runs the same number of batches (their collectives stay matched) and none is dropped."""
        n = len(s)
        if self.world <= 1:
            yield from self._batches(s, range(n), bs)
            return
        per = -(-n // self.world)
        order = list(range(n))
        if n:   # DistributedSampler: repeat the list as often as needed (the pad may exceed n)
            order = (order * -(-(per * self.world) // n))[:per * self.world]
        mine = order[self.rank::self.world]
        for i in range(0, len(mine), bs):
            yield s.batch(mine[i:i + bs])

    def _batches(self, s: ImageSet, order: Sequence[int], bs: int) -> Iterable:
        gbs = bs * self.world
        n = len(order)
        stop = n - gbs + 1 if self.world > 1 else n
        for i in range(0, max(stop, 0), gbs):
            sel = list(order[i + self.rank * bs: i + (self.rank + 1) * bs])
            if sel:
                yield s.batch(sel)

    def train_dataloader(self) -> Iterable:
        """Shuffled (torch's global generator, as DataLoader(shuffle=True)) or drawn by the
        difficulty sampler."""
        s = self.train_set
        if self.difficulty_sampler is not None:
            order = list(iter(self.difficulty_sampler))
        else:
            order = torch.randperm(len(s)).tolist()
        return self._batches(s, order, self.train_batch_size)

    def val_dataloader(self) -> Iterable:
        return self._eval_batches(self.val_set, self.val_batch_size)

    def test_dataloader(self) -> Iterable:
        return self._eval_batches(self.test_set, self.test_batch_size)

    def record_img_losses(self, img_names, losses):
        """dataset.py:130-136."""
        if isinstance(img_names, torch.Tensor):
            img_names = img_names.cpu().tolist()
        if isinstance(losses, torch.Tensor):
            losses = losses.cpu().tolist()
        self.sampled_img_names.extend(img_names)
        self.sampled_img_losses.extend(losses)

    def on_epoch_end(self):
        """dataset.py:138-142."""
        if self.difficulty_sampler is not None:
            self.difficulty_sampler.update_img_difficulties(self.sampled_img_names, self.sampled_img_losses)
        self.sampled_img_names = []
        self.sampled_img_losses = []
