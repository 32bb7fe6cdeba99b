"""The data path (vae_amd/data.py) against golden vectors made by the reference's own
dataset.py split/sort and difficulty_sampler.py (tests/golden/make_golden_data.py): the same
train/test split for the same Python `random` state and directory listing, the same test-set
order, and the same sampled indices and per-image weights for the same numpy RNG state."""
import json
import os
import random

import numpy as np
import pytest
import torch

from vae_amd import data as V

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data_path.json")))


@pytest.fixture
def listing_dir(tmp_path, monkeypatch):
    for n in GOLD["listing"]:
        (tmp_path / n).write_bytes(b"")
    real = os.listdir
    monkeypatch.setattr(V.os, "listdir", lambda p: list(GOLD["listing"]) if str(p) == str(tmp_path) else real(p))
    return str(tmp_path)


@pytest.mark.parametrize("key", ["split_0.9_1265", "split_0.0_7", "split_0.5_3"])
def test_split_matches_reference(listing_dir, key):
    _, ratio, seed = key.split("_")
    random.seed(int(seed))
    tr, te = V.split_images(listing_dir, float(ratio))
    assert [os.path.basename(p) for p in tr] == GOLD[key]["train"]
    assert [os.path.basename(p) for p in te] == GOLD[key]["test"]
    # run-ids never straddle the split
    rid = lambda n: V._COMPLEX.search(n).group(4) if V._COMPLEX.search(n) else None
    a = {rid(os.path.basename(p)) for p in tr} - {None}
    b = {rid(os.path.basename(p)) for p in te} - {None}
    assert not (a & b)


def test_sort_matches_reference():
    assert V.sort_images(GOLD["sort_in"]) == GOLD["sort_out"]
    with pytest.raises(ValueError):
        V.sort_images(["bad_name.png"])


def test_difficulty_sampler_matches_reference():
    g = GOLD["sampler"]
    np.random.seed(g["np_seed"])
    s = V.ImgDifficultySampler([f"/data/{i}.png" for i in range(g["n"])], batch_size=4)
    assert len(s) == g["n"]
    assert list(iter(s)) == g["epoch1"]
    s.update_img_difficulties(g["names1"], g["losses1"])
    np.testing.assert_allclose(s.img_weights, g["weights1"], rtol=1e-12)
    assert list(iter(s)) == g["epoch2"]
    s.update_img_difficulties(g["names2"], g["losses2"])
    np.testing.assert_allclose(s.img_weights, g["weights2"], rtol=1e-12)


def test_data_module_batches_and_loss_recording(tmp_path):
    """VAEDataset on a small PNG folder: resident uint8 pixels, the reference's batch tuples, the
    difficulty sampler fed by record_img_losses / on_epoch_end."""
    from PIL import Image
    d = tmp_path / "set"
    d.mkdir()
    rng = np.random.RandomState(0)
    for i in range(20):
        Image.fromarray(rng.randint(0, 256, size=(80, 80, 3), dtype=np.uint8)).save(d / f"{i}.png")
    random.seed(1)
    dm = V.VAEDataset(str(tmp_path), train_batch_size=4, val_batch_size=3, patch_size=64, train_dataset="set",
                      use_difficulty_sampling=True)
    dm.setup()
    assert len(dm.train_set) == 18 and len(dm.val_set) == 2 and dm.test_set is dm.val_set
    assert dm.train_set.pixels.dtype == torch.uint8 and tuple(dm.train_set.pixels.shape[1:]) == (3, 64, 64)
    # Resize + ToTensor of the first training image (PIL bilinear), as default_loader would give it
    p0 = os.path.join(str(d), dm.train_set.names[0])
    want = torch.from_numpy(np.asarray(Image.open(p0).convert("RGB").resize((64, 64), Image.BILINEAR)).copy())
    assert torch.equal(dm.train_set.pixels[0], want.permute(2, 0, 1))
    np.random.seed(0)
    batches = list(dm.train_dataloader())
    assert sum(b[0].shape[0] for b in batches) == 18
    imgs, labels, names = batches[0]
    assert imgs.dtype == torch.float32 and float(imgs.max()) <= 1.0 and labels.dtype == torch.float64
    for imgs, _, names in batches:
        dm.record_img_losses(names, torch.full((len(names),), 0.5))
    dm.on_epoch_end()
    assert dm.sampled_img_names == [] and float(np.min(dm.difficulty_sampler.img_weights)) > 0
    vb = list(dm.val_dataloader())
    assert [b[0].shape[0] for b in vb] == [2]


@pytest.mark.parametrize("world,n,bs", [(2, 9, 4), (3, 10, 2), (4, 3, 8), (2, 8, 4), (8, 2, 4), (8, 3, 1)])
def test_eval_loaders_cover_every_image_on_every_rank_count(world, n, bs):
    """val / test loaders with several ranks evaluate every image (DistributedSampler
    padding: wrap-around to a multiple of world, rank r takes r, r+world, ...) and every rank
    runs the same number of batches, so their loss all-reduces stay matched."""
    imgs = torch.arange(n, dtype=torch.float32).view(n, 1, 1, 1).expand(n, 3, 2, 2).contiguous()
    names = [f"{i}.png" for i in range(n)]
    seen, counts = [], []
    for rank in range(world):
        dm = V.VAEDataset("", val_batch_size=bs, test_batch_size=bs, train_dataset=None, patch_size=2,
                          rank=rank, world=world)
        dm.val_set = dm.test_set = V.ImageSet(imgs, names)
        batches = list(dm.val_dataloader())
        counts.append(len(batches))
        for x, _, nm in batches:
            seen += nm
            assert x.shape[0] == len(nm) <= bs
    assert len(set(counts)) == 1
    assert set(seen) == set(names)
    assert len(seen) == -(-n // world) * world


@pytest.mark.parametrize("w,h,want", [(64, 64, (64, 64)), (128, 128, (64, 64)), (128, 96, (85, 64)),
                                      (96, 128, (64, 85)), (50, 200, (64, 256))])
def test_resize_follows_torchvision_shorter_edge(w, h, want):
    """transforms.Resize(int) (dataset.py:78) scales the shorter edge (torchvision
    _compute_resized_output_size: int(size * long / short) for the other one)."""
    assert V.resized_size(w, h, 64) == want


def test_load_images_rejects_non_square(tmp_path):
    from PIL import Image
    Image.new("RGB", (96, 128), (10, 20, 30)).save(tmp_path / "a.png")
    Image.new("RGB", (128, 128), (10, 20, 30)).save(tmp_path / "b.png")
    x = V.load_images([str(tmp_path / "b.png")], 64)
    assert x.shape == (1, 3, 64, 64) and int(x[0, 1, 5, 5]) == 20
    with pytest.raises(ValueError, match="64x85"):
        V.load_images([str(tmp_path / "a.png")], 64)
