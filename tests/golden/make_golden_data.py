"""Golden vectors for the data path (vae_amd/data.py), produced by the reference's own code.

Run in the survey container, where /root/reference is importable:

    python tests/golden/make_golden_data.py      # writes tests/golden/data_path.json

difficulty_sampler.py imports as is.  dataset.py needs pytorch_lightning and torchvision, which
are absent; only its split/sort methods are exercised here, with in-memory stand-in modules for
those imports (the same recipe the survey used for torchvision).  No reference
file is copied or modified; the fixture is data (file names, index sequences, weights)."""
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data_path.json")


def _stub_imports():
    pl = types.ModuleType("pytorch_lightning")
    pl.LightningDataModule = object
    tv = types.ModuleType("torchvision")
    tvd = types.ModuleType("torchvision.datasets")
    tvf = types.ModuleType("torchvision.datasets.folder")
    tvf.default_loader = lambda p: None
    tvt = types.ModuleType("torchvision.transforms")
    sys.modules.update({"pytorch_lightning": pl, "torchvision": tv, "torchvision.datasets": tvd,
                        "torchvision.datasets.folder": tvf, "torchvision.transforms": tvt})


def main():
    sys.path.insert(0, REF)
    _stub_imports()
    import dataset as D
    import difficulty_sampler as S
    names = [f"{i}.png" for i in range(23)]
    names += [f"iter{it}_env{e}_step{st}_run-id{r}.png" for r in (3, 11, 42, 7, 19) for it in (1, 2)
              for e in (0, 1) for st in (5, 17)]
    names += ["notes.txt"]
    out = {"listing": names}
    with tempfile.TemporaryDirectory() as d:
        for n in names:
            open(os.path.join(d, n), "w").close()
        # the split depends on the order os.listdir returns: pin it to `names` for the reference
        # call (and the test replays the same order)
        real_listdir = os.listdir
        os.listdir = lambda path: list(names) if path == d else real_listdir(path)
        mod = D.VAEDataset.__new__(D.VAEDataset)
        try:
            for ratio, seed in ((0.9, 1265), (0.0, 7), (0.5, 3)):
                random.seed(seed)
                tr, te = D.VAEDataset.split_images(mod, d, train_ratio=ratio)
                out[f"split_{ratio}_{seed}"] = {"train": [os.path.basename(p) for p in tr],
                                                "test": [os.path.basename(p) for p in te]}
        finally:
            os.listdir = real_listdir
    mixed = ["/x/10.png", "/x/2.png", "iter2_env1_step3_run-id5.png", "iter1_env0_step9_run-id5.png",
             "iter1_env0_step2_run-id4.png", "/x/0.png"]
    out["sort_in"] = mixed
    out["sort_out"] = D.VAEDataset.sort_images(mod, mixed)

    class _DS:
        images = [f"/data/{i}.png" for i in range(12)]

        def __len__(self):
            return len(self.images)
    np.random.seed(3)
    smp = S.ImgDifficultySampler(_DS(), batch_size=4)
    e1 = list(iter(smp))
    seen = [f"{i}.png" for i in e1]
    rng = np.random.RandomState(5)
    losses = [float(v) for v in rng.uniform(0.001, 0.05, size=len(seen))]
    smp.update_img_difficulties(seen, losses)
    w1 = smp.img_weights.tolist()
    e2 = list(iter(smp))
    seen2 = [f"{i}.png" for i in e2[:7]]
    losses2 = [float(v) for v in rng.uniform(0.0, 0.2, size=len(seen2))]
    smp.update_img_difficulties(seen2, losses2)
    out["sampler"] = {"np_seed": 3, "n": 12, "epoch1": e1, "names1": seen, "losses1": losses, "weights1": w1,
                      "epoch2": e2, "names2": seen2, "losses2": losses2, "weights2": smp.img_weights.tolist()}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
