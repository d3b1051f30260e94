"""DriveDataset (my_dataset.py:15-257) scan / decode / collate on the CPU; the
augmentation plans the workers build (numpy only)."""
import numpy as np
import pytest
import torch

from _dataset_util import make_tree


def test_scan_and_plain_tensors(tmp_path):
    from stfunet.dataset import DriveDataset
    n = make_tree(str(tmp_path))
    ds = DriveDataset(str(tmp_path), "train", use_pk_maps=True)
    assert len(ds) == n
    x, t = ds[0]
    assert x.shape == (11, 1, 64, 80) and x.dtype == torch.float32 and t.dtype == torch.int64
    assert float(x.max()) <= 1.0 and set(torch.unique(t).tolist()) <= {0, 1}
    xb, tb = ds.collate_fn([ds[0], ds[1]])
    assert xb.shape == (2, 11, 1, 64, 80) and tb.shape == (2, 64, 80)
    missing_vp = [i for i, d in enumerate(ds.patient_data) if d["patient_id"] == "P001"][0]
    assert float(ds[missing_vp][0][10].abs().max()) == 0.0          # absent PK map -> zeros


def test_plans_through_dataloader_workers(tmp_path):
    from stfunet.augment import DeviceAugment
    from stfunet.dataset import DriveDataset
    make_tree(str(tmp_path))
    aug = DeviceAugment(seed=5, device="cpu")
    ds = DriveDataset(str(tmp_path), "train", transforms=aug)
    frames, mask, params = ds[0]
    assert frames.shape == (8, 64, 80) and frames.dtype == np.uint8 and mask.max() <= 1
    assert len(params) == 8 and params[0]["crop"] == 224
    loader = torch.utils.data.DataLoader(ds, batch_size=2, num_workers=2, collate_fn=ds.collate_fn)
    plans = list(loader)
    assert len(plans) == 3
    for p in plans:
        assert p["n"] == p["B"] * 8 and p["out_hw"] == (224, 224)
        assert p["blob"].dtype == np.uint8 and p["o_desc"] % 16 == 0


def test_rejects_foreign_transforms(tmp_path):
    from stfunet.dataset import DriveDataset
    make_tree(str(tmp_path))
    with pytest.raises(TypeError):
        DriveDataset(str(tmp_path), "train", transforms=lambda a, b: (a, b))


def _identity(batch):
    return batch


def test_seeded_workers_draw_different_streams(tmp_path):
    """Each DataLoader worker re-creates the seeded generator from (seed, worker id,
    worker seed): two workers never replay the same parameter stream, and a run with the
    same torch seed reproduces the same draws."""
    from stfunet.augment import DeviceAugment
    from stfunet.dataset import DriveDataset
    make_tree(str(tmp_path))
    ds = DriveDataset(str(tmp_path), "train", transforms=DeviceAugment(seed=5, device="cpu"))

    def run():
        torch.manual_seed(0)
        loader = torch.utils.data.DataLoader(ds, batch_size=1, num_workers=2, collate_fn=_identity)
        return [b[0][2] for b in loader]
    params = run()
    assert len(params) >= 2
    assert params[0] != params[1]                        # worker 0 vs worker 1, first draw each
    assert run() == params
