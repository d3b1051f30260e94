"""Device augmentation (stf_augment_frames / stf_augment_masks) vs the CPU oracle
(oracle/augment.py, itself pinned to Pillow by tests/golden/aug_pil.npz).  Bit-exact:
uint8 geometry and the fp32 (v/255 - mean)/std values compared with torch.equal."""
import os
import random
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
from oracle import augment as A  # noqa: E402

pytestmark = pytest.mark.gpu


def run(aug, frames, masks, params):
    x, t = aug(frames, masks, params)
    torch.cuda.synchronize()
    return x.cpu(), t.cpu()


def check(x, t, frames, masks, params):
    for b in range(len(frames)):
        want_x, want_t = A.sample(frames[b], masks[b], params[b])
        assert torch.equal(x[b], torch.from_numpy(want_x)), b
        assert torch.equal(t[b], torch.from_numpy(want_t)), b


def test_golden_cases_bit_exact():
    """Every Pillow fixture case (resize / flips / rotation / crop incl. padding / eval)
    as a batch of one sample with two frames (the frame and its negative)."""
    from make_golden_aug import SHAPES, case_inputs
    from stfunet.augment import DeviceAugment
    z = np.load(os.path.join(GOLDEN, "aug_pil.npz"))
    aug = DeviceAugment(device="cuda")
    for i, (h, w) in enumerate(SHAPES):
        v = z[f"p{i}"]
        p = dict(h2=int(v[2]), w2=int(v[3]), hflip=bool(v[4]), vflip=bool(v[5]),
                 angle=float(v[7]) if v[6] else None, crop=int(v[8]) or None, h0=int(v[9]), w0=int(v[10]))
        img, m = case_inputs(i, h, w)
        frames = [np.stack([img, 255 - img])]
        x, t = run(aug, frames, [m], [[p, p]])
        u8 = np.asarray(z[f"ref_img{i}"])
        assert torch.equal(x[0, 0, 0], torch.from_numpy(A.normalize(u8))), i
        assert torch.equal(t[0], torch.from_numpy(z[f"ref_mask{i}"].astype(np.int64))), i
        check(x, t, frames, [m], [[p, p]])


@pytest.mark.parametrize("paired", [True, False])
def test_training_batch_matches_oracle(paired):
    """B=4 samples of T=8 frames + 3 PK maps, ragged source sizes, drawn parameters
    (paired, or the reference's per-frame draws)."""
    from stfunet.augment import DeviceAugment
    rng = np.random.default_rng(3)
    sizes = [(256, 256), (240, 300), (300, 210), (128, 160)]
    frames = [rng.integers(0, 256, (11, h, w), dtype=np.uint8) for h, w in sizes]
    masks = [(rng.random((h, w)) < 0.2).astype(np.uint8) for h, w in sizes]
    aug = DeviceAugment(seed=17, paired=paired, device="cuda")
    params = [aug.draw_sample(11, h, w) for h, w in sizes]
    x, t = run(aug, frames, masks, params)
    assert x.shape == (4, 11, 1, 224, 224) and t.shape == (4, 224, 224) and t.dtype == torch.int64
    check(x, t, frames, masks, params)
    if not paired:
        assert len({id(p) for p in params[0]}) == 11


def test_eval_and_edge_sizes():
    """Eval mode (resize to 224 only, non-square output), an identity resize, the
    smallest draw (128: crop padding on both axes), rotation near +-30 with flips."""
    from stfunet.augment import DeviceAugment
    rng = np.random.default_rng(4)
    ev = DeviceAugment(train=False, device="cuda")
    frames = [rng.integers(0, 256, (2, 240, 300), dtype=np.uint8) for _ in range(2)]
    masks = [(rng.random((240, 300)) < 0.5).astype(np.uint8) for _ in range(2)]
    params = [ev.draw_sample(2, 240, 300) for _ in range(2)]
    x, t = run(ev, frames, masks, params)
    assert x.shape == (2, 2, 1, 224, 280)
    check(x, t, frames, masks, params)
    img = [rng.integers(0, 256, (1, 256, 256), dtype=np.uint8)]
    m = [(rng.random((256, 256)) < 0.5).astype(np.uint8)]
    tr = DeviceAugment(device="cuda")
    for p in (dict(h2=256, w2=256, hflip=False, vflip=False, angle=None, crop=224, h0=32, w0=0),
              dict(h2=128, w2=128, hflip=True, vflip=False, angle=29.999, crop=224, h0=0, w0=0),
              dict(h2=307, w2=307, hflip=True, vflip=True, angle=-29.5, crop=224, h0=83, w0=1)):
        x, t = run(tr, img, m, [[p]])
        check(x, t, img, m, [[p]])


def test_rejects_mixed_output_sizes():
    from stfunet.augment import DeviceAugment
    ev = DeviceAugment(train=False, device="cuda")
    frames = [np.zeros((1, 240, 300), np.uint8), np.zeros((1, 256, 256), np.uint8)]
    masks = [np.zeros((240, 300), np.uint8), np.zeros((256, 256), np.uint8)]
    with pytest.raises(ValueError):
        ev(frames, masks)


def test_device_loader_matches_oracle(tmp_path):
    """DriveDataset -> DataLoader (plans built in the batch) -> DeviceLoader, against the
    oracle applied to the same decoded frames with the same draws."""
    import torch.utils.data
    from _dataset_util import make_tree
    from stfunet.augment import DeviceAugment
    from stfunet.dataset import DeviceLoader, DriveDataset
    make_tree(str(tmp_path), size=(200, 260))
    ds = DriveDataset(str(tmp_path), "train", transforms=DeviceAugment(seed=9, device="cuda"), use_pk_maps=True)
    loader = DeviceLoader(torch.utils.data.DataLoader(ds, batch_size=2, collate_fn=ds.collate_fn), ds.transforms)
    twin = DeviceAugment(seed=9, device="cpu")
    i = 0
    for x, t in loader:
        x, t = x.cpu(), t.cpu()
        for b in range(x.shape[0]):
            frames, mask = ds._raw(i)
            params = twin.draw_sample(*frames.shape)
            want_x, want_t = A.sample(frames, mask, params)
            assert torch.equal(x[b], torch.from_numpy(want_x)) and torch.equal(t[b], torch.from_numpy(want_t))
            i += 1
    assert i == len(ds)


def test_train_one_epoch_from_device_loader(tmp_path):
    """The device-augmented loader is a drop-in for the reference's DataLoader: one epoch
    of engine.train_one_epoch (UNet in=8, flat channels) over it, finite loss."""
    import torch.utils.data
    from _dataset_util import make_tree
    from stfunet import engine
    from stfunet.augment import DeviceAugment
    from stfunet.dataset import DeviceLoader, DriveDataset
    from stfunet.optim import AdamW
    from stfunet.unet import UNet
    make_tree(str(tmp_path), n_patients=2, slices=2, size=(160, 160), pk=False)
    ds = DriveDataset(str(tmp_path), "train", transforms=DeviceAugment(seed=2, device="cuda"))
    loader = DeviceLoader(torch.utils.data.DataLoader(ds, batch_size=2, shuffle=True, collate_fn=ds.collate_fn),
                          ds.transforms)
    model = UNet(in_channels=8, num_classes=2, base_c=16).cuda()
    opt = AdamW([q for q in model.parameters() if q.requires_grad], lr=1e-3, weight_decay=1e-4)
    sched = engine.create_lr_scheduler(opt, len(loader), 1, warmup=True)
    loss, lr = engine.train_one_epoch(model, opt, loader, torch.device("cuda"), 0, 2, lr_scheduler=sched,
                                      print_freq=100)
    assert np.isfinite(loss) and lr > 0
