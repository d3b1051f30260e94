"""Paired augmentation, CPU side: the oracle against Pillow (committed fixtures and live
Pillow calls), and the product's host tables / draws against the oracle."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stf-unet_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from oracle import augment as A  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "aug_pil.npz")


def golden_cases():
    from make_golden_aug import SHAPES, case_inputs
    z = np.load(GOLD)
    for i, (h, w) in enumerate(SHAPES):
        v = z[f"p{i}"]
        p = dict(h2=int(v[2]), w2=int(v[3]), hflip=bool(v[4]), vflip=bool(v[5]),
                 angle=float(v[7]) if v[6] else None, crop=int(v[8]) or None, h0=int(v[9]), w0=int(v[10]))
        img, m = case_inputs(i, h, w)
        yield i, img, m, p, z[f"ref_img{i}"], z[f"ref_mask{i}"]


def test_oracle_matches_pillow_fixtures():
    n = 0
    for i, img, m, p, ref_img, ref_mask in golden_cases():
        assert np.array_equal(A.frame_u8(img, p), ref_img), i
        assert np.array_equal(A.mask(m, p), ref_mask), i
        n += 1
    assert n == 10


def test_oracle_matches_live_pillow():
    """Random sizes / angles against Pillow in this process (Pillow is importable)."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(5)
    for _ in range(6):
        h, w = (int(v) for v in rng.integers(24, 160, 2))
        h2, w2 = (int(v) for v in rng.integers(16, 200, 2))
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
        assert np.array_equal(A.resize_bilinear(img, h2, w2),
                              np.array(Image.fromarray(img).resize((w2, h2), Image.BILINEAR)))
        assert np.array_equal(A.resize_nearest(img, h2, w2),
                              np.array(Image.fromarray(img).resize((w2, h2), Image.NEAREST)))
        ang = float(rng.uniform(-45, 45))
        m = A.rotate_matrix(ang, w, h)
        assert np.array_equal(A.rotate_bilinear(img, m),
                              np.array(Image.fromarray(img).rotate(ang, resample=Image.BILINEAR, expand=False)))
        assert np.array_equal(A.rotate_nearest(img, m),
                              np.array(Image.fromarray(img).rotate(ang, resample=Image.NEAREST, expand=False)))


def test_host_tables_match_oracle():
    from stfunet import augment as G
    for insz, outsz in [(256, 128), (256, 307), (256, 256), (300, 217), (96, 224), (1000, 130), (7, 3)]:
        rows, ks = G.bilinear_rows(insz, outsz)
        b, k = A.resize_coeffs(insz, outsz)
        rows = rows.reshape(outsz, ks + 2)
        assert ks == k.shape[1]
        assert np.array_equal(rows[:, :2], b) and np.array_equal(rows[:, 2:], k), (insz, outsz)
        assert np.array_equal(G.nearest_index(insz, outsz), A.nearest_table(insz, outsz)), (insz, outsz)
    for ang in (-29.9, -3.25, 0.5, 17.0, 29.99):
        m, fx = G.rotation(ang, 231, 244)
        mo = A.rotate_matrix(ang, 231, 244)
        assert list(m) == mo
        assert fx[0] == A.fix16(mo[0]) and fx[4] == A.fix16(mo[2] + mo[1] * 0.5 + mo[0] * 0.5)


def test_draw_order_matches_reference_sequence():
    """DeviceAugment's draws == the oracle's restatement of the reference's Compose order."""
    from stfunet import augment as G
    aug = G.DeviceAugment(train=True, seed=11, device="cpu", paired=False)
    r = random.Random(11)
    for h, w in [(256, 256), (240, 300), (96, 128)]:
        got = aug.draw_sample(4, h, w)
        want = [A.draw_train(r, h, w) for _ in range(4)]
        assert got == want
    paired = G.DeviceAugment(train=True, seed=3, device="cpu", paired=True).draw_sample(8, 256, 256)
    assert all(p is paired[0] for p in paired)
    default = G.DeviceAugment(train=True, seed=3, device="cpu").draw_sample(8, 256, 256)
    assert len({repr(p) for p in default}) > 1                  # reference default: a draw per frame


def test_unseeded_augment_pickles():
    """seed=None keeps no module reference: picklable for spawn / forkserver workers."""
    import pickle
    from stfunet import augment as G
    aug = pickle.loads(pickle.dumps(G.DeviceAugment(train=True, device="cpu")))
    assert aug.rng is random
    seeded = G.DeviceAugment(train=True, seed=4, device="cpu")
    seeded.draw(64, 64)
    twin = pickle.loads(pickle.dumps(seeded))
    assert twin.draw(64, 64) == seeded.draw(64, 64)


def test_eval_size_rule():
    from stfunet import augment as G
    for h, w in [(256, 256), (240, 300), (300, 210), (224, 500)]:
        assert G.resized_size(h, w, 224) == A.resized_size(h, w, 224)
