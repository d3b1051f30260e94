"""CPU checks of the drop-in surface and the C ABI (no kernel launches)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO
from oracle import unet as o_unet


@pytest.mark.parametrize("base_c,in_ch", [(64, 8), (8, 8), (64, 11)])
def test_unet_state_dict_matches_reference_keys(base_c, in_ch):
    from stfunet.unet import UNet
    m = UNet(in_channels=in_ch, num_classes=2, base_c=base_c)
    sd = m.state_dict()
    ref = o_unet.param_shapes(in_ch, 2, base_c)
    assert list(sd.keys()) == list(ref.keys())
    for k, shp in ref.items():
        assert tuple(sd[k].shape) == tuple(shp), k
    assert len(sd) == 136
    assert UNet.input_format == "flat_channels"
    if base_c == 64 and in_ch == 8:
        # SURVEY.md section 6 quotes 31,042,434, the count for in_channels=1 (enc1.0 has 64*1*9)
        assert sum(p.numel() for p in m.parameters()) == 31_046_466


def test_unet_refuses_cpu_fallback():
    from stfunet.unet import UNet
    m = UNet(8, 2, 8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 8, 32, 32))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "stfunet.h")).read()
    return sorted(set(re.findall(r"\b(stf_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_library_exports_every_header_symbol(dtype):
    """Both builds (bf16 and fp16 activation storage) export every declared entry point."""
    from stfunet import _lib
    lib = _lib.load(dtype)
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/stfunet.h but not exported"
    assert set(syms) == set(_lib.EXPORTED)
    assert lib.stf_abi_version() == 17
    assert lib.stf_storage_type() == _lib.STORAGE_CODE[dtype]
    assert b"invalid argument" in lib.stf_error_string(100001)


def test_storage_selection():
    from stfunet import _lib
    assert _lib.storage_dtype() == torch.bfloat16 and _lib.storage_for(None) == torch.bfloat16
    assert _lib.storage_for(torch.float16) == torch.float16
    with _lib.storage(torch.float16):
        assert _lib.storage_dtype() == torch.float16 and _lib.load().stf_storage_type() == 1
    assert _lib.storage_dtype() == torch.bfloat16
    with pytest.raises(ValueError):
        with _lib.storage(torch.float32):
            pass


def test_library_rejects_bad_shapes_without_launch():
    from stfunet import _lib
    lib = _lib.load()
    g = _lib.ConvGeom(1, 8, 8, 12, 12, 8, 8, 3, 3, 1, 1, 0)      # Cs=12: not a multiple of 8
    a = _lib.IgemmArgs(g, None, None, 64, None, 64, None, None, 0)
    assert lib.stf_igemm(ctypes.byref(a), None) == 100001
    assert lib.stf_bn_act(None, 8, 1, 4, 4, 12, 1, None, None, 1, None, 0, None, None, None, 12, None,
                          None) == 100001
    # stem BN+ReLU+MaxPool(3,2,1) (stf.hip bn_act_maxpool3): its unit index is 32-bit,
    # so a launch whose N*Ho*Wo*C/8 units (plus the grid stride) reach 2^31 is refused up front;
    # the largest accepted one writes through 64-bit offsets.  Fake non-null pointers: nothing runs.
    fake = ctypes.c_void_p(1 << 20)
    big = (1 << 31) // (128 * 128 * 8) + 1              # 512^2 input, C = 64: 128 x 128 x 8 units per image
    assert lib.stf_bn_act_maxpool3s2(fake, big, 256, 256, 64, 1, fake, fake, fake, fake, None) == 100001
    assert lib.stf_bn_act_maxpool3s2(fake, 8, 256, 256, 12, 1, fake, fake, fake, fake, None) == 100001
    # the DecoderBlock size fallback's argument checks (C % 8, strides, alignment)
    assert lib.stf_bilinear_ac_fwd(fake, 1, 6, 8, 12, 12, fake, 5, 7, 12, None) == 100001
    assert lib.stf_bilinear_ac_bwd(fake, 1, 5, 7, 64, 60, fake, 6, 8, 64, None) == 100001
    assert lib.stf_bilinear_ac_fwd(ctypes.c_void_p(8), 1, 6, 8, 64, 64, fake, 5, 7, 64, None) == 100001


def test_preprocess_and_lr_schedule_match_reference():
    from stfunet import engine
    from stfunet.unet import UNet
    x = torch.randn(2, 8, 1, 16, 16)
    assert engine.preprocess_input(x, UNet(8, 2, 8)).shape == (2, 8, 16, 16)
    assert engine.preprocess_input(x, object()).shape == x.shape
    g = np.load(os.path.join(GOLDEN, "lr_table.npz"))
    f = engine.lr_lambda(10, 3)
    assert np.allclose([f(i) for i in range(30)], g["lr"], atol=1e-12)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = engine.create_lr_scheduler(opt, 10, 3)
    got = []
    for _ in range(30):
        got.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert np.allclose(got, g["lr"], atol=1e-12)


def test_engine_metrics_match_reference():
    from stfunet import engine
    g = np.load(os.path.join(GOLDEN, "metrics_kat.npz"))
    logits, target = torch.from_numpy(g["logits"]), torch.from_numpy(g["target"])
    cm = engine.ConfusionMatrix(2)
    cm.update(target.flatten(), logits.argmax(1).flatten())
    assert np.array_equal(cm.mat.numpy(), g["confmat"])
    dc = engine.DiceCoefficient(2, ignore_index=255)
    dc.update(logits, target)
    dc.update(torch.from_numpy(g["logits_absent"]), torch.from_numpy(g["target_absent"]))
    assert np.allclose(dc.compute().numpy(), g["dice_per_class"], atol=1e-6)
    assert abs(dc.value.item() - float(g["dice_value"])) < 1e-6


def test_product_synthetic_cases_match_fixture_generator():
    """stfunet.synthetic.splitmix_dce_case (bench.py's Dice leg) regenerates the fixture inputs
    bit for bit (oracle.cases.dce_case wrote them)."""
    import torch
    from oracle.cases import dce_case
    from stfunet.synthetic import splitmix_dce_case
    for seed in (0, 5, 2003):
        a, b = dce_case(seed, 2, 8, 32, 48), splitmix_dce_case(seed, 2, 8, 32, 48)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_product_canonical_init_matches_fixture_init():
    """stfunet.synthetic.canonical_state_dict (bench.py's STF Dice leg restarts the reference's
    training from it) equals oracle.init's, which wrote the fixtures, bit for bit; and the
    half-resolution target option equals dce_case's."""
    from oracle.cases import dce_case
    from oracle.init import canonical_state_dict as ref_init
    from stfunet import STFLSTMUNet
    from stfunet.synthetic import canonical_state_dict, splitmix_dce_case
    tmpl = STFLSTMUNet(time_steps=4, use_pk_maps=True).state_dict()
    a, b = canonical_state_dict(tmpl, seed=0), ref_init(tmpl, seed=0)
    assert list(a) == list(b) and all(torch.equal(a[k], b[k]) for k in a)
    x0, t0 = dce_case(4001, 2, 4, 64, 64, target_hw=(32, 32))
    x1, t1 = splitmix_dce_case(4001, 2, 4, 64, 64, target_hw=(32, 32))
    assert torch.equal(x0, x1) and torch.equal(t0, t1) and t1.shape == (2, 32, 32)


def test_size_queries_depend_only_on_the_cached_signature():
    """nhwc.igemm / nhwc._wgrad ask stf_igemm_stat_tiles / _bnr_tiles / _ws_bytes and
    stf_wgrad_plan once per launch signature (geometry, flags, which optional pointers are
    set, the destination's 16-B alignment) and reuse the answer: the C functions must not
    look at anything else, e.g. the pointer values themselves (host-only calls, no GPU)."""
    from stfunet import _lib
    lib = _lib.load()
    shapes = [  # N, Hs, Ws, Cs, Hd, Wd, R, S, stride, pad, transposed, Nout, groups
        (64, 256, 256, 64, 256, 256, 3, 3, 1, 1, 0, 64, 1),       # halo, full resolution
        (64, 16, 16, 512, 16, 16, 3, 3, 1, 1, 0, 1024, 1),         # 16^2 bottleneck
        (128, 8, 8, 512, 8, 8, 3, 3, 1, 1, 0, 512, 8),             # STF layer4: split-K, grouped
        (128, 16, 16, 256, 8, 8, 3, 3, 2, 1, 0, 512, 8),           # strided
        (16, 8, 8, 512, 16, 16, 3, 3, 2, 1, 1, 256, 1),            # transposed gather
        (64, 256, 256, 8, 256, 256, 3, 3, 1, 1, 0, 64, 1),         # 8-channel network input
    ]
    for N, Hs, Ws, Cs, Hd, Wd, R, S, st, pad, tr, nout, groups in shapes:
        M = N * Hd * Wd
        res = set()
        for base in (1 << 32, (7 << 36) + 4096):
            g = _lib.ConvGeom(N, Hs, Ws, Cs, Cs, Hd, Wd, R, S, st, pad, tr)
            a = _lib.IgemmArgs(g, base, base + (1 << 30), nout, base + (2 << 30), nout, None, None, 0,
                               M // groups if groups > 1 else 0, 0, None)
            a.stats = base + (3 << 30)
            q = (lib.stf_igemm_stat_tiles(ctypes.byref(a)), lib.stf_igemm_ws_bytes(ctypes.byref(a)))
            epi = _lib.BnrEpi(base + (4 << 30), nout, base, base, base, base, 1, base)
            a.stats = None
            a.bnr = ctypes.pointer(epi)
            q += (lib.stf_igemm_bnr_tiles(ctypes.byref(a)), lib.stf_igemm_ws_bytes(ctypes.byref(a)))
            if not tr and Cs % 64 == 0 and nout % 64 == 0:
                w = _lib.WgradArgs(g, base, nout, nout, base + (1 << 30), None, 0, 0)
                sp, nb = ctypes.c_int(0), ctypes.c_size_t(0)
                assert lib.stf_wgrad_plan(ctypes.byref(w), ctypes.byref(sp), ctypes.byref(nb)) == 0
                q += (sp.value, nb.value)
            res.add(q)
        assert len(res) == 1, (N, Hs, Cs, nout, res)


def test_stat_tile_query_does_not_depend_on_the_stats_pointer():
    """Callers ask stf_igemm_stat_tiles BEFORE the statistics buffer exists (its size is the
    answer), so the answer -- and the kernel the launch will pick -- must not change once the
    pointer is set; a multi-image halo path chosen only with stats set once left rows of the
    buffer unwritten (host-only calls, no GPU)."""
    from stfunet import _lib
    lib = _lib.load()
    shapes = [  # N, H, W, Cs, Nout, groups
        (128, 16, 16, 256, 256, 8),     # STF layer3: two images per 16x32 halo tile
        (4, 16, 16, 64, 128, 2),        # even images per group
        (3, 16, 16, 64, 64, 3),         # one image per group
        (128, 8, 8, 512, 512, 8),       # STF layer4: four images per 8x32 tile
        (8, 8, 8, 256, 128, 2),
        (6, 8, 8, 256, 128, 2),         # not a multiple of four images
        (64, 256, 256, 64, 64, 1),
        (64, 32, 32, 512, 512, 1),
    ]
    for N, H, W, Cs, nout, groups in shapes:
        M = N * H * W
        g = _lib.ConvGeom(N, H, W, Cs, Cs, H, W, 3, 3, 1, 1, 0)
        a = _lib.IgemmArgs(g, 1 << 32, 2 << 32, nout, 3 << 32, nout, None, None, 0,
                           M // groups if groups > 1 else 0, 0, None)
        before = (lib.stf_igemm_stat_tiles(ctypes.byref(a)), lib.stf_igemm_ws_bytes(ctypes.byref(a)))
        a.stats = 4 << 32
        after = (lib.stf_igemm_stat_tiles(ctypes.byref(a)), lib.stf_igemm_ws_bytes(ctypes.byref(a)))
        assert before[0] == after[0], (N, H, Cs, nout, groups, before, after)


def _ref_keys():
    import json
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("which", ["unet_in8", "unet_in11", "stf_t8", "stf_t8_pk"])
def test_state_dict_keys_match_reference_modules(which):
    """Key order and shapes equal the reference modules' (tests/golden/state_dict_keys.json,
    written by make_golden.py from src/unet.py and src/stf_lstm_unet.py imported by path):
    UNet 136 keys, STFLSTMUNet 296 keys, 304 with PK maps."""
    from stfunet import STFLSTMUNet, UNet
    ref = _ref_keys()
    m = {"unet_in8": lambda: UNet(8, 2, 64), "unet_in11": lambda: UNet(11, 2, 64),
         "stf_t8": lambda: STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8),
         "stf_t8_pk": lambda: STFLSTMUNet(in_channels=1, num_classes=2, time_steps=8, use_pk_maps=True)}[which]()
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert got == ref[which]
    assert len(got) == {"unet_in8": 136, "unet_in11": 136, "stf_t8": 296, "stf_t8_pk": 304}[which]
    assert sum(p.numel() for p in m.parameters()) == ref["param_counts"][which]
    if which.startswith("stf"):          # no input_format attribute: preprocess_input passes through
        assert getattr(m, "input_format", "time_sequence") == "time_sequence"


def test_stf_accepts_reference_state_dict_roundtrip():
    """A reference-shaped STF checkpoint (keys / shapes from the fixture) loads strictly."""
    from stfunet import STFLSTMUNet
    ref = _ref_keys()["stf_t8_pk"]
    sd = {k: torch.full(shape, 0.5) if shape else torch.tensor(3) for k, shape in ref}
    m = STFLSTMUNet(use_pk_maps=True)
    m.load_state_dict(sd, strict=True)
    assert torch.equal(m.state_dict()["lstm4.weight_hh_l0"], torch.full((2048, 512), 0.5))


def test_stf_refuses_unsupported_shapes_up_front():
    """Frames smaller than 32 (layer4 would have no pixel), a wrong rank and too few frames for
    the PK maps are refused with a ValueError before any device work; sizes not divisible by 32
    are valid (the reference's bilinear size fallback, src/stf_lstm_unet.py:56-57) and reach the
    device guard."""
    from stfunet import STFLSTMUNet
    m = STFLSTMUNet(time_steps=4)
    with pytest.raises(ValueError, match="H, W >= 32"):
        m(torch.zeros(1, 4, 1, 24, 64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 4, 1, 48, 72))
    with pytest.raises(ValueError, match=r"\[B, T, C, H, W\]"):
        m(torch.zeros(4, 1, 64, 64))
    mp = STFLSTMUNet(time_steps=4, use_pk_maps=True)
    with pytest.raises(ValueError, match="no time steps"):
        mp(torch.zeros(1, mp.pk_channels, 1, 64, 64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):     # valid shape: the device guard
        m(torch.zeros(1, 4, 1, 64, 64))


def test_epoch_results_file_and_checkpoint_dict(tmp_path):
    """train.py:151-162 results-file name, the per-epoch block of :289-301, the checkpoint
    dict of :304-311 (+ 'scaler' under --amp), resume_from (:249-256) and EarlyStopping
    (early_stopping.py:9-24)."""
    import datetime
    from stfunet import engine
    from stfunet.unet import UNet
    now = datetime.datetime(2025, 5, 23, 9, 7)
    path = engine.results_file_name("stflstm", use_pk_maps=True, now=now, out_dir=str(tmp_path / "output"))
    assert path == str(tmp_path / "output" / "stflstm_results_0523-0907_pk.txt")
    assert engine.results_file_name("unet", now=now, out_dir=str(tmp_path)).endswith("unet_results_0523-0907.txt")
    cm = engine.ConfusionMatrix(2)
    cm.update(torch.tensor([0, 0, 1, 1, 1]), torch.tensor([0, 1, 1, 1, 0]))
    em = {"dice": 0.61234, "global_accuracy": 0.6, "confusion_matrix": cm,
          "mean_metrics": {"miou": 0.41666, "mprecision": 0.58333, "mrecall": 0.58333}}
    engine.write_epoch_results(path, 3, 0.123456, 1e-3 / 3, em)
    engine.write_epoch_results(path, 4, 0.1, 2e-4, em)
    text = open(path).read()
    block = ("[epoch: 3]\ntrain_loss: 0.1235\nlr: 0.000333\ndice: 0.6123\nglobal_acc: 0.6000\n"
             "mean_iou: 0.4167\nmean_precision: 0.5833\nmean_recall: 0.5833\n"
             "global correct: 60.0\naverage row correct: ['50.0', '66.7']\nIoU: ['33.3', '50.0']\n"
             "mean IoU: 41.7\n\n")
    assert text.startswith(block) and text.count("[epoch: ") == 2
    m = UNet(8, 2, 8)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    sch = engine.create_lr_scheduler(opt, 4, 3)
    scaler = torch.amp.GradScaler("cuda", enabled=False)
    ck = engine.checkpoint_dict(m, opt, sch, 5, {"amp": False})
    assert set(ck) == {"model", "optimizer", "lr_scheduler", "epoch", "args"}
    ck = engine.checkpoint_dict(m, opt, sch, 5, {"amp": True}, scaler=scaler)
    assert set(ck) == {"model", "optimizer", "lr_scheduler", "epoch", "args", "scaler"}
    m2 = UNet(8, 2, 8)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-3)
    assert engine.resume_from(ck, m2, opt2, engine.create_lr_scheduler(opt2, 4, 3), scaler) == 6
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))
    es = engine.EarlyStopping(patience=2)
    assert [es.step(v) for v in (0.5, 0.6, 0.6, 0.55)] == [False, False, False, True] and es.early_stop


def test_plan_bookkeeping_on_host():
    """The launch-plan entry points' host-side state machine (no launches: CPU-only):
    one recording per thread, stop without record refused, empty ranges replay, out-of-range
    replays refused, timing of an untimed plan is empty."""
    import ctypes
    from stfunet import _lib
    lib = _lib.load()
    einval = 100001
    h = lib.stf_plan_create()
    assert h and lib.stf_plan_size(h) == 0
    assert lib.stf_plan_stop() == einval
    assert lib.stf_plan_record(h) == 0
    assert lib.stf_plan_record(h) == einval                # one recording per thread
    assert lib.stf_plan_tag(b"igemm", 1.0) == 0 and lib.stf_plan_tag_end() == 0
    assert lib.stf_plan_replay(h, 0, 0, None) == einval    # not while it records
    assert lib.stf_plan_stop() == 0
    assert lib.stf_plan_size(h) == 0
    assert lib.stf_plan_replay(h, 0, 0, None) == 0
    assert lib.stf_plan_replay(h, 0, 1, None) == einval
    assert lib.stf_plan_replay(h, 1, 0, None) == einval
    n, ms, fl = ctypes.c_int(-1), ctypes.c_double(-1), ctypes.c_double(-1)
    assert lib.stf_plan_timing(h, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(fl)) == 0
    assert (n.value, ms.value, fl.value) == (0, 0.0, 0.0)
    assert lib.stf_plan_tag(b"outside", 1.0) == 0           # a tag outside a recording is ignored
    lib.stf_plan_destroy(h)
