"""BatchNorm finalize fused into its consumer pass (stf_bn_act_fin / stf_bn_bwd_apply_fin,
ABI v13; opt-in, STF_BN_FIN=1) against the separate finalize launch: bit for bit.

The fused kernels fold the partial slabs in the separate kernel's fixed fp64 order
(reduce.h fold16_pair_256), so every output -- the normalised activation, mean / invstd /
scale / shift, the running statistics (direct for one group, parked rows + the batched
update for several), dy, dgamma / dbeta (direct, or parked + stf_bn_groupsum_batch) --
must be identical, on a first launch and on repeated launches through the same flags slab
(a new epoch per launch), including shapes where a group has fewer workgroups than
16-channel chunks (one workgroup folds several) and partial slabs longer than the direct
fold (stage-1 pre-pass).  The whole STF and UNet training steps (eager, then plan replays)
are compared the same way.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, H, W, C, groups, tiles): 512 channels over 8 workgroups per group (several chunks per
# workgroup), the STF grouped shapes, a slab longer than FOLD16_ROWS (stage-1 pre-pass)
SHAPES = [(2, 8, 8, 512, 1, 7), (8, 16, 16, 64, 4, 300), (16, 8, 8, 256, 8, 33), (4, 64, 64, 128, 2, 1500)]


def _bn(C, seed):
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    g = torch.Generator(device="cpu").manual_seed(seed)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    return bn


def _stats(G, tiles, C, Mg, seed):
    """A plausible [G][tiles][2][C] slab: per-row sums of Mg / tiles values of mean ~N(0,1), var ~1."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    rows = Mg / tiles
    mu = torch.randn(G, tiles, C, generator=g)
    s1 = mu * rows
    s2 = (mu * mu + torch.rand(G, tiles, C, generator=g) + 0.5) * rows
    return torch.stack([s1, s2], 2).reshape(-1).to(DEV)


@pytest.mark.parametrize("N,H,W,C,G,tiles", SHAPES)
@pytest.mark.parametrize("res", [False, True])
def test_forward_fused_finalize_bitwise(monkeypatch, N, H, W, C, G, tiles, res):
    from stfunet import nhwc
    M = N * H * W
    monkeypatch.setenv("STF_BN_FIN", "1")
    assert nhwc.fin_fused(M, C, G)
    y = nhwc.new_feat(N, H, W, C, DEV)
    y.buf.normal_()
    r = nhwc.new_feat(N, H, W, C, DEV) if res else None
    if res:
        r.buf.normal_()
    out = {}
    for mode in ("0", "1", "1"):                      # the second fused run reuses the flags slab
        monkeypatch.setenv("STF_BN_FIN", mode)
        bn = _bn(C, 1)
        if mode == "1" and "1" in out:
            bn = out["bn1"]                           # the same module: the same slab
            with torch.no_grad():
                bn.running_mean.copy_(out["rm0"])
                bn.running_var.copy_(out["rv0"])
        rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
        stats = _stats(G, tiles, C, M // G, 2)
        st = nhwc.bn_finalize(stats, tiles, bn, M, True, G)
        assert (st._pending is not None) == (mode == "1")
        o = nhwc.new_feat(N, H, W, C, DEV)
        nhwc.bn_act(y, st, o, relu=True, res=r)
        nhwc.flush_batches_tracked()
        torch.cuda.synchronize()
        res_ = [o.buf.clone(), st.mean.clone(), st.invstd.clone(), st.scale.clone(), st.shift.clone(),
                bn.running_mean.clone(), bn.running_var.clone()]
        if mode == "0":
            out["0"] = res_
        elif "1" not in out:
            out["1"], out["bn1"], out["rm0"], out["rv0"] = res_, bn, rm0, rv0
        else:
            out["1b"] = res_
    for key in ("1", "1b"):
        for i, (a, b) in enumerate(zip(out["0"], out[key])):
            assert torch.equal(a, b), (key, i, (a.float() - b.float()).abs().max().item())
    assert nhwc.fin_sync_timeouts() == 0


@pytest.mark.parametrize("N,H,W,C,tiles", [(2, 16, 16, 64, 5), (2, 8, 8, 512, 3), (4, 64, 64, 128, 1500)])
def test_pooled_forward_fused_finalize_bitwise(monkeypatch, N, H, W, C, tiles):
    """bn_act with the fused 2x2 max pool (UNet Down) and one statistics group."""
    from stfunet import nhwc
    M = N * H * W
    y = nhwc.new_feat(N, H, W, C, DEV)
    y.buf.normal_()
    out = []
    for mode in ("0", "1", "1"):
        monkeypatch.setenv("STF_BN_FIN", mode)
        bn = _bn(C, 1) if mode == "0" or len(out) == 1 else bn
        if len(out) == 2:
            with torch.no_grad():
                bn.running_mean.copy_(rm0)
                bn.running_var.copy_(rv0)
        rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
        st = nhwc.bn_finalize(_stats(1, tiles, C, M, 2), tiles, bn, M, True, 1)
        o = nhwc.new_feat(N, H, W, C, DEV)
        pooled = nhwc.new_feat(N, H // 2, W // 2, C, DEV)
        nhwc.bn_act(y, st, o, relu=True, pooled=pooled)
        assert st._pending is None
        nhwc.flush_batches_tracked()
        torch.cuda.synchronize()
        out.append([o.buf.clone(), pooled.buf.clone(), st.mean.clone(), st.scale.clone(), st.shift.clone(),
                    bn.running_mean.clone(), bn.running_var.clone()])
    for k in (1, 2):
        for i, (a, b) in enumerate(zip(out[0], out[k])):
            assert torch.equal(a, b), (k, i)
    assert nhwc.fin_sync_timeouts() == 0


@pytest.mark.parametrize("N,H,W,C,G,tiles", SHAPES)
@pytest.mark.parametrize("mask", [False, True])
def test_backward_fused_finalize_bitwise(monkeypatch, N, H, W, C, G, tiles, mask):
    from stfunet import nhwc
    M = N * H * W
    y = nhwc.new_feat(N, H, W, C, DEV)
    y.buf.normal_()
    gin = nhwc.new_feat(N, H, W, C, DEV)
    gin.buf.normal_()
    bn = _bn(C, 3)
    monkeypatch.setenv("STF_BN_FIN", "0")
    st = nhwc.bn_finalize(_stats(G, tiles, C, M // G, 4), tiles, bn, M, True, G)
    nhwc.flush_batches_tracked()                      # (its deferred running-statistics update)
    torch.cuda.synchronize()
    out = {}
    for k, mode in enumerate(("0", "1", "1")):
        monkeypatch.setenv("STF_BN_FIN", mode)
        part = _stats(G, tiles, C, M // G, 5)
        dgamma = torch.zeros(C, device=DEV)
        dbeta = torch.zeros(C, device=DEV)
        dst = nhwc.new_feat(N, H, W, C, DEV)
        nhwc.bn_backward_from_partial(gin, y, st, bn, part, tiles, dgamma, dbeta, out=dst, mask_relu=mask)
        nhwc.flush_bn_grads()
        torch.cuda.synchronize()
        out[k] = [dst.buf.clone(), dgamma, dbeta]
    for k in (1, 2):
        for i, (a, b) in enumerate(zip(out[0], out[k])):
            assert torch.equal(a, b), (k, i, (a.float() - b.float()).abs().max().item())
    assert nhwc.fin_sync_timeouts() == 0


def _train_steps(model, x, t, steps):
    from stfunet.loss import criterion
    res = []
    for _ in range(steps):
        for p in model.parameters():
            p.grad = None
        out = model(x)["out"]
        loss = criterion({"out": out}, t)
        loss.backward()
        res.append([out.detach().clone(), loss.detach().clone()] +
                   [p.grad.detach().clone() for p in model.parameters()] +
                   [b.detach().clone() for b in model.buffers()])
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("model", ["stf", "unet"])
def test_training_step_fused_finalize_bitwise(monkeypatch, model):
    """Three training steps (eager + record, then two plan replays) with the fused finalize equal
    the separate-launch steps bit for bit: logits, loss, every gradient and every buffer
    (running statistics, num_batches_tracked)."""
    from oracle.init import canonical_state_dict
    from stfunet import STFLSTMUNet, UNet, nhwc
    if model == "stf":
        g = np.load(os.path.join(GOLDEN, "stf_t4.npz"))
        x, t = torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["target"]).to(DEV)
    else:
        from stfunet.synthetic import dce_batch
        x, t = dce_batch(4, 3, 64, 64, seed=6, device=DEV)
        x = x.flatten(1, 2)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("STF_BN_FIN", mode)
        if model == "stf":
            m = STFLSTMUNet(time_steps=4)
            m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
        else:
            torch.manual_seed(11)
            m = UNet(in_channels=3, num_classes=2, base_c=32)
        m = m.to(DEV).train()
        res[mode] = _train_steps(m, x, t, 3)
    for s, (a_s, b_s) in enumerate(zip(res["0"], res["1"])):
        for i, (a, b) in enumerate(zip(a_s, b_s)):
            assert torch.equal(a, b), (s, i)
    assert nhwc.fin_sync_timeouts() == 0
