"""Split-bf16 fp32 contractions (VO_F32X3 / ops.F32X3): the mixed-precision training step's fp32 side
(encoder FFT blocks, variance predictors) computes each fp32 product as three bf16 MFMAs over the hi / lo
bf16 halves of its operands.  Accuracy bar, written here: within 2e-5 rel-L2 of a float64 reference (the
dropped lo * lo term and the lo roundings leave <= 3 * 2^-18 per product; the exact-f32 MFMA path sits
near 1e-7, bf16 near 3e-3), i.e. >= 100x closer to fp32 than the bf16 path on the same data."""

import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu

TOL = 2e-5


@pytest.mark.parametrize("B,T,Ci,Co,K,dil,act", [
    # the encoder / variance-predictor shapes at C4 (B = 32, T_src = 12), the fused q/k/v and fc Linears
    (32, 12, 256, 1024, 9, 1, 1), (32, 12, 1024, 256, 1, 1, 0), (32, 12, 256, 256, 3, 1, 1), (32, 12, 256, 768, 1, 1, 0),
    # longer sequences (tile shapes past the short-sequence path), dilation + leaky-ReLU prologue, ragged Co
    (2, 300, 256, 256, 3, 1, 0), (3, 257, 128, 128, 7, 3, 2), (2, 40, 64, 20, 3, 1, 0), (3, 9, 32, 28, 5, 1, 2),
    (5, 16, 1024, 256, 1, 1, 0), (3, 17, 256, 256, 3, 1, 1),
    # utterance-segment tiles: a batch that leaves the last tile partial, one-row utterances, halo 8 with
    # dilation, Co not a multiple of the tile
    (3, 7, 256, 64, 9, 1, 1), (7, 1, 64, 512, 3, 1, 0), (6, 16, 32, 48, 5, 2, 2)])
def test_conv1d_f32x3_vs_float64(B, T, Ci, Co, K, dil, act):
    from visual_onoma_to_wave_amd import ops
    g = torch.Generator().manual_seed(B * 100 + T + Co)
    x = torch.randn(B, T, Ci, generator=g)
    w = torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5
    b = torch.randn(Co, generator=g) * 0.1
    pad = dil * (K - 1) // 2
    xin = F.leaky_relu(x.double(), 0.1) if act == 2 else x.double()
    ref = F.conv1d(xin.transpose(1, 2), w.double(), b.double(), padding=pad, dilation=dil).transpose(1, 2)
    if act == 1:
        ref = F.relu(ref)
    kw = dict(Co=Co, K=K, dil=dil, pad=pad, pre_act=ops.ACT_LRELU if act == 2 else 0, pre_slope=0.1,
              post_act=ops.ACT_RELU if act == 1 else 0, out_dtype=torch.float32)
    wp = ops.pack_conv_weight(w.cuda(), torch.float32)
    got = ops.conv1d(x.cuda(), wp, b.cuda(), compute_dtype=ops.F32X3, **kw)
    again = ops.conv1d(x.cuda(), wp, b.cuda(), compute_dtype=ops.F32X3, **kw)
    assert torch.equal(got, again)
    e3 = rel_l2(got.double().cpu(), ref)
    wb = ops.pack_conv_weight(w.cuda(), torch.bfloat16)
    e16 = rel_l2(ops.conv1d(x.cuda(), wb, b.cuda(), compute_dtype=torch.bfloat16, **kw).double().cpu(), ref)
    print(f"F32X3 rel-L2 {e3:.2e}, bf16 {e16:.2e}")
    assert e3 < TOL and e3 * 100 < e16, (e3, e16)


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("B,T,Ci,Co,K,dil,pad,pre", [
    (32, 12, 256, 1024, 9, 1, 4, None), (32, 12, 1024, 256, 1, 1, 0, None), (32, 12, 256, 256, 3, 1, 1, None),
    (2, 300, 80, 512, 7, 1, 3, None), (3, 517, 256, 256, 3, 1, 1, 0.1), (1, 5, 64, 64, 7, 3, 9, 0.1)])
def test_conv1d_wgrad_f32x3_vs_float64(B, T, Ci, Co, K, dil, pad, pre, bias):
    from visual_onoma_to_wave_amd import ops
    if bias and pre is not None:
        pytest.skip("the fused bias sums dY as stored; pre applies to x here, kept to the plain case")
    g = torch.Generator().manual_seed(T + K + Ci + Co)
    x = torch.randn(B, T, Ci, generator=g)
    T_out = T + 2 * pad - dil * (K - 1)
    gy = torch.randn(B, T_out, Co, generator=g)
    xa = F.leaky_relu(x.double(), pre) if pre is not None else x.double()
    ref = torch.nn.grad.conv1d_weight(xa.transpose(1, 2), (Co, Ci, K), gy.double().transpose(1, 2), padding=pad,
                                      dilation=dil)
    kw = dict(dil=dil, pad=pad, pre_b=pre, with_bias=bias, split=True)
    got = ops.conv1d_wgrad(gy.cuda(), x.cuda(), K, **kw)
    again = ops.conv1d_wgrad(gy.cuda(), x.cuda(), K, **kw)
    gw, ag = (got[0], again[0]) if bias else (got, again)
    assert torch.equal(gw, ag)
    e3 = rel_l2(gw.double().cpu(), ref)
    e16 = rel_l2(ops.conv1d_wgrad(gy.cuda().bfloat16(), x.cuda().bfloat16(), K, dil=dil, pad=pad,
                                  pre_b=pre).double().cpu(), ref)
    print(f"F32X3 wgrad rel-L2 {e3:.2e}, bf16 {e16:.2e}")
    assert e3 < TOL and e3 * 100 < e16, (e3, e16)
    if bias:
        assert torch.equal(got[1], again[1])
        assert rel_l2(got[1].double().cpu(), gy.double().sum((0, 1))) < TOL


def test_conv1d_fn_f32x3_autograd_vs_float64():
    """AG.conv1d with compute_dtype ops.F32X3 (forward, input and weight / bias gradients) against float64
    autograd on the CPU -- the encoder FFN w_1 at C4."""
    from visual_onoma_to_wave_amd import autograd as AG, ops
    g = torch.Generator().manual_seed(7)
    B, T, Ci, Co, K = 32, 12, 256, 1024, 9
    x = torch.randn(B, T, Ci, generator=g)
    w = torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5
    b = torch.randn(Co, generator=g) * 0.1
    gy = torch.randn(B, T, Co, generator=g)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yd = F.relu(F.conv1d(xd.transpose(1, 2), wd, bd, padding=K // 2)).transpose(1, 2)
    yd.backward(gy.double())
    xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
    yc = AG.conv1d(xc, wc, bc, K=K, pad=K // 2, relu=True, compute_dtype=ops.F32X3)
    assert yc.dtype == torch.float32
    yc.backward(gy.cuda())
    for name, got, ref in (("y", yc, yd), ("dx", xc.grad, xd.grad), ("dw", wc.grad, wd.grad), ("db", bc.grad, bd.grad)):
        e = rel_l2(got.detach().double().cpu(), ref.detach())
        print(name, f"{e:.2e}")
        assert e < TOL, (name, e)


@pytest.mark.parametrize("cdt", ["f32", "x3"])
@pytest.mark.parametrize("B,T,Ci,Co,K,dil", [(32, 12, 256, 1024, 9, 1), (5, 16, 1024, 256, 1, 1), (3, 7, 256, 64, 9, 1),
                                             (6, 16, 32, 48, 5, 2)])
def test_segment_tiles_bit_identical(B, T, Ci, Co, K, dil, cdt):
    """The utterance-segment tiles (default, seg_cfg 3 = 8 utterances per tile) and the one-utterance tiles
    (seg_cfg 4) give bit-identical outputs: per element the same chunk / tap / split order."""
    from visual_onoma_to_wave_amd import _lib, ops
    L = _lib.lib()
    g = torch.Generator().manual_seed(B + T + Co)
    x = torch.randn(B, T, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5).cuda()
    b = (torch.randn(Co, generator=g) * 0.1).cuda()
    wp = ops.pack_conv_weight(w, torch.float32)
    cd = ops.F32X3 if cdt == "x3" else torch.float32
    outs = []
    try:
        for cfg in (0, 3, 4):
            assert L.vo_tune(b"seg_cfg", cfg) == 0
            outs.append(ops.conv1d(x, wp, b, Co=Co, K=K, dil=dil, pad=dil * (K - 1) // 2, post_act=ops.ACT_RELU,
                                   compute_dtype=cd))
    finally:
        L.vo_tune(b"seg_cfg", 0)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
