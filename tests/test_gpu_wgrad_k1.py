"""The K = 1 weight-gradient kernel (wgrad_k1_kernel: the decoder's Linear layers at C4) against the per-tap
kernel (vo_tune wgrad_cfg 14) on the same bf16 operands -- fp32 sums of the same products in other groupings:
<= 1e-6 rel-L2 -- and against torch in float64; the fused bias against the column sums; deterministic run
to run; every split plan (wgrad_cfg 15 / 16) gives the same result within the grouping bar."""

import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("B,T,Ci,Co", [
    # C4 decoder shapes (B = 32, T_mel = 512): q/k/v, fc, FFN w_2, mel_linear
    (32, 512, 256, 768), (32, 512, 256, 256), (32, 512, 1024, 256), (32, 512, 256, 80),
    # ragged rows (a chunk and a split cut mid-way), tiles partly outside M and N, one short utterance
    (3, 777, 1024, 256), (2, 300, 40, 200), (1, 5, 64, 64), (7, 100, 136, 520)])
def test_wgrad_k1_vs_per_tap_and_float64(B, T, Ci, Co, bias):
    from visual_onoma_to_wave_amd import _lib, ops
    L = _lib.lib()
    g = torch.Generator().manual_seed(B * T + Ci + Co)
    x = torch.randn(B, T, Ci, generator=g).to(torch.bfloat16)
    gy = torch.randn(B, T, Co, generator=g).to(torch.bfloat16)
    xa, gya = x.cuda(), gy.cuda()
    try:
        assert L.vo_tune(b"wgrad_cfg", 14) == 0
        ref = ops.conv1d_wgrad(gya, xa, 1, with_bias=bias)
        outs = []
        for cfg in (0, 15, 16):
            assert L.vo_tune(b"wgrad_cfg", cfg) == 0
            outs.append(ops.conv1d_wgrad(gya, xa, 1, with_bias=bias))
        assert L.vo_tune(b"wgrad_cfg", 0) == 0
        again = ops.conv1d_wgrad(gya, xa, 1, with_bias=bias)
    finally:
        L.vo_tune(b"wgrad_cfg", 0)
    refw, gw, agw = (ref[0], outs[0][0], again[0]) if bias else (ref, outs[0], again)
    assert gw.shape == (Co, Ci, 1)
    assert torch.equal(gw, agw)
    assert rel_l2(gw.cpu(), refw.cpu()) < 1e-6, rel_l2(gw.cpu(), refw.cpu())
    for o in outs[1:]:
        ow = o[0] if bias else o
        assert rel_l2(ow.cpu(), refw.cpu()) < 1e-6
    t64 = torch.einsum("btm,btn->mn", gy.double(), x.double())[:, :, None]
    assert rel_l2(gw.double().cpu(), t64) < 1e-5
    if bias:
        assert torch.equal(outs[0][1], again[1])
        assert rel_l2(outs[0][1].double().cpu(), gy.double().sum((0, 1))) < 1e-6


@pytest.mark.parametrize("B,T,Ci,Co,K,out_dt", [
    (32, 512, 1024, 256, 9, torch.bfloat16),  # the C4 decoder's FFN w_1 input gradient
    (16, 1000, 1024, 128, 9, torch.float32), (9, 911, 512, 64, 5, torch.bfloat16), (32, 512, 2048, 256, 1, torch.bfloat16)])
def test_conv1d_bf16_split_reduction(B, T, Ci, Co, K, out_dt):
    """Deep bf16 convs into <= 256 channels run on the 256 x 256 tile with their chunks split over workgroups
    (fp32 partials added in split order): against torch fp32 (bf16 bar 1e-2), against the unsplit tiles
    (splitk_cfg 3) within the output rounding, and deterministic run to run."""
    import torch.nn.functional as F
    from visual_onoma_to_wave_amd import _lib, ops
    L = _lib.lib()
    g = torch.Generator().manual_seed(B + T + Ci + Co)
    x = torch.randn(B, T, Ci, generator=g).to(torch.bfloat16)
    w = torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5
    wp = ops.pack_conv_weight(w.cuda(), torch.bfloat16)
    ref = F.conv1d(x.float().transpose(1, 2), w.bfloat16().float(), padding=K // 2).transpose(1, 2)
    kw = dict(Co=Co, K=K, pad=K // 2, out_dtype=out_dt, compute_dtype=torch.bfloat16)
    try:
        got = ops.conv1d(x.cuda(), wp, None, **kw)
        again = ops.conv1d(x.cuda(), wp, None, **kw)
        assert L.vo_tune(b"splitk_cfg", 3) == 0
        unsplit = ops.conv1d(x.cuda(), wp, None, **kw)
    finally:
        L.vo_tune(b"splitk_cfg", 0)
    assert torch.equal(got, again)
    assert rel_l2(got.float().cpu(), ref) < 1e-2
    assert rel_l2(got.float().cpu(), unsplit.float().cpu()) < (4e-3 if out_dt == torch.bfloat16 else 1e-5)



@pytest.mark.parametrize("B,T,Ci,Co,K,S,g,pad", [
    # the MSD's grouped strided layers (k = 41, stride 2 / 4, groups 4 / 16), an MPD-style stride 3, ragged T
    (4, 4096, 128, 128, 41, 2, 4, 20), (4, 4096, 128, 256, 41, 2, 16, 20), (4, 2048, 256, 512, 41, 4, 16, 20),
    (3, 2731, 32, 128, 5, 3, 1, 2), (2, 1000, 64, 64, 7, 2, 1, 3), (2, 777, 128, 256, 41, 2, 16, 20),
    # short utterances (T_out 65..257, up to half of each chunk padding: many-tap convs only)
    (8, 1025, 256, 512, 41, 4, 16, 20), (8, 257, 512, 1024, 41, 4, 16, 20), (4, 128, 1024, 1024, 41, 1, 16, 20)])
def test_wgrad_multitap_strided_vs_per_tap(B, T, Ci, Co, K, S, g, pad):
    """Strided convs on the multi-tap kernel (window 64 S + 64 rows, B row = A row x S + tap) against the
    per-tap kernel (wgrad_mt 2) on the same bf16 operands, <= 1e-6 rel-L2, and against torch; deterministic."""
    import torch.nn.functional as F
    from visual_onoma_to_wave_amd import _lib, ops
    L = _lib.lib()
    gen = torch.Generator().manual_seed(B * T + K + Co + S)
    x = torch.randn(B, T, Ci, generator=gen).to(torch.bfloat16)
    T_out = (T + 2 * pad - K) // S + 1
    gy = torch.randn(B, T_out, Co, generator=gen).to(torch.bfloat16)
    xa, gya = x.cuda(), gy.cuda()
    kw = dict(S=S, pad=pad, pre_b=0.1, groups=g)
    try:
        assert L.vo_tune(b"wgrad_mt", 2) == 0
        ref = ops.conv1d_wgrad(gya, xa, K, **kw)
        assert L.vo_tune(b"wgrad_mt", 0) == 0
        got = ops.conv1d_wgrad(gya, xa, K, **kw)
        again = ops.conv1d_wgrad(gya, xa, K, **kw)
    finally:
        L.vo_tune(b"wgrad_mt", 0)
    assert torch.equal(got, again)
    assert rel_l2(got.cpu(), ref.cpu()) < 1e-6, rel_l2(got.cpu(), ref.cpu())
    xt = F.leaky_relu(x.float(), 0.1).to(torch.bfloat16).float()
    tw = torch.nn.grad.conv1d_weight(xt.transpose(1, 2), (Co, Ci // g, K), gy.float().transpose(1, 2), stride=S,
                                     padding=pad, groups=g)
    assert rel_l2(got.cpu(), tw) < 1e-5

