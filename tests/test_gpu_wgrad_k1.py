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
