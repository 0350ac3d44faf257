"""vo_pack_dgrad_phase (the input-gradient weights of one stride phase of a strided / grouped
discriminator conv, hifigan/gan_ops._dgrad) against the PyTorch composition it replaces: per-group
transpose, zero rows for padded input channels, the phase's taps reversed, grouped packing -- bit
for bit, dense and into a persistent zeroed buffer (diagonal blocks only)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

# (Co, Ci, K, groups, S, ci_out, co_in): MPD layers (K 5, S 3; first layer Ci 1 padded to 8, post Co 1
# padded to 8), MSD grouped layers (K 41, S 2 / 4, groups 4 / 16)
CASES = [(32, 1, 5, 1, 3, 8, 32), (128, 32, 5, 1, 3, 32, 128), (1024, 512, 5, 1, 3, 512, 1024),
         (128, 128, 41, 4, 2, 128, 128), (256, 128, 41, 16, 2, 128, 256), (1024, 512, 41, 16, 4, 512, 1024),
         (128, 1, 15, 1, 1, 8, 128), (1, 1024, 3, 1, 1, 1024, 8)]


def _reference(w, g, S, k_r, ci_out, co_in, dt):
    from visual_onoma_to_wave_amd import ops
    Co, cig, K = w.shape
    cog, Ci = Co // g, cig * g
    wt = w.float().reshape(g, cog, cig, K).transpose(1, 2).reshape(Ci, cog, K)
    if ci_out > Ci:
        wt = torch.cat([wt, wt.new_zeros((ci_out - Ci, cog, K))])
    wsel = wt[:, :, k_r::S].flip(-1).contiguous()
    return ops.pack_grouped_weight(wsel, dt, g if ci_out == Ci else 1, co_in)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Co,Ci,K,g,S,ci_out,co_in", CASES)
def test_pack_dgrad_phase_matches_torch_composition(device, dt, Co, Ci, K, g, S, ci_out, co_in):
    from visual_onoma_to_wave_amd import ops
    gen = torch.Generator().manual_seed(Co + Ci + K + g + S)
    w = torch.randn(Co, Ci // g, K, generator=gen).cuda()
    for k_r in range(min(S, K)):
        J = len(range(k_r, K, S))
        ref = _reference(w, g, S, k_r, ci_out, co_in, dt)
        got = ops.pack_dgrad_phase(w, g, S, k_r, J, ci_out, co_in, dt)
        assert got.shape == ref.shape and torch.equal(got, ref), (k_r, J)
        slot = torch.zeros((J, ci_out, co_in), dtype=dt, device="cuda")
        got2 = ops.pack_dgrad_phase(w, g, S, k_r, J, ci_out, co_in, dt, out=slot)
        assert got2.data_ptr() == slot.data_ptr() and torch.equal(got2, ref), (k_r, J)
