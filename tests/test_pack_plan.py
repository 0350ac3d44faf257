"""gan_ops._pack_plan (the layouts gan_ops.prepack writes in one vo_pack_batch launch) against the
layouts the per-conv paths allocate, on the C5 step's real layer list -- host logic only (the
bit-exact GPU comparison is tests/test_gpu_gan.py::test_pack_batch_matches_single_packs)."""

import torch

from helpers import hifigan_h


def _layers():
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.hifigan import gan_ops as G
    from visual_onoma_to_wave_amd.hifigan.discriminators import (MultiPeriodDiscriminator, MultiScaleDiscriminator,
                                                                 _conv_w)

    def wshape(m):
        return tuple(_conv_w(m, m.weight_v if hasattr(m, "weight_g") else m.weight_orig).shape)
    out = [(wshape(m), G.conv_spec(s, sp, r), s) for m, sp, s, r in
           hifigan.Generator(hifigan.AttrDict(hifigan_h()))._train_plan(16, 32)]
    for d in MultiPeriodDiscriminator().discriminators:
        out += [(wshape(m), G.conv_spec(s, sp), s) for m, sp, s in d._layers(32, 8192)]
    T = 8192
    for i, d in enumerate(MultiScaleDiscriminator().discriminators):
        T = T // 2 + 1 if i else T
        out += [(wshape(m), G.conv_spec(s, sp), s) for m, sp, s in d._layers(32, T)]
    return out


def test_pack_plan_layouts_match_the_per_conv_paths():
    from visual_onoma_to_wave_amd.hifigan import gan_ops as G
    layers = _layers()
    assert len(layers) == 78 + 30 + 24
    dt = torch.bfloat16
    for wshape, spec, shape in layers:
        plan = {tag: (dshape, f) for tag, dshape, f in G._pack_plan(wshape, spec, dt, shape[-1], True)}
        fwd_shape, f = plan[(spec, dt, "fwd")]
        if spec.transposed is not None:
            Ci, Co, K = wshape
            s = spec.transposed[0]
            assert fwd_shape == (2, s * Co, Ci) and (spec, dt, "dgrad_convt") in plan
        else:
            Co, cig, K = wshape
            co_rows = max(Co, spec.co_pad or 0)
            ld = cig * spec.groups if spec.ci_pad is None else spec.ci_pad
            assert fwd_shape == (K, co_rows, ld), (wshape, spec)
            if spec.plain():
                assert plan[(spec, dt, "dgrad_plain")][0] == (K, cig, Co)
            else:  # one input-gradient layout per stride phase that has taps (gan_ops._dgrad)
                S = spec.stride
                phases = [r for r in range(S) if len(range((r + spec.pad) % S, K, S))]
                co_in = -(-Co // 8) * 8
                for r in phases:
                    J = len(range((r + spec.pad) % S, K, S))
                    assert plan[(spec, dt, "dgrad", r, shape[-1], co_in)][0] == (J, shape[-1], co_in)
                assert len(plan) == 1 + len(phases)
        for dshape, f in plan.values():  # every job stays inside its destination and its source
            assert f["T"] == dshape[0] and f["dst_rows"] == dshape[1] and f["ld"] == dshape[2]
            assert ((f["rows"] - 1) // f["rpg"]) * f["cpg"] + f["width"] <= f["ld"]
            if f["mode"] == 0:
                last = f["tap0"] + f["tstep"] * (f["T"] - 1)
                assert 0 <= min(f["tap0"], last) and max(f["tap0"], last) < f["K"]
                assert abs(f["tstep"]) * (f["T"] - 1) + 1 <= 48


def test_joined_spec_predicate():
    """conv_spec: short sequences (N >= 8, T_out <= 64, dense, no dilation, no residual) run joined
    with their padding made explicit; anything else keeps its spec."""
    from visual_onoma_to_wave_amd.hifigan import gan_ops as G
    sp = G.ConvSpec(K=5, pad=2, stride=3)
    assert G.conv_spec((16, 100, 32), sp).pad == 0
    assert G.conv_spec((4, 100, 32), sp) == sp                     # too few sequences
    assert G.conv_spec((16, 1000, 32), sp) == sp                   # too long
    assert G.conv_spec((16, 100, 32), sp, has_res=True) == sp      # residual inputs
    assert G.conv_spec((16, 30, 32), G.ConvSpec(K=3, pad=3, dil=3)).dil == 3 and \
        G.conv_spec((16, 30, 32), G.ConvSpec(K=3, pad=3, dil=3)).pad == 3
