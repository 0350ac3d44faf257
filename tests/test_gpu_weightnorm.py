"""Batched weight normalisation (vo_weight_norm / vo_weight_norm_bwd, hifigan/gan_ops.WeightNormFn)
against PyTorch's torch._weight_norm(v, g, 0) and its autograd, on the HiFi-GAN layer shapes: Conv1d
(Co, Ci, K), the MPD's Conv2d (Co, Ci, K, 1), grouped MSD convs (Co, Ci / g, K), ConvTranspose1d
(Ci, Co, K) -- row lengths that are and are not multiples of 4, and more layers than one launch
holds (24)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(32, 1, 5, 1), (128, 32, 5, 1), (1024, 1024, 5, 1), (1, 1024, 3, 1), (128, 1, 15), (128, 32, 41),
          (1024, 64, 41), (256, 128, 16), (512, 80, 7), (32, 32, 11), (1, 32, 7), (3, 3, 3)]


def _layers(seed, n):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n):
        shp = SHAPES[i % len(SHAPES)]
        v = torch.randn(shp, generator=g) * 0.05
        gain = torch.rand((shp[0],) + (1,) * (len(shp) - 1), generator=g) + 0.5
        out.append((v.cuda(), gain.cuda()))
    return out


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("n", [1, 12, 30])
def test_weight_norm_forward_backward_vs_torch(device, n):
    from visual_onoma_to_wave_amd.hifigan import gan_ops as G
    layers = _layers(n, n)
    vs = [v.clone().requires_grad_(True) for v, _ in layers]
    gs = [g.clone().requires_grad_(True) for _, g in layers]
    ws = G.WeightNormFn.apply(n, *vs, *gs)
    vr = [v.clone().requires_grad_(True) for v, _ in layers]
    gr = [g.clone().requires_grad_(True) for _, g in layers]
    wr = [torch._weight_norm(v, g, 0) for v, g in zip(vr, gr)]
    for w, r in zip(ws, wr):
        assert w.shape == r.shape
        assert rel(w, r) < 1e-6
    up = [torch.randn_like(w) for w in ws]
    torch.autograd.backward(ws, up)
    torch.autograd.backward(wr, up)
    for a, b in zip(vs + gs, vr + gr):
        assert rel(a.grad, b.grad) < 1e-5, (a.shape, rel(a.grad, b.grad))


def test_weight_norm_deterministic_and_no_grad_path(device):
    from visual_onoma_to_wave_amd import ops
    layers = _layers(7, 26)
    vs, gs = [v for v, _ in layers], [g for _, g in layers]
    a = ops.weight_norm(vs, gs)
    b = ops.weight_norm(vs, gs)
    for x, y, (v, g) in zip(a, b, layers):
        assert torch.equal(x, y)
        assert rel(x, torch._weight_norm(v, g, 0)) < 1e-6


def test_weight_norm_rejects_bad_tables(device):
    from visual_onoma_to_wave_amd import ops
    v = torch.randn(4, 3, 5, device="cuda")
    with pytest.raises(ValueError):
        ops.weight_norm([v], [torch.ones(3, device="cuda")])  # one gain per row of dim 0
    with pytest.raises(ValueError):
        ops.weight_norm([v.transpose(1, 2)], [torch.ones(4, device="cuda")])  # contiguous only


def test_weight_norm_unaligned_outputs(device):
    """The public C ABI takes any fp32 pointers: outputs offset by one float (not 16-byte aligned)
    must take the scalar path (the float4 predicate covers w, dw and dv too)."""
    from visual_onoma_to_wave_amd import _lib, ops
    v, g = _layers(3, 2)[1]                             # (128, 32, 5, 1): 160-float rows
    rows, lens = ops._wn_check([v], [g])
    wbuf = torch.full((v.numel() + 1,), float("nan"), device="cuda")
    w = wbuf[1:].view_as(v)
    _lib.check(_lib.lib().vo_weight_norm(1, ops._ptr_table([v]), ops._ptr_table([g]), ops._ptr_table([w]), rows,
                                          lens, ops._stream(v)), "vo_weight_norm")
    assert rel(w, torch._weight_norm(v, g, 0)) < 1e-6
    dw = torch.randn_like(v)
    dvbuf = torch.full((v.numel() + 1,), float("nan"), device="cuda")
    dv = dvbuf[1:].view_as(v)
    dg = torch.empty_like(g)
    _lib.check(_lib.lib().vo_weight_norm_bwd(1, ops._ptr_table([v]), ops._ptr_table([g]), ops._ptr_table([dw]),
                                              ops._ptr_table([dv]), ops._ptr_table([dg]), rows, lens, ops._stream(v)),
               "vo_weight_norm_bwd")
    vr, gr = v.clone().requires_grad_(True), g.clone().requires_grad_(True)
    torch._weight_norm(vr, gr, 0).backward(dw)
    assert rel(dv, vr.grad) < 1e-5 and rel(dg, gr.grad) < 1e-5
