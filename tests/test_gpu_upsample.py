"""HiFi-GAN generator tail kernels: the streaming polyphase upsampler (csrc/upsample.hip, ups2
128 -> 64 and ups3 64 -> 32, k4 s2) and the row-partials conv_post (csrc/vocoder_glue.hip).

The HiFi-GAN ConvTranspose1d (scripts/hifigan/models.py:139-141,153-154, lrelu 0.1 in front)
in its bf16 polyphase form runs on `ups_kernel` when the output is bf16; the generic tiled conv
(`vo_tune("ups_cfg", 1)`) is the same arithmetic in the same order, so the two must agree
bit for bit.  Both are checked against a plain PyTorch fp32 ConvTranspose1d (rel-L2 <= 1e-2,
the bf16 tolerance of SURVEY.md 8(c))."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _run(x, w_t, bias, u, k, slope, cfg):
    from visual_onoma_to_wave_amd import _lib, ops
    wb = ops.pack_conv_weight(w_t, torch.bfloat16, transposed_stride=u)
    _lib.lib().vo_tune(b"ups_cfg", cfg)
    try:
        pre = ops.ACT_LRELU if slope is not None else ops.ACT_NONE
        y = ops.conv1d(x, wb, bias, Co=u * w_t.shape[1], K=2, pad=1, pre_act=pre,
                       pre_slope=slope if slope is not None else 0.0,
                       transposed=dict(stride=u, pad=(k - u) // 2, cout=w_t.shape[1]),
                       out_dtype=torch.bfloat16, compute_dtype=torch.bfloat16)
        torch.cuda.synchronize()
    finally:
        _lib.lib().vo_tune(b"ups_cfg", 0)
    return y


def _ref(x, w_t, bias, u, k, slope):
    xt = x.float().transpose(1, 2)
    if slope is not None:
        xt = F.leaky_relu(xt, slope)
    return F.conv_transpose1d(xt, w_t.to(torch.bfloat16).float(), bias, stride=u,
                              padding=(k - u) // 2).transpose(1, 2)


@pytest.mark.parametrize("Ci,Cout", [(128, 64), (64, 32)])
@pytest.mark.parametrize("B,T", [(1, 1), (1, 15), (2, 16), (3, 17), (2, 31), (1, 33), (4, 1000), (32, 4096)])
@pytest.mark.parametrize("slope", [0.1, None])
def test_ups_stream_matches_generic_and_torch(device, Ci, Cout, B, T, slope):
    u, k = 2, 4
    g = torch.Generator().manual_seed(1234 + T + Ci)
    x = torch.randn(B, T, Ci, generator=g).to(torch.bfloat16).to(device)
    w_t = (torch.randn(Ci, Cout, k, generator=g) * 0.05).to(device)
    bias = torch.randn(Cout, generator=g).to(device)
    y = _run(x, w_t, bias, u, k, slope, 0)
    y_gen = _run(x, w_t, bias, u, k, slope, 1)
    assert y.shape == (B, 2 * T, Cout)
    assert torch.equal(y, y_gen), (y.float() - y_gen.float()).abs().max().item()
    ref = _ref(x, w_t, bias, u, k, slope)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("Ci,Cout", [(256, 128)])
@pytest.mark.parametrize("B,T", [(1, 1), (2, 17), (3, 100), (4, 513)])
def test_ups_wide_matches_generic_and_torch(device, Ci, Cout, B, T):
    """ups1 shape (k16 s8): column-block kernel (upsw_kernel) vs the tiled conv."""
    u, k = 8, 16
    g = torch.Generator().manual_seed(77 + T)
    x = torch.randn(B, T, Ci, generator=g).to(torch.bfloat16).to(device)
    w_t = (torch.randn(Ci, Cout, k, generator=g) * 0.05).to(device)
    bias = torch.randn(Cout, generator=g).to(device)
    y = _run(x, w_t, bias, u, k, 0.1, 0)
    y_gen = _run(x, w_t, bias, u, k, 0.1, 1)
    assert y.shape == (B, 8 * T, Cout)
    assert torch.equal(y, y_gen), (y.float() - y_gen.float()).abs().max().item()
    ref = _ref(x, w_t, bias, u, k, 0.1)
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_ups_stream_c3_size(device):
    """C3-sized ups1 / ups2 / ups3 (B = 32 x 512 frames): bit-identical to the generic path."""
    for Ci, Cout, T, u, k in ((128, 64, 32768, 2, 4), (64, 32, 65536, 2, 4), (256, 128, 4096, 8, 16)):
        g = torch.Generator().manual_seed(Ci)
        x = torch.randn(32, T, Ci, generator=g).to(torch.bfloat16).to(device)
        w_t = (torch.randn(Ci, Cout, k, generator=g) * 0.05).to(device)
        bias = torch.randn(Cout, generator=g).to(device)
        y = _run(x, w_t, bias, u, k, 0.1, 0)
        y_gen = _run(x, w_t, bias, u, k, 0.1, 1)
        assert torch.equal(y, y_gen), Ci
        del x, y, y_gen


@pytest.mark.parametrize("B,T", [(1, 1), (1, 5), (2, 250), (3, 251), (1, 1000), (2, 131072)])
def test_conv_post_rows_kernel(device, B, T):
    """HiFi-GAN tail lrelu(0.01) -> Conv1d(32 -> 1, k7, pad 3) -> tanh (models.py:161-163) on
    the row-partials kernel (bf16 input, C = 32, K = 7) against the LDS-stencil kernel
    (`post_cfg` 1; same math, another fp32 summation order) and PyTorch fp32."""
    from visual_onoma_to_wave_amd import _lib, ops
    g = torch.Generator().manual_seed(T)
    x = torch.randn(B, T, 32, generator=g).to(torch.bfloat16).to(device)
    w = (torch.randn(1, 32, 7, generator=g) * 0.1).to(device)
    bias = 0.05
    w_kc = w[0].t().contiguous()
    y = ops.conv_post(x, w_kc, bias, slope=0.01)
    _lib.lib().vo_tune(b"post_cfg", 1)
    try:
        y_st = ops.conv_post(x, w_kc, bias, slope=0.01)
    finally:
        _lib.lib().vo_tune(b"post_cfg", 0)
    ref = torch.tanh(F.conv1d(F.leaky_relu(x.float().transpose(1, 2), 0.01), w, torch.tensor([bias], device=device),
                              padding=3))[:, 0]
    assert y.shape == (B, T)
    assert (y - y_st).abs().max().item() < 1e-5
    assert (y - ref).abs().max().item() < 1e-5
