"""Split-reduction path of vo_conv1d for fp32 convs over short sequences (T_out <= 16: the glyph
encoder's FFT blocks and the variance predictors at T_src ~ 12; SubLayers.py:85-93,
modules.py:216-259).  Each split adds its fp32 partial in a fixed order, so the result is
deterministic; it differs from the unsplit kernel only by fp32 summation order (<= 1e-5
rel-L2 against PyTorch fp32, the fp32 module tolerance of SURVEY.md 8(c))."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [  # B, T, Ci, Co, K, post, res
    (32, 12, 256, 1024, 9, "relu", False),   # FFN w_1
    (32, 12, 1024, 256, 1, None, True),      # FFN w_2 + residual
    (32, 12, 256, 256, 3, "relu", False),    # variance predictor conv
    (4, 16, 256, 1024, 9, "relu", False),
    (3, 1, 256, 256, 3, None, False),        # one glyph
    (2, 5, 80, 128, 5, "tanh", True),        # Ci not a multiple of 32
]


def _conv(x, w, b, K, post, res, cfg):
    from visual_onoma_to_wave_amd import _lib, ops
    act = {None: ops.ACT_NONE, "relu": ops.ACT_RELU, "tanh": ops.ACT_TANH}[post]
    wp = ops.pack_conv_weight(w, torch.float32)
    _lib.lib().vo_tune(b"splitk_cfg", cfg)
    try:
        y = ops.conv1d(x, wp, b, Co=w.shape[0], K=K, pad=(K - 1) // 2, post_act=act, res1=res, out_scale=0.5,
                       compute_dtype=torch.float32, out_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        _lib.lib().vo_tune(b"splitk_cfg", 0)
    return y


@pytest.mark.parametrize("B,T,Ci,Co,K,post,use_res", CASES)
def test_splitk_matches_unsplit_and_torch(device, B, T, Ci, Co, K, post, use_res):
    g = torch.Generator().manual_seed(Ci + Co + K + T)
    x = torch.randn(B, T, Ci, generator=g).to(device)
    w = (torch.randn(Co, Ci, K, generator=g) / (Ci * K) ** 0.5).to(device)
    b = torch.randn(Co, generator=g).to(device)
    res = torch.randn(B, T, Co, generator=g).to(device) if use_res else None
    y = _conv(x, w, b, K, post, res, 0)
    y1 = _conv(x, w, b, K, post, res, 1)
    assert torch.equal(y, _conv(x, w, b, K, post, res, 0))  # deterministic
    ref = F.conv1d(x.transpose(1, 2), w, b, padding=(K - 1) // 2).transpose(1, 2)
    ref = {None: ref, "relu": F.relu(ref), "tanh": torch.tanh(ref)}[post]
    if use_res:
        ref = ref + res
    ref = ref * 0.5
    for out in (y, y1):
        err = ((out - ref).norm() / ref.norm()).item()
        assert err < 1e-5, err


def test_splitk_workspace_query(device):
    """The query names a split for the FFN w_1 shape only in fp32 and only for short sequences."""
    from visual_onoma_to_wave_amd import _lib
    d = _lib.Conv1dDesc()
    d.B, d.T_in, d.T_out, d.Ci, d.Co, d.K, d.dil, d.pad = 32, 12, 12, 256, 1024, 9, 1, 4
    d.ldx, d.ldy = 256, 1024
    d.x_dtype = d.y_dtype = d.compute_dtype = _lib.VO_F32
    n = _lib.lib().vo_conv1d_workspace_size(ctypes.byref(d))
    assert n == 8 * 32 * 12 * 1024 * 4  # K = 9: one chunk (9 steps) per split
    d.T_out = d.T_in = 512
    assert _lib.lib().vo_conv1d_workspace_size(ctypes.byref(d)) == 0
    d.T_out = d.T_in = 12
    d.x_dtype = d.y_dtype = d.compute_dtype = _lib.VO_BF16
    assert _lib.lib().vo_conv1d_workspace_size(ctypes.byref(d)) == 0
