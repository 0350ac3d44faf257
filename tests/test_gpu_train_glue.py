"""The round-2 training glue on HIP (train_glue.hip, disc.hip adjoints): forward and gradients
against torch autograd of the reference formulation in fp64 on the CPU.

* BatchNorm with batch statistics: PostNet's BatchNorm1d (scripts/transformer/Layers.py:129-137)
  on channels-last (B, T, C) and the glyph encoder's single-channel BatchNorm2d
  (scripts/model/visual_feature_extractor.py:40-47); running statistics and
  ``num_batches_tracked`` as nn.BatchNorm* updates them;
* the glyph encoder's Conv2d(1, 1, 3, padding=1): dx, dW, db;
* the HiFi-GAN training mel (oracle.gan.mel_spectrogram, the meldataset recipe) backward;
* the discriminator input transforms: MPD period fold (reflect pad), channels-last copy, MSD
  AvgPool1d(4, 2, padding=2).

Tolerances (relative L2): fp32 kernels 1e-5 (BatchNorm, conv: short fp32 sums), 1e-4 for the
mel backward (1024-point fp32 FFTs and a 1 / melsum factor), bf16 activations 1e-2; the
transform adjoints exact up to one fp32 rounding (<= 1e-6).
"""

import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu


def _bn_case(shape, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g, dtype=torch.float64) * 1.7 + 0.4
    gy = torch.randn(shape, generator=g, dtype=torch.float64)
    C = shape[-1] if len(shape) == 3 else 1
    bn = torch.nn.BatchNorm1d(C) if len(shape) == 3 else torch.nn.BatchNorm2d(1)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.2, 0.2, generator=g)
        bn.running_mean.uniform_(-0.1, 0.1, generator=g)
        bn.running_var.uniform_(0.8, 1.2, generator=g)
    return x, gy, bn


@pytest.mark.parametrize("shape,dtype", [((4, 300, 512), torch.float32), ((3, 77, 80), torch.float32),
                                         ((8, 512, 512), torch.bfloat16), ((384, 1, 24, 102), torch.float32),
                                         ((5, 1, 24, 7), torch.float32), ((3, 77, 80), torch.bfloat16),
                                         # vectorised kernels (C % V == 0, C = 1 with M % V == 0) and the
                                         # scalar ones (C = 1, M = 45; C = 12: not a whole bf16 vector)
                                         ((3, 1, 5, 3), torch.float32), ((2, 33, 12), torch.bfloat16),
                                         ((32, 512, 512), torch.bfloat16)])
def test_batch_norm_train_fwd_bwd(shape, dtype):
    """y, running mean / var, num_batches_tracked, dx, dgamma, dbeta vs nn.BatchNorm in train mode."""
    from visual_onoma_to_wave_amd import autograd as AG
    x, gy, bn = _bn_case(shape, dtype, sum(shape))
    ref_bn = torch.nn.BatchNorm1d(bn.num_features).double() if len(shape) == 3 else torch.nn.BatchNorm2d(1).double()
    ref_bn.load_state_dict(bn.state_dict())
    ref_bn.train()
    # the reference runs (B, C, T); ours is channels-last (B, T, C)
    xr = x.to(dtype).double().requires_grad_(True)
    yr = ref_bn(xr.transpose(1, 2) if len(shape) == 3 else xr)
    yr = yr.transpose(1, 2) if len(shape) == 3 else yr
    (yr * gy).sum().backward()

    bn = bn.cuda().train()
    xg = x.to(dtype).cuda().requires_grad_(True)
    dims = (0, 1) if len(shape) == 3 else (0, 2, 3)
    y = AG.batch_norm_train(xg, bn, dims)
    assert y.dtype == dtype and y.shape == x.shape
    y.backward(gy.to(dtype).cuda())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    errs = {"y": rel_l2(y.detach().float().cpu(), yr.detach()), "dx": rel_l2(xg.grad.float().cpu(), xr.grad),
            "dgamma": rel_l2(bn.weight.grad.cpu(), ref_bn.weight.grad),
            "dbeta": rel_l2(bn.bias.grad.cpu(), ref_bn.bias.grad),
            "running_mean": rel_l2(bn.running_mean.cpu(), ref_bn.running_mean),
            "running_var": rel_l2(bn.running_var.cpu(), ref_bn.running_var)}
    print(shape, dtype, {k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < (1e-5 if k.startswith("running") else tol) for k, v in errs.items()), errs
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1


def test_batch_norm_train_no_affine_no_tracking():
    from visual_onoma_to_wave_amd import autograd as AG
    bn = torch.nn.BatchNorm1d(64, affine=False, track_running_stats=False).cuda()
    x = torch.randn(2, 50, 64, device="cuda", requires_grad=True)
    y = AG.batch_norm_train(x, bn, (0, 1))
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = F.batch_norm(xr.transpose(1, 2), None, None, training=True).transpose(1, 2)
    g = torch.randn_like(yr)
    y.backward(g.float().cuda())
    (yr * g).sum().backward()
    assert rel_l2(y.detach().cpu(), yr.detach()) < 1e-5 and rel_l2(x.grad.cpu(), xr.grad) < 1e-5


@pytest.mark.parametrize("N,H,W", [(384, 24, 102), (3, 5, 4), (1, 1, 1)])
def test_vfe_conv_fwd_bwd(N, H, W):
    from visual_onoma_to_wave_amd import autograd as AG
    g = torch.Generator().manual_seed(N * H + W)
    conv = torch.nn.Conv2d(1, 1, 3, padding=1)
    with torch.no_grad():
        conv.weight.uniform_(-0.5, 0.5, generator=g)
        conv.bias.uniform_(-0.1, 0.1, generator=g)
    x = torch.rand(N, 1, H, W, generator=g, dtype=torch.float64)
    gy = torch.randn(N, 1, H, W, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    br = conv.bias.detach().double().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, padding=1)
    (yr * gy).sum().backward()
    conv = conv.cuda()
    xg = x.float().cuda().requires_grad_(True)
    y = AG.vfe_conv(xg, conv)
    y.backward(gy.float().cuda())
    errs = {"y": rel_l2(y.detach().cpu(), yr.detach()), "dx": rel_l2(xg.grad.cpu(), xr.grad),
            "dw": rel_l2(conv.weight.grad.cpu(), wr.grad), "db": rel_l2(conv.bias.grad.cpu(), br.grad)}
    print((N, H, W), {k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 1e-5 for v in errs.values()), errs


@pytest.mark.parametrize("B,N", [(2, 8192), (3, 4000), (1, 1024)])
def test_stft_mel_backward_vs_torch_autograd(B, N):
    """MelFn (forward vo_stft_mel_ex, backward vo_stft_mel_bwd) against autograd through
    oracle.gan.mel_spectrogram in fp64; N = 4000 is not a multiple of the hop and N = 1024 puts
    most samples inside the reflect-padded regions."""
    from oracle.mel import librosa_mel
    from visual_onoma_to_wave_amd.hifigan.discriminators import MelLoss
    g = torch.Generator().manual_seed(B * N)
    wav = (torch.rand(B, N, generator=g, dtype=torch.float64) * 2 - 1) * 0.6
    wr = wav.clone().requires_grad_(True)
    # oracle.gan.mel_spectrogram's recipe in double precision
    basis = torch.from_numpy(librosa_mel(22050, 1024, 80, 0.0, 8000.0)).double()
    p = (1024 - 256) // 2
    yy = F.pad(wr[:, None, :], (p, p), mode="reflect")[:, 0]
    spec = torch.stft(yy, 1024, hop_length=256, win_length=1024, window=torch.hann_window(1024, dtype=torch.float64),
                      center=False, return_complex=True)
    mel64 = torch.log(torch.clamp(basis @ torch.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-9), min=1e-5))
    gm = torch.randn(mel64.shape, generator=g, dtype=torch.float64)
    (mel64 * gm).sum().backward()
    ml = MelLoss(1024, 80, 22050, 256, 1024, 0, 8000.0).cuda()
    wg = wav.float().cuda().requires_grad_(True)
    mel = ml.mel(wg)
    mel.backward(gm.float().cuda())
    e_fwd = rel_l2(mel.detach().cpu(), mel64.detach())
    e_bwd = rel_l2(wg.grad.cpu(), wr.grad)
    print((B, N), f"fwd {e_fwd:.1e} bwd {e_bwd:.1e}")
    assert e_fwd < 1e-4 and e_bwd < 1e-4


@pytest.mark.parametrize("T", [8192, 8191, 8190, 100])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_disc_input_adjoints(T, dtype):
    """Period fold (p = 2, 3, 5, 7, 11: reflect pad to a multiple of p), the channels-last copy and
    AvgPool1d(4, 2, padding=2): gradients vs autograd of the reference formulation."""
    from visual_onoma_to_wave_amd.hifigan import gan_ops as GO
    g = torch.Generator().manual_seed(T)
    B = 3
    wav = torch.randn(B, T, generator=g)
    for p in (2, 3, 5, 7, 11):
        wr = wav.clone().double().requires_grad_(True)
        x = wr
        if T % p:
            x = F.pad(x[:, None, :], (0, p - T % p), "reflect")[:, 0]
        x = x.view(B, -1, p)  # (B, H, p): column c = samples h p + c
        gy = torch.randn(B * p, x.shape[1], 8, generator=g).to(dtype)
        gcol = gy[..., 0].double().view(B, p, -1).transpose(1, 2)  # (B, H, p)
        (x * gcol).sum().backward()
        wg = wav.cuda().requires_grad_(True)
        out = GO.PeriodFoldFn.apply(wg, p, dtype)
        assert out.shape == gy.shape
        out.backward(gy.cuda())
        assert rel_l2(wg.grad.cpu(), wr.grad) < 1e-6, p
    wg = wav.cuda().requires_grad_(True)
    gy = torch.randn(B, T, 8, generator=g).to(dtype)
    GO.WavCl8Fn.apply(wg, dtype).backward(gy.cuda())
    assert torch.equal(wg.grad.cpu(), gy[..., 0].float())
    wr = wav.clone().double().requires_grad_(True)
    yr = F.avg_pool1d(wr[:, None, :], 4, 2, padding=2)[:, 0]
    gp = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    (yr * gp).sum().backward()
    wg = wav.cuda().requires_grad_(True)
    y = GO.AvgPoolFn.apply(wg)
    assert y.shape == yr.shape
    y.backward(gp.float().cuda())
    assert rel_l2(wg.grad.cpu(), wr.grad) < 1e-6


@pytest.mark.parametrize("n_fft,hop,win", [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)])
def test_stft_mag_fwd_bwd(n_fft, hop, win):
    """vo_stft_mag / vo_stft_mag_bwd (StftMagFn) against torch.stft autograd in fp64."""
    from oracle import gan as G
    from visual_onoma_to_wave_amd.hifigan import gan_ops as GO
    g = torch.Generator().manual_seed(n_fft + hop)
    x = (torch.rand(2, 8192, generator=g, dtype=torch.float64) * 2 - 1) * 0.5
    xr = x.clone().requires_grad_(True)
    mr = G.stft_mag(xr, n_fft, hop, win)
    gm = torch.randn(mr.shape, generator=g, dtype=torch.float64)
    (mr * gm).sum().backward()
    window = torch.zeros(n_fft, dtype=torch.float64)
    window[(n_fft - win) // 2: (n_fft - win) // 2 + win] = torch.hann_window(win, dtype=torch.float64)
    xg = x.float().cuda().requires_grad_(True)
    m = GO.StftMagFn.apply(xg, window.float().cuda(), n_fft, hop)
    m.backward(gm.float().cuda())
    e_f, e_b = rel_l2(m.detach().cpu(), mr.detach()), rel_l2(xg.grad.cpu(), xr.grad)
    print((n_fft, hop, win), f"fwd {e_f:.1e} bwd {e_b:.1e}")
    assert m.shape == mr.shape and e_f < 1e-5 and e_b < 1e-4


def test_multi_resolution_stft_loss_vs_oracle():
    """MultiResolutionSTFTLoss (HIP magnitudes, reductions and gradients) against
    oracle.gan.multi_resolution_stft_loss autograd in fp64: both loss terms and d/dwav_hat."""
    from oracle import gan as G
    from visual_onoma_to_wave_amd.hifigan.discriminators import MultiResolutionSTFTLoss
    g = torch.Generator().manual_seed(3)
    y = (torch.rand(3, 8192, generator=g, dtype=torch.float64) * 2 - 1) * 0.5
    x = y + 0.1 * torch.randn(3, 8192, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    sc_r, mag_r = G.multi_resolution_stft_loss(xr, y)
    (sc_r + 0.5 * mag_r).backward()
    loss = MultiResolutionSTFTLoss().cuda()
    xg = x.float().cuda().requires_grad_(True)
    sc, mag = loss(xg, y.float().cuda())
    (sc + 0.5 * mag).backward()
    print(f"sc {float(sc):.6f} vs {float(sc_r):.6f}, mag {float(mag):.6f} vs {float(mag_r):.6f}, "
          f"grad {rel_l2(xg.grad.cpu(), xr.grad):.1e}")
    assert abs(float(sc) - float(sc_r)) < 1e-5 * max(1.0, float(sc_r))
    assert abs(float(mag) - float(mag_r)) < 1e-5 * max(1.0, float(mag_r))
    assert rel_l2(xg.grad.cpu(), xr.grad) < 1e-4
    # deterministic: the same call again gives the same bits
    sc2, mag2 = loss(xg.detach(), y.float().cuda())
    assert torch.equal(sc2, sc.detach()) and torch.equal(mag2, mag.detach())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bucket_embed_vs_torch(dt):
    """Training-side energy embedding (vo_bucket_embed / vo_embed_bwd, modules.py:53-64,101-104):
    bucket indices exact (targets on and next to every bin edge), out = x + table[idx], dx = dy, and
    the table gradient against nn.Embedding's autograd."""
    from visual_onoma_to_wave_amd import autograd as AG
    g = torch.Generator().manual_seed(3)
    B, T, D = 32, 12, 256
    bins = torch.linspace(-1.06798, 5.10888, 255)
    tgt = torch.randn(B, T, generator=g) * 2 + 1
    tgt[0, :6] = bins[torch.tensor([0, 1, 100, 200, 253, 254])]          # exactly on edges (right=False)
    tgt[1, :5] = torch.tensor([-5.0, 9.0, float(bins[7]) - 1e-6, float(bins[7]) + 1e-6, float("nan")])
    emb = torch.nn.Embedding(256, D)
    x = torch.randn(B, T, D, generator=g)
    xg = x.to(dt).cuda().requires_grad_(True)
    e_h = torch.nn.Embedding(256, D).cuda()
    e_h.weight.data.copy_(emb.weight.data)
    out = AG.bucket_embed(xg, e_h, tgt.cuda(), bins.cuda())
    idx_ref = torch.bucketize(tgt, bins)
    xr = x.to(dt).float().requires_grad_(True)
    ref = xr + emb(idx_ref)
    if dt == torch.float32:
        assert torch.equal(out.detach().cpu(), ref.detach())
    else:
        assert torch.equal(out.detach().cpu(), ref.detach().to(dt))
    dy = torch.randn(B, T, D, generator=g)
    out.backward(dy.to(dt).cuda())
    ref.backward(dy.to(dt).float())
    assert torch.equal(xg.grad.cpu(), dy.to(dt))
    err = float((e_h.weight.grad.cpu() - emb.weight.grad).norm() / emb.weight.grad.norm())
    assert err < 1e-6, err
    assert int(idx_ref[1, 4]) == 255  # NaN -> len(bins), as torch.bucketize
    # a table with fewer than len(bins) + 1 rows is refused before any launch
    from visual_onoma_to_wave_amd import ops
    with pytest.raises(Exception, match="table has 200 rows"):
        ops.bucket_embed(x.cuda().contiguous(), tgt.cuda(), bins.cuda(), torch.zeros(200, D, device="cuda"))


@pytest.mark.parametrize("dtype,shape", [(torch.bfloat16, (32, 512, 256)), (torch.float32, (32, 12, 256)),
                                         (torch.float32, (3, 7, 5)), (torch.bfloat16, (2, 3, 3))])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_dropout_counter_mask(dtype, shape, p):
    """autograd.dropout (vo_dropout): kept elements are x / (1 - p) exactly as F.dropout scales them, the
    keep rate is 1 - p, the backward applies the forward's mask (no mask tensor), a new call draws a new
    mask, and n % 8 tails are covered."""
    from visual_onoma_to_wave_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    x = (torch.rand(shape, device="cuda", generator=g) + 0.5).to(dtype).requires_grad_(True)
    y = AG.dropout(x, p)
    keep = y.detach() != 0
    scaled = (x.detach().float() * (1.0 / (1.0 - p))).to(dtype)
    assert torch.equal(y.detach()[keep], scaled[keep])
    n = x.numel()
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 5 * (p * (1 - p) / n) ** 0.5 + 1e-9, rate
    gy = torch.rand(shape, device="cuda", generator=g).to(dtype) + 1.0
    y.backward(gy)
    gk = x.grad != 0
    assert torch.equal(gk, keep)
    assert torch.equal(x.grad[keep], (gy.float() * (1.0 / (1.0 - p))).to(dtype)[keep])
    if n > 1000:
        y2 = AG.dropout(x.detach(), p)
        assert not torch.equal(y2 != 0, keep)


def test_dropout_graph_replays_draw_new_masks():
    """Captured in a HIP graph, every replay draws a new step seed (torch's graph-safe generator)."""
    from visual_onoma_to_wave_amd import autograd as AG
    x = torch.ones(64, 1024, device="cuda", dtype=torch.bfloat16)
    AG.begin_dropout_step(x.device)
    AG.dropout(x, 0.5)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        AG.begin_dropout_step(x.device)  # the step's seed, drawn inside the graph
        y = AG.dropout(x, 0.5)
    masks = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        masks.append(y != 0)
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


@pytest.mark.parametrize("xdt,rdt,dual", [(torch.bfloat16, torch.float32, True), (torch.float32, torch.float32, False),
                                          (torch.bfloat16, torch.bfloat16, False)])
@pytest.mark.parametrize("B,T,D,p,use", [(32, 512, 256, 0.2, "both"), (3, 37, 256, 0.5, "both"), (32, 12, 256, 0.2, "y"),
                                         (2, 5, 512, 0.1, "copy")])
def test_layernorm_dropout_fused(B, T, D, p, use, xdt, rdt, dual):
    """autograd.layernorm_drop (the training FFT block's sublayer dropout inside its LayerNorm kernels) vs the fp32
    autograd of LayerNorm(mask * x / (1 - p) + res) + pad-row zeroing, the mask taken from vo_dropout with the SAME
    (seed, salt) on a tensor of ones: the forward, the x gradient's zero pattern -- exactly the dropout mask (a
    round-5 fusion attempt got it wrong and was dropped) -- and values, the residual / gamma / beta gradients.
    use: which outputs feed the loss ("copy": only the bf16 copy, as the last decoder layer)."""
    import torch.nn.functional as F
    from visual_onoma_to_wave_amd import autograd as AG
    from visual_onoma_to_wave_amd import ops
    if use == "copy" and not dual:
        pytest.skip("the copy exists in the dual form only")
    g = torch.Generator(device="cuda").manual_seed(B * T + D)
    x = torch.randn(B, T, D, device="cuda", generator=g).to(xdt)
    res = torch.randn(B, T, D, device="cuda", generator=g).to(rdt)
    gam = (1.0 + 0.1 * torch.randn(D, device="cuda", generator=g))
    bet = 0.1 * torch.randn(D, device="cuda", generator=g)
    lens = torch.randint(1, T + 1, (B,), device="cuda", generator=g).int()
    AG.begin_dropout_step(x.device)
    seed = AG._DROP["seed"]
    salt = AG._DROP["site"] + 1  # the salt layernorm_drop takes next
    mask = ops.dropout(torch.ones(B, T, D, device="cuda"), p, seed, salt) != 0  # vo_dropout's draw
    xi, ri = x.float().requires_grad_(True), res.float().requires_grad_(True)
    gi, bi = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    yref = F.layer_norm(xi * mask * (1.0 / (1.0 - p)) + ri, (D,), gi, bi, 1e-5)
    yref = yref.masked_fill((torch.arange(T, device="cuda")[None, :] >= lens.long()[:, None])[..., None], 0.0)
    gy = torch.randn(B, T, D, device="cuda", generator=g)
    gy16 = torch.randn(B, T, D, device="cuda", generator=g).to(torch.bfloat16)
    gtot = (gy if use != "copy" else 0.0) + (gy16.float() if (dual and use != "y") else 0.0)
    rx, rr, rg, rb = torch.autograd.grad(yref, (xi, ri, gi, bi), gtot)
    xc, rc = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
    gc, bc = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    out = AG.layernorm_drop(xc, rc, gc, bc, lens, p, dual)
    y, y16 = out if dual else (out, None)
    assert AG._DROP["site"] == salt
    tol = 1e-5 if xdt == torch.float32 and rdt == torch.float32 else 1e-2
    assert y.dtype == rdt and rel_l2(y.detach().float().cpu(), yref.detach().cpu()) < (1e-5 if rdt == torch.float32 else 1e-2)
    if dual:
        assert torch.equal(y16.detach(), y.detach().to(torch.bfloat16))
    outs, grads = [], []
    if use != "copy":
        outs.append(y), grads.append(gy.to(y.dtype))
    if dual and use != "y":
        outs.append(y16), grads.append(gy16)
    dx, dr, dg, db = torch.autograd.grad(outs, (xc, rc, gc, bc), grads)
    live = (torch.arange(T, device="cuda")[None, :] < lens.long()[:, None])[..., None].expand(B, T, D)
    # the x gradient is zero exactly where the mask dropped (or the row is padding): the same mask both ways
    assert torch.equal((dx != 0) | ~live, mask | ~live)
    assert dx.dtype == xdt and dr.dtype == rdt
    assert rel_l2(dx.float().cpu(), rx.cpu()) < tol and rel_l2(dr.float().cpu(), rr.cpu()) < tol
    assert rel_l2(dg.cpu(), rg.cpu()) < max(tol, 1e-5) and rel_l2(db.cpu(), rb.cpu()) < max(tol, 1e-5)
