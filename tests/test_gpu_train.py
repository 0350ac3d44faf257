"""Training path (C4) on the GPU: teacher-forced forward in train mode (BatchNorm batch
statistics; dropout probabilities set to 0 so both sides are deterministic), FastSpeech2Loss,
backward -- loss terms and parameter gradients against the oracle's autograd on the CPU.

Tolerances: fp32 mode (exact-f32 MFMA forward and HIP dgrad) rel-L2 <= 1e-4 on losses and
<= 2e-3 on gradients (long backward chains through LayerNorm / softmax in a different
summation order); mixed mode loss within 2e-2."""

import numpy as np
import pytest
import torch

from helpers import configs, golden, rel_l2, stats, vtts_arrays
from weights import load_into

pytestmark = pytest.mark.gpu


def _no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0


def _batch(g, dev):
    t = lambda k: torch.from_numpy(np.array(g[k])).to(dev)  # noqa: E731
    return (None, t("in_audiotypes"), t("in_texts"), t("in_src_lens"), int(g["in_max_src_len"]), t("in_mels"),
            t("in_mel_lens"), int(g["in_max_mel_len"]), t("in_e_targets"), None, t("in_d_targets"),
            t("in_images"), None)


def _oracle_grads(arrays, batch_cpu):
    from oracle import acoustic as A
    from oracle import training as TR
    sd = A.complete_state_dict(arrays, stats()["energy"])
    for k, v in sd.items():
        if v.dtype == torch.float32 and "position_enc" not in k and "bins" not in k and "running" not in k:
            v.requires_grad_(True)
    out = A.vtts_forward(sd, *batch_cpu[1:12], energy_stats=stats()["energy"], training=True)
    losses = TR.fastspeech2_loss(batch_cpu, out)
    losses[0].backward()
    return [float(x) for x in losses], {k: v.grad for k, v in sd.items() if v.grad is not None}


@pytest.mark.parametrize("mode", ["fp32", "mixed"])
def test_train_step_grads_vs_oracle(device, mode):
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    arrays = vtts_arrays()
    g = golden("vtts_tf")
    m = vTTS(*configs())
    load_into(m, arrays)
    m = m.to(device).train().set_precision(mode)
    _no_dropout(m)
    batch = _batch(g, device)
    out = m(*(batch[1:]), True)
    losses = FastSpeech2Loss()(batch, out)
    losses[0].backward()
    ref_losses, ref_grads = _oracle_grads(arrays, _batch(g, "cpu"))
    got = [float(x) for x in losses]
    tol = 1e-4 if mode == "fp32" else 2e-2
    np.testing.assert_allclose(got, ref_losses, rtol=tol, atol=1e-6)
    if mode != "fp32":
        return
    named = dict(m.named_parameters())
    checked, bad = 0, []
    for k, gr in ref_grads.items():
        p = named.get(k)
        if p is None or p.grad is None:
            continue
        # conv biases feeding a train-mode BatchNorm have an exactly-zero true gradient
        # (both sides are rounding noise ~1e-8): an absolute floor covers them
        err = float((p.grad.cpu() - gr).norm())
        if err > 2e-3 * float(gr.norm()) + 1e-5:
            bad.append((k, err, float(gr.norm())))
        checked += 1
    assert not bad, bad[:10]
    assert checked > 150


def test_training_reduces_loss(device):
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import train_step
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(device).train()
    opt = ScheduledOptim(m, tc, mc, 0)
    batch = _batch(golden("vtts_tf"), device)
    first = None
    for _ in range(12):
        losses = train_step(m, opt, FastSpeech2Loss(), batch)
        first = first if first is not None else float(losses[0])
    assert float(losses[0]) < 0.8 * first


def test_step_batched_packs_bit_identical(device):
    """autograd's step-batched weight packs (every conv's forward and input-gradient layouts of a step in
    one vo_pack_batch call per dtype, the fused q/k/v weights written by three jobs) against per-call
    packs (VO_C4_PREPACK=0 behaviour): four mixed-precision training steps with the optimizer moving the
    weights, losses and every parameter bit for bit; at most two pack calls (fp32 encoder, bf16
    decoder) per step, also in the first step after reset_packs() (the stores seeded from the layouts
    earlier steps used, as inside a graph capture)."""
    from visual_onoma_to_wave_amd import autograd as AG
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import train_step
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)
    batch = _batch(golden("vtts_tf"), device)
    runs = []
    saved = AG.PREPACK
    try:
        for prepack in (False, True):
            AG.PREPACK = prepack
            AG.reset_packs()
            m = vTTS(pc, mc, tc)
            load_into(m, vtts_arrays())
            m = m.to(device).train().set_precision("mixed")
            _no_dropout(m)
            opt = ScheduledOptim(m, tc, mc, 0)
            losses = []
            for i in range(4):
                if i == 3:  # a store emptied (as around a graph capture) is re-seeded: still one batch per dtype
                    AG.reset_packs()
                b0 = AG.STATS["batches"]
                losses.append([float(x) for x in train_step(m, opt, FastSpeech2Loss(), batch)])
                if prepack and i > 0:
                    assert AG.STATS["batches"] - b0 <= 2
            runs.append((losses, [p.detach().clone() for p in m.parameters()]))
    finally:
        AG.PREPACK = saved
        AG.reset_packs()
    (l0, p0), (l1, p1) = runs
    assert l0 == l1
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


def test_graphed_train_step_matches_eager(device):
    """train.GraphedTrainStep (HIP-graph replay with the capturable Adam and a device-tensor
    learning rate, replays launched back to back with no host wait) against the same number of
    eager train_step calls (fp32, dropout off, the same capturable Adam).  The warm-up steps
    before the capture are undone, so 12 calls are 12 updates.  Every backward kernel is
    deterministic (row-split partials added in a fixed order, no atomics), so two eager runs are
    bit-identical and the replayed run must be too: a stale input, learning rate or packed
    weight, an extra warm-up update or a read outside stream order would show as any difference."""
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import GraphedTrainStep, train_step
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)  # steps that move the weights
    batch = _batch(golden("vtts_tf"), device)
    finals = []
    for graphed in (False, False, True):
        m = vTTS(pc, mc, tc)
        load_into(m, vtts_arrays())
        m = m.to(device).train().set_precision("fp32")
        _no_dropout(m)
        opt = ScheduledOptim(m, tc, mc, 0, capturable=True)
        per_step = []
        if graphed:
            run = GraphedTrainStep(m, opt, FastSpeech2Loss(), warmup=3)
            for _ in range(12):
                losses = run(batch)
                per_step.append(losses[0].detach().clone())  # stream-ordered read, no host wait
        else:
            for _ in range(12):
                losses = train_step(m, opt, FastSpeech2Loss(), batch)
                per_step.append(losses[0].detach().clone())
        torch.cuda.synchronize()
        assert opt.current_step == 12
        finals.append((np.array([float(x) for x in per_step]),
                       torch.cat([p.detach().flatten().cpu() for p in m.parameters()])))
    (l0, p0), (l1, p1), (lg, pg) = finals
    assert np.isfinite(lg).all() and l0[-1] < 0.6 * l0[0]  # the twelve updates really train
    print(f"graphed vs eager: params {float((pg - p0).norm() / p0.norm()):.2e}, per-step losses "
          f"{float(np.abs(lg - l0).max()):.2e}; eager vs eager {float((p1 - p0).norm() / p0.norm()):.2e}")
    assert torch.equal(p1, p0) and np.array_equal(l1, l0), "eager training is not deterministic"
    assert torch.equal(pg, p0) and np.array_equal(lg, l0), "graph replay differs from the eager steps"


def test_inference_after_graphed_training_uses_new_weights(device):
    """Replays update parameters without bumping their version counters: the inference pack
    cache must not serve weights packed before the graphed steps."""
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import GraphedTrainStep
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)
    g = golden("vtts_tf")
    batch = _batch(g, device)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(device).set_precision("fp32")
    _no_dropout(m)
    args = tuple(batch[1:]) + (True,)

    def infer(model):
        model.eval()
        with torch.no_grad():
            out = model(*args)[1].clone()
        model.train()
        return out
    before = infer(m)
    run = GraphedTrainStep(m, ScheduledOptim(m, tc, mc, 0, capturable=True), FastSpeech2Loss(), warmup=1)
    for _ in range(3):
        run(batch)
    after = infer(m)
    fresh = vTTS(pc, mc, tc).to(device).set_precision("fp32")
    fresh.load_state_dict(m.state_dict())
    ref = infer(fresh)
    torch.cuda.synchronize()
    assert rel_l2(after.cpu(), ref.cpu()) < 1e-6
    assert rel_l2(after.cpu(), before.cpu()) > 1e-4


@pytest.mark.parametrize("dt,D,with_res,with_lens", [
    (torch.float32, 256, True, True), (torch.float32, 256, False, False), (torch.bfloat16, 256, True, True),
    (torch.float32, 512, True, False), (torch.bfloat16, 512, False, True)])
@pytest.mark.parametrize("B,T", [(3, 37), (32, 512), (1, 1)])
def test_layernorm_bwd_vs_torch(B, T, D, dt, with_res, with_lens):
    """vo_layernorm_bwd vs the fp32 autograd of LayerNorm(x + res) + pad-row masked_fill."""
    import torch.nn.functional as F
    from visual_onoma_to_wave_amd import ops
    gen = torch.Generator().manual_seed(B * T + D)
    x = torch.randn(B, T, D, generator=gen).to(dt)
    res = torch.randn(B, T, D, generator=gen).to(dt) if with_res else None
    gy = torch.randn(B, T, D, generator=gen).to(dt)
    g = 1.0 + 0.1 * torch.randn(D, generator=gen)
    bta = 0.1 * torch.randn(D, generator=gen)
    lens = torch.randint(1, T + 1, (B,), generator=gen).int() if with_lens else None
    xi = x.float().requires_grad_(True)
    gi, bi = g.clone().requires_grad_(True), bta.clone().requires_grad_(True)
    h = xi + res.float() if with_res else xi
    y = F.layer_norm(h, (D,), gi, bi, 1e-5)
    if with_lens:
        y = y.masked_fill((torch.arange(T)[None, :] >= lens.long()[:, None])[..., None], 0.0)
    rx, rg, rb = torch.autograd.grad(y, (xi, gi, bi), gy.float())
    gh, dg, db = ops.layernorm_bwd(x.cuda(), gy.cuda(), g.cuda(), res=res.cuda() if with_res else None,
                                   lens=lens.cuda() if with_lens else None)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert gh.dtype == dt and rel_l2(gh.float().cpu(), rx) < tol
    assert rel_l2(dg.cpu(), rg) < 1e-5 and rel_l2(db.cpu(), rb) < 1e-5


@pytest.mark.parametrize("B,T,D,with_lens", [(3, 37, 256, True), (32, 512, 256, True), (2, 5, 512, False)])
@pytest.mark.parametrize("use", ["both", "copy"])
def test_layernorm_dual_train_vs_torch(B, T, D, with_lens, use):
    """autograd.layernorm_dual (the mixed training decoder's LayerNorm: bf16 sublayer output x, fp32
    residual stream res -> fp32 y and its bf16 copy y16) vs the fp32 autograd of LayerNorm(x + res) +
    pad-row masked_fill; the two incoming gradients (y's and y16's) summed in the backward kernel.
    use = "copy": only y16 is read downstream (the last decoder layer)."""
    import torch.nn.functional as F
    from visual_onoma_to_wave_amd import autograd as AG
    gen = torch.Generator().manual_seed(B * T + D)
    x = torch.randn(B, T, D, generator=gen).to(torch.bfloat16)
    res = torch.randn(B, T, D, generator=gen)
    g = 1.0 + 0.1 * torch.randn(D, generator=gen)
    bta = 0.1 * torch.randn(D, generator=gen)
    lens = torch.randint(1, T + 1, (B,), generator=gen).int() if with_lens else None
    gy = torch.randn(B, T, D, generator=gen)
    gy16 = torch.randn(B, T, D, generator=gen).to(torch.bfloat16)
    xi, ri = x.float().requires_grad_(True), res.clone().requires_grad_(True)
    gi, bi = g.clone().requires_grad_(True), bta.clone().requires_grad_(True)
    y = F.layer_norm(xi + ri, (D,), gi, bi, 1e-5)
    if with_lens:
        y = y.masked_fill((torch.arange(T)[None, :] >= lens.long()[:, None])[..., None], 0.0)
    gtot = gy16.float() + (gy if use == "both" else 0.0)
    rx, rr, rg, rb = torch.autograd.grad(y, (xi, ri, gi, bi), gtot)
    xc, rc = x.cuda().requires_grad_(True), res.cuda().requires_grad_(True)
    gc, bc = g.cuda().requires_grad_(True), bta.cuda().requires_grad_(True)
    y32, y16 = AG.layernorm_dual(xc, rc, gc, bc, lens.cuda() if with_lens else None)
    assert y32.dtype == torch.float32 and y16.dtype == torch.bfloat16
    assert rel_l2(y32.detach().cpu(), y.detach()) < 1e-6
    assert torch.equal(y16.detach(), y32.detach().to(torch.bfloat16))
    outs, grads = ((y32, y16), (gy.cuda(), gy16.cuda())) if use == "both" else ((y16,), (gy16.cuda(),))
    dx, dr, dg, db = torch.autograd.grad(outs, (xc, rc, gc, bc), grads)
    assert dx.dtype == torch.bfloat16 and dr.dtype == torch.float32
    assert rel_l2(dr.cpu(), rr) < 1e-5 and rel_l2(dx.float().cpu(), rx) < 1e-2
    assert rel_l2(dg.cpu(), rg) < 1e-5 and rel_l2(db.cpu(), rb) < 1e-5


def _torch_attention(qkv, lens, n_head):
    """fp32 reference of vo_attention: head split of SubLayers.py:39-46, SDPA of Modules.py:14-25
    with the key-padding mask of Models.py:104 / 187."""
    B, L, D3 = qkv.shape
    D = D3 // 3
    dk = D // n_head
    q, k, v = (t.reshape(B, L, n_head, dk).transpose(1, 2) for t in qkv.split(D, dim=-1))
    s = q @ k.transpose(-1, -2) / dk ** 0.5
    mask = torch.arange(L)[None, None, None, :] >= lens.long()[:, None, None, None]
    p = torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)
    return (p @ v).transpose(1, 2).reshape(B, L, D)


@pytest.mark.parametrize("with_lse", [False, True])
@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,L,H,ragged", [(2, 12, 2, True), (4, 512, 2, True), (3, 100, 2, False),
                                          (2, 1, 2, False), (1, 1000, 2, True), (2, 130, 1, True)])
def test_attention_bwd_vs_torch(B, L, H, ragged, dt, tol, with_lse):
    """vo_attention_bwd (dQ | dK | dV) vs the fp32 autograd of the reference SDPA, ragged key
    padding, L not a multiple of the 64-row tiles; with_lse: the forward's row log-sum-exp handed to
    vo_attention_bwd_lse (bf16: the version-2 kernels)."""
    from visual_onoma_to_wave_amd import ops
    gen = torch.Generator().manual_seed(B * L + H)
    D = 128 * H
    qkv = torch.randn(B, L, 3 * D, generator=gen).to(dt)
    lens = torch.randint(1, L + 1, (B,), generator=gen).int() if ragged else torch.full((B,), L, dtype=torch.int32)
    gout = torch.randn(B, L, D, generator=gen).to(dt)
    qi = qkv.float().requires_grad_(True)
    ref_out = _torch_attention(qi, lens, H)
    (ref,) = torch.autograd.grad(ref_out, qi, gout.float())
    qc, lc = qkv.cuda(), lens.cuda()
    if with_lse:
        out, lse = ops.attention(qc, lc, H, with_lse=True)
        assert torch.equal(out, ops.attention(qc, lc, H))  # the lse output changes nothing else
        got = ops.attention_bwd(qc, out, gout.cuda(), lc, H, lse=lse)
        # the row log-sum-exp itself vs the reference softmax's
        dk = 128
        qf = qkv.float().reshape(B, L, 3, H, dk)
        sc = torch.einsum("bqhd,bkhd->bhqk", qf[:, :, 0], qf[:, :, 1]) / dk ** 0.5
        sc = sc.masked_fill(torch.arange(L)[None, None, None, :] >= lens.long()[:, None, None, None], float("-inf"))
        ref_lse = torch.logsumexp(sc, dim=-1)
        assert torch.allclose(lse.cpu(), ref_lse, rtol=1e-4, atol=1e-3 if dt == torch.bfloat16 else 1e-4)
    else:
        out = ops.attention(qc, lc, H)
        got = ops.attention_bwd(qc, out, gout.cuda(), lc, H)
    assert got.dtype == dt and got.shape == qkv.shape
    got = got.float().cpu()
    for part in range(3):  # dQ, dK, dV separately (padded keys: exactly zero)
        sl = slice(part * D, (part + 1) * D)
        # L = 1: softmax over one key is constant, so the reference dQ / dK are exactly 0 and
        # ours carry the rounding of P (dP - rowsum(dO o O)); the floor scales with |dO|
        err = float((got[..., sl] - ref[..., sl]).norm())
        den = max(float(ref[..., sl].norm()), 1e-2 * float(gout.float().norm()))
        assert err < tol * den, (part, err / den)
    for bi in range(B):
        assert torch.count_nonzero(got[bi, int(lens[bi]):, D:]) == 0


@pytest.mark.parametrize("go_dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("max_len_delta", [0, 7, -5])
def test_length_regulate_bwd_vs_torch(go_dt, max_len_delta):
    """vo_length_regulate_bwd vs the autograd of the reference expand + pad / crop
    (modules.py:132-159, tools.py:669-687): fractional (truncated), zero and negative
    durations, padded and cropped outputs."""
    from visual_onoma_to_wave_amd import ops
    gen = torch.Generator().manual_seed(7 + max_len_delta)
    B, T, D = 3, 13, 256
    dur = torch.rand(B, T, generator=gen) * 9.0 - 1.0  # [-1, 8): negatives and fractions
    dur[0, 3] = 0.0
    reps = torch.clamp(torch.trunc(dur), min=0).long()
    max_len = int(reps.sum(1).max()) + max_len_delta
    x = torch.randn(B, T, D, generator=gen).requires_grad_(True)
    outs = []
    for b in range(B):
        e = torch.cat([x[b, j:j + 1].expand(int(reps[b, j]), D) for j in range(T)], 0)
        e = e[:max_len] if e.shape[0] > max_len else torch.nn.functional.pad(e, (0, 0, 0, max_len - e.shape[0]))
        outs.append(e)
    ref_out = torch.stack(outs)
    go = torch.randn(B, max_len, D, generator=gen).to(go_dt)
    (ref,) = torch.autograd.grad(ref_out, x, go.float())
    got = ops.length_regulate_bwd(go.cuda(), dur.cuda(), T, out_dtype=torch.float32).cpu()
    assert rel_l2(got, ref) < 1e-6
