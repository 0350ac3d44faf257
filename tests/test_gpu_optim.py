"""The multi-tensor HIP Adam / AdamW (visual_onoma_to_wave_amd.optim.FusedAdam, vo_adam_multi) against
torch.optim.Adam / AdamW (the reference's optimizer, scripts/model/optimizer.py:9-15, and the HiFi-GAN V1
recipe's AdamW) over several steps: parameters within rel-L2 1e-6, moments within 1e-5 (fp32, the same
update order; fused multiply-adds and powf vs Python-double bias corrections differ in the last bits).  Also: unaligned gradient views
(bucket slices), more tensors than one launch holds, a state_dict round trip with torch's Adam, and a
HIP-graph replay equal to eager steps bit for bit."""

import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu

SHAPES = [(1,), (3,), (5, 7), (256, 256), (513,), (1024, 64, 3), (2, 3, 5, 7), (4097,)]


def _params(seed, n):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(SHAPES[i % len(SHAPES)], generator=g) for i in range(n)]


def _grads(seed, ps, steps):
    g = torch.Generator().manual_seed(seed)
    return [[torch.randn(p.shape, generator=g) * (0.1 + i) for i, p in enumerate(ps)] for _ in range(steps)]


@pytest.mark.parametrize("decoupled,wd,n", [(False, 0.0, 8), (False, 0.01, 70), (True, 0.01, 9), (True, 0.0, 130)])
def test_fused_adam_vs_torch(decoupled, wd, n):
    from visual_onoma_to_wave_amd.optim import FusedAdam
    init = _params(n, n)
    grads = _grads(n + 1, init, 5)
    kw = dict(lr=2e-3, betas=(0.8, 0.99), eps=1e-8, weight_decay=wd)
    pr = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    pf = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    ref = (torch.optim.AdamW if decoupled else torch.optim.Adam)(pr, foreach=False, **kw)
    got = FusedAdam(pf, decoupled=decoupled, **kw)
    # gradients as views into one flat buffer at a 1-float offset (GradBucketer slices are not aligned)
    flat = torch.empty(1 + sum(p.numel() for p in init), device="cuda")
    for gs in grads:
        off = 1
        for a, b, g in zip(pr, pf, gs):
            a.grad = g.cuda()
            v = flat[off: off + g.numel()].view_as(g)
            v.copy_(g.cuda())
            b.grad = v
            off += g.numel()
        ref.step()
        got.step()
    for a, b in zip(pr, pf):
        assert rel_l2(b.detach().cpu(), a.detach().cpu()) < 1e-6
        sa, sb = ref.state[a], got.state[b]
        assert rel_l2(sb["exp_avg"].cpu(), sa["exp_avg"].cpu()) < 1e-5
        assert rel_l2(sb["exp_avg_sq"].cpu(), sa["exp_avg_sq"].cpu()) < 1e-5
        assert float(sb["step"]) == float(sa["step"]) == 5.0


def test_fused_adam_state_dict_interchange():
    """A torch Adam state (the reference checkpoint's "optimizer" entry) loads into FusedAdam and the
    next steps continue as torch's would; FusedAdam's state_dict loads back into torch Adam."""
    from visual_onoma_to_wave_amd.optim import FusedAdam
    init = _params(3, 6)
    grads = _grads(4, init, 6)
    kw = dict(lr=1e-3, betas=(0.9, 0.98), eps=1e-9, weight_decay=0.0)
    pr = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    ref = torch.optim.Adam(pr, foreach=False, **kw)
    for gs in grads[:3]:
        for a, g in zip(pr, gs):
            a.grad = g.cuda()
        ref.step()
    pf = [torch.nn.Parameter(a.detach().clone()) for a in pr]
    got = FusedAdam(pf, **kw)
    got.load_state_dict(ref.state_dict())
    for gs in grads[3:]:
        for a, b, g in zip(pr, pf, gs):
            a.grad = g.cuda()
            b.grad = g.cuda()
        ref.step()
        got.step()
    for a, b in zip(pr, pf):
        assert rel_l2(b.detach().cpu(), a.detach().cpu()) < 1e-5  # eps 1e-9: tiny denominators
    back = torch.optim.Adam([torch.nn.Parameter(b.detach().clone()) for b in pf], **kw)
    back.load_state_dict(got.state_dict())
    assert float(back.state_dict()["state"][0]["step"]) == 6.0
    assert set(got.state_dict()["param_groups"][0]) == set(ref.state_dict()["param_groups"][0])


def test_fused_adam_graph_replay_matches_eager():
    from visual_onoma_to_wave_amd.optim import FusedAdam
    init = _params(9, 12)
    grads = _grads(10, init, 4)
    outs = []
    for graphed in (False, True):
        ps = [torch.nn.Parameter(p.clone().cuda()) for p in init]
        lr = torch.tensor(1e-3, device="cuda")
        opt = FusedAdam(ps, lr=lr, betas=(0.8, 0.99), weight_decay=0.01, decoupled=True, capturable=True)
        static = [g.cuda() for g in grads[0]]
        for p, g in zip(ps, static):
            p.grad = g
        if graphed:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                opt.step()  # warm-up: creates the state
            torch.cuda.current_stream().wait_stream(s)
            with torch.no_grad():
                for p, q in zip(ps, init):
                    p.copy_(q.cuda())
                for st in opt.state.values():
                    for k in ("exp_avg", "exp_avg_sq", "step"):
                        st[k].zero_()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                opt.step()
        for i, gs in enumerate(grads):
            for s_, g in zip(static, gs):
                s_.copy_(g.cuda())
            lr.fill_(1e-3 * (i + 1))
            graph.replay() if graphed else opt.step()
        torch.cuda.synchronize()
        outs.append(torch.cat([p.detach().flatten().cpu() for p in ps]))
    assert torch.equal(outs[0], outs[1])


def test_fused_adam_bumps_parameter_versions():
    """The HIP update writes the parameters outside autograd; it bumps their version counters as
    torch's in-place updates do, so caches keyed on them (packed bf16 weights) see every step."""
    from visual_onoma_to_wave_amd.optim import FusedAdam
    ps = [torch.nn.Parameter(p.cuda()) for p in _params(5, 3)]
    opt = FusedAdam(ps, lr=1e-3)
    before = [p._version for p in ps]
    for p, g in zip(ps, _grads(6, ps, 1)[0]):
        p.grad = g.cuda()
    opt.step()
    assert all(p._version > v for p, v in zip(ps, before))


def test_gan_trainer_fused_adamw_matches_torch_adamw(monkeypatch):
    """Two eager HiFi-GAN V1 steps (fp32 compute) with the fused AdamW against the same steps with
    torch.optim.AdamW: the generator's packed weights must follow every update (a stale pack would
    leave the second step's forward on the first step's weights)."""
    from helpers import hifigan_arrays, hifigan_h
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan, optim
    mel_g = torch.Generator().manual_seed(2)
    mel = (torch.randn(2, 32, 80, generator=mel_g) - 4.0).cuda()
    y = (0.3 * torch.randn(2, 8192, generator=mel_g)).clamp(-1, 1).cuda()
    finals = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(optim, "AdamW", lambda params, *a, **kw: torch.optim.AdamW(params, *a, **kw))
        torch.manual_seed(1234)
        g = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
        load_into(g, hifigan_arrays())
        tr = hifigan.HifiGanTrainer(g.cuda(), hifigan.AttrDict(hifigan_h()), capturable=True)
        tr.set_compute_dtype(torch.float32)
        for _ in range(2):
            losses = tr.step(mel, y)
        torch.cuda.synchronize()
        finals.append(({k: float(v) for k, v in losses.items()},
                       torch.cat([p.detach().flatten().cpu() for p in g.parameters()])))
    (lf, gf), (lt, gt) = finals
    assert rel_l2(gf, gt) < 1e-4
    for k in lt:
        assert abs(lf[k] - lt[k]) <= 1e-3 * abs(lt[k]) + 1e-5, (k, lf[k], lt[k])


def test_capturable_lr_survives_load_state_dict():
    """A capturable FusedAdam (device-tensor lr, the graphed C4 / C5 steps) keeps its lr tensor through
    load_state_dict (the loaded value is copied into it), so a step captured after a resume still
    follows the schedule: replays at lr = 0 leave the parameters unchanged, replays at a new lr move
    them exactly as eager steps at that lr do.  A float-lr group refuses to be captured."""
    from visual_onoma_to_wave_amd.optim import FusedAdam
    init = _params(5, 4)
    grads = [g.cuda() for g in _grads(6, init, 1)[0]]
    src = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    ref_opt = torch.optim.Adam(src, lr=3e-3)
    for p, g in zip(src, grads):
        p.grad = g.clone()
    ref_opt.step()
    sd = ref_opt.state_dict()

    ps = [torch.nn.Parameter(p.detach().clone()) for p in src]
    lr_t = torch.tensor(1e-3, device="cuda")
    opt = FusedAdam(ps, lr=lr_t, capturable=True)
    opt.load_state_dict(sd)
    assert opt.param_groups[0]["lr"] is lr_t and float(lr_t) == pytest.approx(3e-3)
    for p, g in zip(ps, grads):
        p.grad = g.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        opt.step()  # warm-up (allocates nothing new; state exists)
    torch.cuda.current_stream().wait_stream(s)
    eager = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    ref2 = FusedAdam(eager, lr=torch.tensor(0.0, device="cuda"), capturable=True)
    ref2.load_state_dict(opt.state_dict())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt.step()
    lr_t.fill_(0.0)
    before = [p.detach().clone() for p in ps]
    graph.replay()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b.detach()) for a, b in zip(before, ps))  # lr 0: no movement
    lr_t.fill_(5e-3)
    graph.replay()
    ref2.param_groups[0]["lr"].fill_(0.0)
    for p, g in zip(eager, grads):
        p.grad = g.clone()
    ref2.step()  # the lr-0 step (advances the step count as the replay did)
    ref2.param_groups[0]["lr"].fill_(5e-3)
    ref2.step()
    torch.cuda.synchronize()
    for a, b in zip(ps, eager):
        assert rel_l2(a.detach().cpu(), b.detach().cpu()) < 1e-6
    moved = max(float((a.detach() - b).abs().max()) for a, b in zip(ps, before))
    assert moved > 1e-4  # the new lr took effect

    # a float learning rate cannot be captured (it would be frozen into the graph)
    fl = FusedAdam([torch.nn.Parameter(init[0].clone().cuda())], lr=1e-3, capturable=True)
    fl.param_groups[0]["params"][0].grad = torch.ones_like(fl.param_groups[0]["params"][0])
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="device-tensor learning rates"):
        with torch.cuda.graph(g2):
            fl.step()


@pytest.mark.parametrize("missing", [False, True])
def test_step_captured_before_load_state_dict_follows_it(missing):
    """A step captured BEFORE load_state_dict: the load copies the step count and the moments into the
    device tensors the graph reads and writes (as it does the learning rate), so the replay continues
    from the loaded state exactly as an eager optimizer that loaded the same state.  missing: the
    loaded state has no moments for one parameter (it never had a gradient there) -- the moments the
    graph reads are zeroed and stay in the state, as the eager optimizer starts that one from zeros."""
    from visual_onoma_to_wave_amd.optim import FusedAdam
    init = _params(5, 4)
    grads = [[g.cuda() for g in gs] for gs in _grads(7, init, 3)]
    ps = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    opt = FusedAdam(ps, lr=torch.tensor(2e-3, device="cuda"), capturable=True)
    for p, g in zip(ps, grads[0]):
        p.grad = g.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        opt.step()  # warm-up: creates the state the graph will use
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt.step()
    # a different optimizer history (three steps of other gradients) to resume from
    src = [torch.nn.Parameter(p.clone().cuda()) for p in init]
    other = torch.optim.Adam(src, lr=2e-3)
    for gs in grads:
        for i, (p, g) in enumerate(zip(src, gs)):
            p.grad = None if (missing and i == 2) else g.clone() * 0.5
        other.step()
    sd = other.state_dict()
    assert (2 in sd["state"]) != missing
    opt.load_state_dict(sd)
    with torch.no_grad():
        for p, q in zip(ps, src):
            p.copy_(q)
    eager = [torch.nn.Parameter(q.detach().clone()) for q in src]
    ref = FusedAdam(eager, lr=torch.tensor(2e-3, device="cuda"), capturable=True)
    ref.load_state_dict(sd)
    for p, q, g in zip(ps, eager, grads[0]):
        p.grad.copy_(g)
        q.grad = g.clone()
    graph.replay()
    ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ps, eager):
        assert torch.equal(a.detach(), b.detach())
    assert float(opt.state[ps[0]]["step"]) == 4.0
    if missing:
        assert "exp_avg" in opt.state[ps[2]]


def test_load_state_dict_refuses_unequal_steps():
    from visual_onoma_to_wave_amd.optim import FusedAdam
    ps = [torch.nn.Parameter(torch.randn(4, device="cuda")) for _ in range(2)]
    ref = torch.optim.Adam(ps, lr=1e-3)
    ps[0].grad = torch.ones_like(ps[0])
    ref.step()
    ps[1].grad = torch.ones_like(ps[1])
    ref.step()  # ps[0] at step 2, ps[1] at step 1
    opt = FusedAdam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1e-3)
    with pytest.raises(ValueError, match="unequal per-parameter steps"):
        opt.load_state_dict(ref.state_dict())
