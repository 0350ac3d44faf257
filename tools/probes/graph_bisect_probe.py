"""Bisect the HIP-graph replay failure of the C4 step (graph_race_probe.py: NaN from the first
replay with CLR graph packet capture on, none with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).

Part 1 captures segments of the step (forward + loss; + backward; the clip + Adam update alone)
and compares one replay with the same segment run eagerly from the same state.  Part 2 captures
single ops (ours and torch's) and compares a replay with the eager result.

    python tools/probes/graph_bisect_probe.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
from helpers import configs, vtts_arrays  # noqa: E402
from weights import load_into  # noqa: E402
from visual_onoma_to_wave_amd import ops, synth  # noqa: E402
from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    a, b = a.double(), b.double()
    if not torch.isfinite(a).all():
        return float("nan")
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def graphed(fn, warm=1):
    """Run fn eagerly `warm` times on a side stream, capture it, replay once; returns the outputs."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    g.replay()
    torch.cuda.synchronize()
    return out, g


def no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0


def model_and_batch(prec):
    pc, mc, tc = configs()
    b = synth.acoustic_batch(1234, 8, 12, 256)
    t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
             t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision(prec)
    no_dropout(m)
    return m, batch, (pc, mc, tc)


def part1(prec):
    m, batch, (pc, mc, tc) = model_and_batch(prec)
    lossf = FastSpeech2Loss()

    def fwd():
        with torch.no_grad():
            out = m(*(batch[1:]), True)
            return torch.stack([x.float() for x in lossf(batch, out)])

    def fwd_bwd():
        for p in m.parameters():
            p.grad = None
        out = m(*(batch[1:]), True)
        losses = lossf(batch, out)
        losses[0].backward()
        return [p.grad for p in m.parameters() if p.grad is not None]

    # running stats of train-mode BatchNorm move every call: snapshot / restore buffers
    bufs = {k: v.clone() for k, v in m.named_buffers()}

    def restore():
        for k, v in m.named_buffers():
            v.copy_(bufs[k])

    restore()
    ref = fwd().clone()
    restore()
    got, _ = graphed(fwd)
    print(f"[{prec}] forward+loss: rel {rel(got, ref):.3e}  got {got[:3].tolist()} ref {ref[:3].tolist()}", flush=True)
    restore()
    ref_g = [g.clone() for g in fwd_bwd()]
    restore()
    got_g, _ = graphed(fwd_bwd)
    errs = [rel(a, b) for a, b in zip(got_g, ref_g)]
    bad = [(i, e) for i, e in enumerate(errs) if not (e < 1e-3)]
    print(f"[{prec}] forward+backward: {len(errs)} grads, max rel {np.nanmax(errs):.3e}, bad {len(bad)} "
          f"{bad[:8]}", flush=True)

    # clip + Adam on fixed gradients
    for cap in (True,):
        ps = [p for p in m.parameters() if p.requires_grad]
        g0 = [torch.randn_like(p) * 1e-2 for p in ps]
        p0 = [p.detach().clone() for p in ps]

        def make():
            opt = ScheduledOptim(m, tc, mc, 0, capturable=cap)
            opt._update_learning_rate()
            return opt

        def step(opt):
            def f():
                for p, g in zip(ps, g0):
                    p.grad = g.clone()
                torch.nn.utils.clip_grad_norm_(ps, 1.0)
                opt._optimizer.step()
                return [p for p in ps]
            return f
        with torch.no_grad():
            for p, v in zip(ps, p0):
                p.copy_(v)
        opt = make()
        step(opt)()
        ref_p = [p.detach().clone() for p in ps]
        with torch.no_grad():
            for p, v in zip(ps, p0):
                p.copy_(v)
        opt = make()
        fn = step(opt)
        # warm-up on a side stream moves parameters too: undo it before the replay
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        with torch.no_grad():
            for p, v in zip(ps, p0):
                p.copy_(v)
        for st in opt._optimizer.state.values():
            for k, v in st.items():
                if torch.is_tensor(v):
                    v.zero_()
        g.replay()
        torch.cuda.synchronize()
        errs = [rel(p.detach(), r) for p, r in zip(ps, ref_p)]
        print(f"[{prec}] clip+Adam(capturable={cap}): max rel {np.nanmax(errs):.3e}, "
              f"nan {sum(1 for e in errs if e != e)}", flush=True)


def part2():
    gen = torch.Generator().manual_seed(0)
    r = lambda *s, dt=torch.float32: torch.randn(*s, generator=gen).to(dev, dt)  # noqa: E731
    cases = {}
    x32, x16 = r(4, 100, 256), r(4, 100, 256, dt=torch.bfloat16)
    w = r(1024, 256, 9) * 0.02
    wp32, wp16 = ops.pack_conv_weight(w, torch.float32), ops.pack_conv_weight(w, torch.bfloat16)
    b = r(1024)
    cases["conv1d f32"] = lambda: ops.conv1d(x32, wp32, b, Co=1024, K=9, pad=4, compute_dtype=torch.float32)
    cases["conv1d bf16"] = lambda: ops.conv1d(x16, wp16, b, Co=1024, K=9, pad=4)
    xs = r(8, 12, 256)
    cases["conv1d f32 splitK"] = lambda: ops.conv1d(xs, wp32, b, Co=1024, K=9, pad=4, compute_dtype=torch.float32)
    cases["pack_conv_weight"] = lambda: ops.pack_conv_weight(w, torch.bfloat16)
    cases["pack_dgrad_weight"] = lambda: ops.pack_dgrad_weight(w, torch.bfloat16)
    g32 = r(1024)
    cases["layernorm"] = lambda: ops.layernorm(x32, g32[:256], g32[256:512], res=x32)
    gy = r(4, 100, 256)
    cases["layernorm_bwd"] = lambda: torch.cat([t.flatten() for t in ops.layernorm_bwd(x32, gy, g32[:256], res=x32)])
    qkv = r(4, 100, 768)
    lens = torch.tensor([100, 70, 3, 99], dtype=torch.int32, device=dev)
    cases["attention"] = lambda: ops.attention(qkv, lens, 2)
    ao = ops.attention(qkv, lens, 2)
    cases["attention_bwd"] = lambda: ops.attention_bwd(qkv, ao, x32, lens, 2)
    dur = torch.tensor(np.random.default_rng(0).integers(0, 20, size=(4, 12)), dtype=torch.float32, device=dev)
    xl = r(4, 12, 256)
    cases["length_regulate"] = lambda: ops.length_regulate(xl, dur, 200)[0]
    gol = r(4, 200, 256)
    cases["length_regulate_bwd"] = lambda: ops.length_regulate_bwd(gol, dur, 12)
    go = r(4, 100, 1024, dt=torch.bfloat16)
    cases["conv1d_wgrad (memset+atomics)"] = lambda: ops.conv1d_wgrad(go, x16, 9, pad=4)
    cases["conv1d_wgrad_bias"] = lambda: torch.cat([t.flatten() for t in ops.conv1d_wgrad(go, x16, 9, pad=4,
                                                                                         with_bias=True)])
    cases["colsum"] = lambda: ops.colsum(go)
    cases["lrelu_mask"] = lambda: ops.lrelu_mask(go, go, 0.0)
    cases["mask_from_lengths"] = lambda: ops.mask_from_lengths(lens, 100)[0]
    cases["torch embedding bwd"] = None
    for name, fn in cases.items():
        if fn is None:
            continue
        try:
            ref = fn().clone()
            torch.cuda.synchronize()
            got, _ = graphed(fn)
            e = rel(got.float(), ref.float())
            print(f"  op {name:34s} rel {e:.3e} {'OK' if e < 1e-5 else 'MISMATCH'}", flush=True)
        except Exception as ex:  # noqa: BLE001
            print(f"  op {name:34s} ERROR {type(ex).__name__}: {ex}", flush=True)


if __name__ == "__main__":
    print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "unset"))
    part2()
    part1("fp32")
    part1("mixed")
