#!/usr/bin/env python3
"""The C4 decoder's attention backward alone (B = 32, L = 512, d_model 256, 2 heads, bf16, the
forward's row log-sum-exp): per-call time of vo_attention_bwd_lse and its fraction of the dense
bf16 peak on the full-L FLOP count (S recompute, dV, dP, dQ, dK: 5 x 2 B H L^2 d_k).

    python tools/probes/attn_bwd_probe.py [--lens full|ragged] [--n 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import ops  # noqa: E402

PEAK = 2.5e15


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="full", choices=["full", "ragged"])
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--att-cfg", default="0", help="comma list of att_cfg values, timed alternately (A/B)")
    a = ap.parse_args()
    B, L, D, H = 32, 512, 256, 2
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B, L, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    dout = torch.randn(B, L, D, device="cuda", generator=g).to(torch.bfloat16)
    if a.lens == "full":
        lens = torch.full((B,), L, dtype=torch.int32, device="cuda")
    else:
        lens = torch.randint(L // 2, L + 1, (B,), generator=g, device="cuda").to(torch.int32)
    out, lse = ops.attention(qkv, lens, H, with_lse=True)
    dq = ops.attention_bwd(qkv, out, dout, lens, H, lse=lse)
    torch.cuda.synchronize()
    assert torch.isfinite(dq.float()).all()
    from visual_onoma_to_wave_amd import _lib
    cfgs = [int(c) for c in a.att_cfg.split(",")]
    ts = {c: [] for c in cfgs}
    ref = None
    for _ in range(5):
        for c in cfgs:
            _lib.lib().vo_tune(b"att_cfg", c)
            got = ops.attention_bwd(qkv, out, dout, lens, H, lse=lse)
            if ref is None:
                ref = got.clone()
            elif not torch.equal(got, ref):
                print(f"att_cfg {c}: DIFFERS from att_cfg {cfgs[0]}", flush=True)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.n):
                ops.attention_bwd(qkv, out, dout, lens, H, lse=lse)
            e.record()
            torch.cuda.synchronize()
            ts[c].append(s.elapsed_time(e) / a.n * 1e3)
    _lib.lib().vo_tune(b"att_cfg", 0)
    fw = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.n):
            ops.attention(qkv, lens, H, out=out, with_lse=True)
        e.record()
        torch.cuda.synchronize()
        fw.append(s.elapsed_time(e) / a.n * 1e3)
    tf = sorted(fw)[2]
    print(f"attention fwd (lens {a.lens}): {tf:.1f} us per call, "
          f"{2 * 2.0 * B * H * L * L * (D // H) / tf / 1e6:.0f} TF/s on full-L FLOPs", flush=True)
    dk = D // H
    fl = 5 * 2.0 * B * H * L * L * dk
    fl_live = 5 * 2.0 * H * dk * float((lens.double() ** 2).sum())
    for c in cfgs:
        t = sorted(ts[c])[2]
        print(f"attention bwd (lens {a.lens}, att_cfg {c}): {t:.1f} us per call, {fl / t / 1e6:.0f} TF/s on full-L "
              f"FLOPs ({fl / t / 1e6 / PEAK * 1e12:.3f} of peak), {fl_live / t / 1e6:.0f} TF/s on live FLOPs", flush=True)


if __name__ == "__main__":
    main()
