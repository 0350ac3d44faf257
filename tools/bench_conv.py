#!/usr/bin/env python3
"""Microbenchmark of the conv1d kernel on the HiFi-GAN MRF shapes (B=32 utterances of
512 mel frames) and the acoustic FFN shape.  Times each launch class with HIP events over
N back-to-back launches on random data; prints TFLOP/s and algorithmic HBM GB/s.

    python tools/bench_conv.py [--iters 20] [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import ops  # noqa: E402


def time_launch(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    B = a.batch
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cases = []
    for stage, (C, T) in enumerate([(256, 4096), (128, 32768), (64, 65536), (32, 131072)]):
        for k, d in [(3, 1), (3, 5), (7, 3), (11, 1), (11, 5)]:
            cases.append(dict(name=f"mrf_s{stage}_k{k}_d{d}", B=B, T=T, Ci=C, Co=C, K=k, dil=d, var=stage + 1,
                              pre=ops.ACT_LRELU, res=(d == 1)))
    cases.append(dict(name="ffn_w1", B=B, T=512, Ci=256, Co=1024, K=9, dil=1, var=0, pre=0, res=False))
    cases.append(dict(name="ffn_w2", B=B, T=512, Ci=1024, Co=256, K=1, dil=1, var=0, pre=0, res=False))
    cases.append(dict(name="ups1", B=B, T=4096, Ci=256, Co=8 * 128, K=2, dil=1, var=0, pre=ops.ACT_LRELU,
                      res=False, up=dict(stride=8, pad=4, cout=128)))
    out = {}
    for c in cases:
        x = torch.randn(c["B"], c["T"], c["Ci"], device=dev).to(torch.bfloat16)
        w = torch.randn(c["Co"], c["Ci"], c["K"], device=dev) / (c["Ci"] * c["K"]) ** 0.5
        wp = ops.pack_conv_weight(w, torch.bfloat16)
        bias = torch.zeros(c["Co"], device=dev)
        pad = c["dil"] * (c["K"] - 1) // 2
        up = c.get("up")
        if up:
            wt = torch.randn(c["Ci"], up["cout"], 2 * up["stride"], device=dev) / c["Ci"] ** 0.5
            wp = ops.pack_conv_weight(wt, torch.bfloat16, transposed_stride=up["stride"])
            bias = torch.zeros(up["cout"], device=dev)
            y = torch.empty(c["B"], c["T"] * up["stride"], up["cout"], device=dev, dtype=torch.bfloat16)
            fn = lambda: ops.conv1d(x, wp, bias, Co=c["Co"], K=2, pad=1, pre_act=c["pre"], pre_slope=0.1,  # noqa
                                    transposed=up, out=y, compute_dtype=torch.bfloat16)
        else:
            y = torch.empty(c["B"], c["T"], c["Co"], device=dev, dtype=torch.bfloat16)
            r = torch.randn_like(y) if c["res"] else None
            fn = lambda: ops.conv1d(x, wp, bias, Co=c["Co"], K=c["K"], dil=c["dil"], pad=pad,  # noqa
                                    pre_act=c["pre"], pre_slope=0.1, res1=r, out=y, variant=c["var"],
                                    compute_dtype=torch.bfloat16)
        ms = time_launch(fn, a.iters)
        flops = 2.0 * c["B"] * c["T"] * c["Co"] * c["Ci"] * c["K"]
        nbytes = 2.0 * c["B"] * c["T"] * (c["Ci"] + c["Co"] * (2 if c["res"] else 1))
        out[c["name"]] = dict(ms=round(ms, 4), tflops=round(flops / ms / 1e9, 1),
                              gbs=round(nbytes / ms / 1e6, 1))
        print(f'{c["name"]:18s} {ms:8.4f} ms {flops / ms / 1e9:8.1f} TF/s {nbytes / ms / 1e6:8.1f} GB/s', flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
