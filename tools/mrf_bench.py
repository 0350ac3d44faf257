#!/usr/bin/env python3
"""Per-launch times of every HiFi-GAN MRF kernel at the bench shapes (B = 32, T_mel = 512):
stage 0 (C = 256: two conv launches per ResBlock iteration), stages 1-3 (C = 128 / 64 / 32:
the k = 3 block launch and the k = 7 / 11 pair launches), with the MRF accumulator, on random
bf16 activations and weights.  Each variant of a ``--tune key=v1,v2`` sweep is checked bit for
bit against the first one and timed in interleaved rounds in this one process.

    python tools/mrf_bench.py [--stages 0,1,2,3] [--tune pair_cfg=0,7] [--rounds 3] [--n 10]
"""
import argparse
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

PEAK = 2500.0
FRAG = os.environ.get("VO_FRAG", "1") != "0"  # C = 64 / 128 pairs on fragment-ordered weights, as the Generator
# channel widths run on fragment-ordered packs (VO_FRAG_C="128": C = 64 on [K][Co][Ci] packs, for A/B)
FRAG_C = tuple(int(c) for c in os.environ.get("VO_FRAG_C", "64,128").split(","))
ACC = os.environ.get("MRF_BENCH_ACC", "1") != "0"  # pairs with the MRF accumulator (0: plain y)
STAGES = {0: (256, 4096), 1: (128, 32768), 2: (64, 65536), 3: (32, 131072)}
DILS = (1, 3, 5)


def timeit(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def workloads(C, T, B):
    g = torch.Generator(device="cuda").manual_seed(C)
    x = (torch.randn(B, T, C, device="cuda", generator=g)).to(torch.bfloat16)
    acc = (torch.randn(B, T, C, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    y = torch.empty_like(x)

    def w(k):
        return ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (k * C) ** 0.5,
                                    torch.bfloat16)

    def b():
        return torch.randn(C, device="cuda", generator=g) * 0.1

    out = []
    for k in (3, 7, 11):
        p = [(w(k), b(), w(k), b()) for _ in DILS]
        fl1 = 2 * 2.0 * B * T * C * C * k  # one (c1, c2) pair
        if C == 256:
            t = torch.empty_like(x)

            def conv_pair(d, p=p[0], k=k):
                ops.conv1d(x, p[0], p[1], Co=C, K=k, dil=d, pad=d * (k - 1) // 2, pre_act=ops.ACT_LRELU,
                           pre_slope=0.1, post_act=ops.ACT_LRELU, post_slope=0.1, out=t, variant=1)
                ops.conv1d(t, p[2], p[3], Co=C, K=k, pad=(k - 1) // 2, res1=x, out=y, res2=acc,
                           out_scale=1.0 / 3, variant=1)
            for d in DILS:
                out.append((f"k{k} d{d} conv pair", lambda d=d, f=conv_pair: f(d), fl1))
        elif k == 3:
            def rb3(p=p):
                ops.resblock3(x, [q[0] for q in p], [q[1] for q in p], [q[2] for q in p], [q[3] for q in p], DILS,
                              0.1, out=y, out_scale=1.0 / 3, acc=acc)
            out.append(("k3 block (3 pairs)", rb3, 3 * fl1))
        else:
            for d, q in zip(DILS, p):
                if FRAG and C in FRAG_C:  # the Generator's fragment-ordered packs (vo_pack_frag)
                    q = (ops.pack_frag(q[0]), q[1], ops.pack_frag(q[2]), q[3])

                def pair(d=d, q=q, k=k):
                    ops.resblock_pair(x, q[0], q[1], q[2], q[3], k, d, 0.1, out=y, out_scale=1.0 / 3,
                                      acc=acc if ACC else None, frag=FRAG and C in FRAG_C and k in (7, 11))
                out.append((f"k{k} d{d} pair", pair, fl1))
    return y, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="0,1,2,3")
    ap.add_argument("--tune", action="append", default=[], help="key=v1,v2,... (vo_tune sweep)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    keys, vals = [], []
    for t in a.tune:
        k, v = t.split("=")
        keys.append(k)
        vals.append([int(x) for x in v.split(",")])
    combos = list(itertools.product(*vals)) if keys else [()]
    L = _lib.lib()

    def setc(c):
        for k, v in zip(keys, c):
            L.vo_tune(k.encode(), v)

    for s in [int(x) for x in a.stages.split(",")]:
        C, T = STAGES[s]
        y, work = workloads(C, T, a.batch)
        for name, fn, fl in work:
            ref, res = None, {}
            for c in combos:
                setc(c)
                fn()
                torch.cuda.synchronize()
                same = "" if ref is None else ("==" if torch.equal(y, ref) else "DIFF")
                if ref is None:
                    ref = y.clone()
                res[c] = [same]
            for _ in range(a.rounds):
                for c in combos:
                    setc(c)
                    fn()
                    res[c].append(timeit(fn, a.n))
            line = f"s{s} C={C:3d} {name:20s}"
            for c in combos:
                ts = sorted(res[c][1:])
                med = ts[len(ts) // 2]
                lab = ",".join(f"{k}={v}" for k, v in zip(keys, c)) or "default"
                line += f" | {lab}{res[c][0]} {med * 1e3:7.1f} us {fl / med / 1e9:6.0f} TF/s ({fl / med / 1e9 / PEAK:.3f})"
            print(line, flush=True)
        setc(tuple(0 for _ in keys))
        del y, work
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
