#!/usr/bin/env python3
"""vo_pack_batch throughput on the C5 step's pack plans (generator, MPD, MSD weight-normed scales):
time per launch set and the algorithmic bytes (fp32 weights read once, packed layouts written)
per second, against the per-layer pack kernels each conv would otherwise launch.

    python tools/probes/pack_batch_probe.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
from helpers import hifigan_h  # noqa: E402
from visual_onoma_to_wave_amd import hifigan, ops  # noqa: E402
from visual_onoma_to_wave_amd.hifigan import gan_ops as G  # noqa: E402
from visual_onoma_to_wave_amd.hifigan.discriminators import (MultiPeriodDiscriminator,  # noqa: E402
                                                             MultiScaleDiscriminator, _conv_w)


def plans():
    h = hifigan.AttrDict(hifigan_h())
    gen = hifigan.Generator(h)
    out = {"generator": [(m, G.conv_spec(s, sp, r), s, m is not gen.conv_pre)
                         for m, sp, s, r in gen._train_plan(16, 32)]}
    mpd = MultiPeriodDiscriminator()
    out["mpd"] = [(m, G.conv_spec(s, sp), s, True) for d in mpd.discriminators for m, sp, s in d._layers(32, 8192)]
    msd, T, lay = MultiScaleDiscriminator(), 8192, []
    for i, d in enumerate(msd.discriminators):
        T = T // 2 + 1 if i else T
        if i:  # the spectral-normed scale packs on use
            lay += [(m, G.conv_spec(s, sp), s, True) for m, sp, s in d._layers(32, T)]
    out["msd"] = lay
    return out


def _time(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        fn()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / reps


def main():
    dt = torch.bfloat16
    for name, layers in plans().items():
        groups = {}
        for m, sp, shape, dgrad in layers:
            w = m.weight_v if hasattr(m, "weight_g") else m.weight
            w = _conv_w(m, w.detach()).contiguous().cuda()
            for tag, dshape, f in G._pack_plan(tuple(w.shape), sp, dt, shape[-1], dgrad):
                dst = torch.zeros(dshape, dtype=dt, device="cuda")
                nb = w.numel() * 4 + f["T"] * f["rows"] * f["width"] * 2
                kind = tag[2] if tag[2] != "dgrad" else f"dgrad_S{sp.stride}"
                for key in ("all", kind):
                    g = groups.setdefault(key, [[], 0])
                    g[0].append((w, dst, f))
                    g[1] += nb
        for key, (jobs, nbytes) in groups.items():
            us = _time(lambda: ops.pack_batch(jobs, dt))
            print(f"{name:10s} {key:12s} {len(jobs):4d} jobs  {nbytes / 1e6:8.1f} MB  {us:8.1f} us  "
                  f"{nbytes / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
