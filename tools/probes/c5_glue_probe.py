#!/usr/bin/env python3
"""Which Python-level ops launch the C5 step's PyTorch glue kernels (fills, copies, adds): one
eager step (B = 16 x 8192, bf16) under torch.profiler, aten ops with their GPU time and the
innermost frames of this package that called them.

    python tools/probes/c5_glue_probe.py [rows]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
from helpers import hifigan_arrays, hifigan_h  # noqa: E402
from weights import load_into  # noqa: E402
from visual_onoma_to_wave_amd import hifigan  # noqa: E402
from visual_onoma_to_wave_amd.hifigan.discriminators import MelLoss  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    h = hifigan.AttrDict(hifigan_h())
    g = hifigan.Generator(h)
    load_into(g, hifigan_arrays())
    g = g.cuda()
    torch.manual_seed(1234)
    tr = hifigan.HifiGanTrainer(g, h).set_compute_dtype(torch.bfloat16)
    B, seg = 16, h.segment_size
    t = torch.arange(seg, dtype=torch.float32) / h.sampling_rate
    y = (0.3 * torch.sin(2 * np.pi * 220.0 * t) + 0.05 * torch.randn(B, seg)).cuda()
    with torch.no_grad():
        x = MelLoss(h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin, h.fmax).cuda().mel(y)
    x = x.transpose(1, 2).contiguous()
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
        tr.step(x, y)
        torch.cuda.synchronize()
    keep = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::cat", "aten::clone",
            "aten::constant_pad_nd", "aten::mul", "aten::where", "aten::contiguous", "aten::sum", "aten::to",
            "aten::slice_backward", "aten::zeros", "aten::zeros_like")
    ka = prof.key_averages(group_by_stack_n=6)
    ev = [e for e in ka if e.key in keep and e.device_time_total > 0]
    ev.sort(key=lambda e: -e.device_time_total)
    tot = sum(e.device_time_total for e in ev)
    print(f"glue ops total GPU time {tot / 1e3:.2f} ms in one eager step")
    for e in ev[:rows]:
        frames = [f for f in e.stack if "visual_onoma_to_wave_amd" in f][:3] or list(e.stack)[:3]
        print(f"{e.key:24s} calls {e.count:4d}  gpu {e.device_time_total / 1e3:7.3f} ms  | " + " <- ".join(
            f.split("visual_onoma_to_wave_amd/")[-1] for f in frames))


if __name__ == "__main__":
    main()
