#!/usr/bin/env python3
"""Where the C5 step's small launches come from: one eager HiFi-GAN training step (bench.py's C5
setup, B = 16 x 8192) under torch.profiler with Python stacks; prints the aten ops that launch
fills, copies and adds, grouped by their innermost package frames.

    python tools/probes/c5_glue_sources.py [n_rows]
"""
import os
import sys
from collections import Counter

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
import bench  # noqa: E402


def main(n=40):
    class A:
        batch, precision, no_graph, comm_dtype, stft_loss, warmup, steps = 16, "mixed", True, "fp32", 0.0, 2, 1
    dev = torch.device("cuda")
    # build the trainer as bench.run_gan does, then profile one more eager step
    from helpers import hifigan_arrays, hifigan_h
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.hifigan.discriminators import MelLoss
    import numpy as np
    h = hifigan.AttrDict(hifigan_h())
    g = hifigan.Generator(h)
    load_into(g, hifigan_arrays())
    g = g.to(dev)
    torch.manual_seed(1234)
    tr = hifigan.HifiGanTrainer(g, h, device=dev).set_compute_dtype(torch.bfloat16)
    seg = h.segment_size
    t = torch.arange(seg, dtype=torch.float32) / h.sampling_rate
    y = (0.3 * torch.sin(2 * np.pi * 220.0 * t) + 0.05 * torch.randn(A.batch, seg)).to(dev)
    with torch.no_grad():
        x = MelLoss(h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin, h.fmax).to(dev).mel(y)
    x = x.transpose(1, 2).contiguous()
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    want = ("fill_", "zero_", "copy_", "add", "add_", "zeros", "mul", "constant_pad_nd", "clone", "sum", "sub", "div",
            "cat", "_to_copy", "new_zeros", "zeros_like", "empty_like", "where")
    cnt = Counter()

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.overloadpacket.__name__
            if name in want:
                node = torch._C._current_autograd_node()
                frames = [f"{os.path.basename(fr.filename)}:{fr.lineno}" for fr in traceback.extract_stack()
                          if "visual_onoma_to_wave_amd" in fr.filename]
                where = (f"[bwd {node.name()}] " if node is not None else "") + " <- ".join(frames[-1:-4:-1])
                cnt[(name, where)] += 1
            return func(*args, **(kwargs or {}))

    with Mode():
        tr.step(x, y)
        torch.cuda.synchronize()
    for (name, where), c in cnt.most_common(int(n)):
        print(f"{c:5d}  {name:16s} {where}")


if __name__ == "__main__":
    main(*sys.argv[1:])
