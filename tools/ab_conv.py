#!/usr/bin/env python3
"""Interleaved A/B of conv1d tuning knobs on MRF shapes (one process, rounds x variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    B = 32
    shapes = [("s0_k3", 256, 4096, 3, 1, 1), ("s1_k3", 128, 32768, 3, 1, 2), ("s1_k11", 128, 32768, 11, 5, 2),
              ("s2_k7", 64, 65536, 7, 3, 3), ("s3_k3", 32, 131072, 3, 1, 4), ("s3_k11", 32, 131072, 11, 5, 4)]
    res = {}
    for name, C, T, k, d, var in shapes:
        x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
        w = ops.pack_conv_weight(torch.randn(C, C, k, device=dev) / (C * k) ** 0.5, torch.bfloat16)
        bias = torch.zeros(C, device=dev)
        y = torch.empty_like(x)
        fn = lambda: ops.conv1d(x, w, bias, Co=C, K=k, dil=d, pad=d * (k - 1) // 2, pre_act=ops.ACT_LRELU,  # noqa
                                pre_slope=0.1, out=y, variant=var, compute_dtype=torch.bfloat16)
        for rnd in range(3):
            for knob in (0, 1):
                _lib.check(_lib.lib().vo_tune(b"conv_persistent", knob), "tune")
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res.setdefault((name, knob), []).append(s.elapsed_time(e) / 10)
        fl = 2.0 * B * T * C * C * k
        for knob in (0, 1):
            t = min(res[(name, knob)])
            print(f"{name:8s} persistent={knob} {t:.4f} ms {fl / t / 1e9:7.1f} TF/s", flush=True)
    _lib.lib().vo_tune(b"conv_persistent", 0)


if __name__ == "__main__":
    main()
