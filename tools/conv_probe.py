#!/usr/bin/env python3
"""Run a few launches of the MRF conv / fused-pair shapes for counter collection (rocprofv3 --pmc).

    python tools/conv_probe.py s1_k11 pair_s2_k11 ...
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from visual_onoma_to_wave_amd import ops  # noqa: E402

SHAPES = {"s0_k11": (256, 4096, 11, 5, 1), "s1_k11": (128, 32768, 11, 5, 2), "s1_k3": (128, 32768, 3, 1, 2),
          "s1_k7": (128, 32768, 7, 3, 2),
          "s2_k7": (64, 65536, 7, 3, 3), "s3_k3": (32, 131072, 3, 1, 4), "s3_k11": (32, 131072, 11, 5, 4)}
PAIRS = {"pair_s1_k3": (128, 32768, 3, 1), "pair_s1_k7": (128, 32768, 7, 3), "pair_s1_k11": (128, 32768, 11, 5),
         "pair_s2_k3": (64, 65536, 3, 1), "pair_s2_k11": (64, 65536, 11, 5), "pair_s3_k3": (32, 131072, 3, 1),
         "pair_s3_k11": (32, 131072, 11, 5), "pair_s2_k7": (64, 65536, 7, 3)}


def main(names, iters=5, B=32):
    dev = torch.device("cuda")
    for name in names:
        if name == "dec_ffn_w1":  # C2 decoder FFN w_1 (transformer/SubLayers.py:85-93): 256 -> 1024, k 9, relu
            x = torch.randn(B, 512, 256, device=dev).to(torch.bfloat16)
            w = ops.pack_conv_weight(torch.randn(1024, 256, 9, device=dev) / (256 * 9) ** 0.5, torch.bfloat16)
            bias = torch.zeros(1024, device=dev)
            y = torch.empty(B, 512, 1024, device=dev, dtype=torch.bfloat16)
            for _ in range(iters):
                ops.conv1d(x, w, bias, Co=1024, K=9, pad=4, post_act=ops.ACT_RELU, out=y, compute_dtype=torch.bfloat16)
            torch.cuda.synchronize()
            continue
        if name in PAIRS:
            C, T, k, d = PAIRS[name]
            x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
            w1 = ops.pack_conv_weight(torch.randn(C, C, k, device=dev) / (C * k) ** 0.5, torch.bfloat16)
            w2 = ops.pack_conv_weight(torch.randn(C, C, k, device=dev) / (C * k) ** 0.5, torch.bfloat16)
            bias = torch.zeros(C, device=dev)
            y = torch.empty_like(x)
            for _ in range(iters):
                ops.resblock_pair(x, w1, bias, w2, bias, k, d, 0.1, out=y)
            torch.cuda.synchronize()
            continue
        C, T, k, d, var = SHAPES[name]
        x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
        w = ops.pack_conv_weight(torch.randn(C, C, k, device=dev) / (C * k) ** 0.5, torch.bfloat16)
        bias = torch.zeros(C, device=dev)
        y = torch.empty_like(x)
        for _ in range(iters):
            ops.conv1d(x, w, bias, Co=C, K=k, dil=d, pad=d * (k - 1) // 2, pre_act=ops.ACT_LRELU, pre_slope=0.1,
                       out=y, variant=var, compute_dtype=torch.bfloat16)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1:] or ["s1_k11", "s3_k3"])
