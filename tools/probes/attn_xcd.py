#!/usr/bin/env python3
"""Attention forward at the C2 shape (B = 32, L = 512, 2 heads, full lengths) and the encoder's fp32
shape, forward and backward with and without the XCD-grouped workgroup order (vo_tune att_xcd: 0 = grouped, 1 = plain
(tile, head) order); outputs compared bit for bit.  python tools/probes/attn_xcd.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def t_us(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    L_ = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(0)
    for (B, L, dt) in ((32, 512, torch.bfloat16), (32, 12, torch.float32), (32, 512, torch.float32)):
        qkv = torch.randn(B, L, 768, device="cuda", generator=g).to(dt)
        lens = torch.full((B,), L, device="cuda", dtype=torch.int32)
        dout = torch.randn(B, L, 256, device="cuda", generator=g).to(dt)
        line = f"B={B} L={L} {str(dt)[6:]}:"
        ref = None
        for cfg in (1, 0):
            assert L_.vo_tune(b"att_xcd", cfg) == 0
            out = ops.attention(qkv, lens, 2)
            dq = ops.attention_bwd(qkv, out, dout, lens, 2)
            same = "" if ref is None else ("==" if torch.equal(out, ref[0]) and torch.equal(dq, ref[1]) else "DIFF")
            ref = (out.clone(), dq.clone()) if ref is None else ref
            f = t_us(lambda: ops.attention(qkv, lens, 2, out=out))
            bw = t_us(lambda: ops.attention_bwd(qkv, out, dout, lens, 2))
            line += f"  [att_xcd={cfg}{same}] fwd {f:7.1f} us bwd {bw:7.1f} us"
        L_.vo_tune(b"att_xcd", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
