#!/usr/bin/env python3
"""The C2 decoder's T_mel convs alone (B = 32 x 512 rows, bf16 input as the mixed decoder now feeds
them), timed for each gen_cfg tile choice (outputs compared bit for bit with gen_cfg 0).

    python tools/probes/dec_convs.py [gen_cfg ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

SHAPES = {  # name: (Ci, Co, K, post_act, out dtype)
    "ffn_w1": (256, 1024, 9, ops.ACT_RELU, torch.bfloat16),
    "qkv": (256, 768, 1, ops.ACT_NONE, torch.bfloat16),
    "ffn_w2": (1024, 256, 1, ops.ACT_NONE, torch.float32),
    "fc": (256, 256, 1, ops.ACT_NONE, torch.float32),
}


def main(cfgs):
    L = _lib.lib()
    B, T = 32, 512
    for name, (ci, co, k, act, odt) in SHAPES.items():
        x = torch.randn(B, T, ci, device="cuda").to(torch.bfloat16)
        w = ops.pack_conv_weight(torch.randn(co, ci, k, device="cuda") / (ci * k) ** 0.5, torch.bfloat16)
        b = torch.randn(co, device="cuda") * 0.1
        y = torch.empty(B, T, co, device="cuda", dtype=odt)
        fn = lambda: ops.conv1d(x, w, b, Co=co, K=k, pad=(k - 1) // 2, post_act=act, out=y,  # noqa: E731
                                compute_dtype=torch.bfloat16)
        ref, line = None, f"{name:7s}"
        for c in cfgs:
            L.vo_tune(b"gen_cfg", c)
            fn()
            torch.cuda.synchronize()
            same = "" if ref is None else ("==" if torch.equal(y, ref) else "DIFF")
            ref = y.clone() if ref is None else ref
            ts = []
            for _ in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    fn()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 20 * 1e3)
            t = sorted(ts)[2]
            fl = 2.0 * B * T * ci * co * k
            line += f" | cfg {c}{same} {t:6.1f} us {fl / t / 1e6:6.0f} TF/s"
        L.vo_tune(b"gen_cfg", 0)
        if k == 1:  # the library GEMM on the same operands (hipBLASLt through torch), for reference
            x2, wt = x.reshape(-1, ci), torch.randn(ci, co, device="cuda").to(torch.bfloat16)
            bb = b.to(odt)
            if odt == torch.float32:
                g = lambda: torch.addmm(bb, x2, wt, out_dtype=torch.float32)  # noqa: E731
            else:
                g = lambda: torch.addmm(bb, x2, wt)  # noqa: E731
            g()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    g()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 20 * 1e3)
            t = sorted(ts)[2]
            line += f" | torch.addmm {t:6.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [0, 1, 10])
