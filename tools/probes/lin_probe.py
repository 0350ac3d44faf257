#!/usr/bin/env python3
"""K = 1 convs (the transformer's Linear layers at B = 32 x 512 rows): conv1d_kernel (lin_cfg 0)
against lin_kernel tiles (lin_cfg 5 / 2 / 3 / 4, A/B library only: VO_LIB_PATH=.../libvonoma_abl.so),
outputs compared bit for bit with conv1d_kernel.

    python tools/probes/lin_probe.py [lin_cfg ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

SHAPES = {  # name: (Ci, Co, post_act, out dtype, residual)
    "qkv": (256, 768, ops.ACT_NONE, torch.bfloat16, False),
    "fc": (256, 256, ops.ACT_NONE, torch.float32, False),
    "ffn_w2": (1024, 256, ops.ACT_NONE, torch.float32, False),
    "w2_dgrad": (256, 1024, ops.ACT_NONE, torch.bfloat16, False),
    "fc_relu_res": (512, 256, ops.ACT_RELU, torch.bfloat16, True),
}


def timeit(fn):
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20 * 1e3)
    return sorted(ts)[2]


def main(cfgs):
    L = _lib.lib()
    B, T = 32, 512
    torch.manual_seed(0)
    for name, (ci, co, act, odt, res) in SHAPES.items():
        x = torch.randn(B, T, ci, device="cuda").to(torch.bfloat16)
        wf = torch.randn(co, ci, 1, device="cuda") / ci ** 0.5
        w = ops.pack_conv_weight(wf, torch.bfloat16)
        b = torch.randn(co, device="cuda") * 0.1
        r = torch.randn(B, T, co, device="cuda").to(odt) if res else None
        y = torch.empty(B, T, co, device="cuda", dtype=odt)
        fn = lambda: ops.conv1d(x, w, b, Co=co, K=1, pad=0, post_act=act, out=y, res1=r,  # noqa: E731
                                compute_dtype=torch.bfloat16)
        ref, line = None, f"{name:11s}"
        for c in [0] + cfgs:
            L.vo_tune(b"lin_cfg", c)
            y.zero_()
            fn()
            torch.cuda.synchronize()
            same = "" if ref is None else ("==" if torch.equal(y, ref) else "DIFF")
            if ref is None:
                ref = y.clone()
                f32 = x.float().reshape(-1, ci) @ wf.to(torch.bfloat16).float()[:, :, 0].t() + b
                if act == ops.ACT_RELU:
                    f32 = f32.relu()
                if res:
                    f32 = f32 + r.float().reshape(-1, co)
                err = (ref.float().reshape(-1, co) - f32).abs().max().item()
                line += f" | max|err| vs fp32 {err:.3g}"
            t = timeit(fn)
            mb = (x.numel() * 2 + y.numel() * y.element_size() + (r.numel() * r.element_size() if res else 0)) / 1e6
            line += f" | cfg {c}{same} {t:6.1f} us {mb / t:5.2f} TB/s"
        L.vo_tune(b"lin_cfg", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [5, 2, 3, 4])
