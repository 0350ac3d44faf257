"""One MRF kernel at a bench shape (B=32), launched a few times, for rocprofv3 counter passes.

    python tools/probes/mrf_probe.py pair C k d [pair_cfg]   |   python tools/probes/mrf_probe.py rb3 C
    python tools/probes/mrf_probe.py conv 256 k d [conv_cfg]  (stage-0 conv, vo_conv1d variant 1, residual on)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

T_OF = {128: 32768, 64: 65536, 32: 131072, 256: 4096}


def main():
    kind, C = sys.argv[1], int(sys.argv[2])
    B, T = 32, T_OF[C]
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    if kind == "pair":
        k, d = int(sys.argv[3]), int(sys.argv[4])
        if len(sys.argv) > 5:
            _lib.lib().vo_tune(b"pair_cfg", int(sys.argv[5]))
        w = [ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
             for _ in range(2)]
        frag = C in (64, 128) and k in (7, 11) and os.environ.get("VO_FRAG", "1") != "0"  # as the Generator
        if frag:
            w = [ops.pack_frag(q) for q in w]
        fn = lambda: ops.resblock_pair(x, w[0], b, w[1], b, k, d, 0.1, out=y, out_scale=1 / 3, acc=y,  # noqa: E731
                                       frag=frag)
    elif kind == "conv":
        k, d = int(sys.argv[3]), int(sys.argv[4])
        if len(sys.argv) > 5:
            _lib.lib().vo_tune(b"conv_cfg", int(sys.argv[5]))
        w = ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
        fn = lambda: ops.conv1d(x, w, b, Co=C, K=k, dil=d, pad=d * (k - 1) // 2, pre_act=ops.ACT_LRELU,  # noqa: E731
                                pre_slope=0.1, out=y, res1=x, variant=1)
    else:
        w1 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda", generator=g) / (C * 3) ** 0.5, torch.bfloat16)
              for _ in range(3)]
        w2 = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda", generator=g) / (C * 3) ** 0.5, torch.bfloat16)
              for _ in range(3)]
        fn = lambda: ops.resblock3(x, w1, [b] * 3, w2, [b] * 3, (1, 3, 5), 0.1, out=y, out_scale=1 / 3, acc=y)  # noqa: E731
    for _ in range(4):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
