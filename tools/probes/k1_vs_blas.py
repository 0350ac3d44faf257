"""K = 1 convs (the decoder's Linear layers at B * T = 16384 rows, bf16) on conv1d_kernel against the
vendor GEMM behind torch.nn.functional.linear (hipBLASLt) on the same operands: per-call time (event pairs
over 50 back-to-back calls) and the two results' rel-L2 distance.  A measurement probe only."""

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from visual_onoma_to_wave_amd import ops  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda", 0)


def clock(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for rows, ci, co in [(16384, 256, 768), (16384, 256, 256), (16384, 1024, 256), (16384, 256, 1024), (16384, 768, 256)]:
    x = torch.randn(32, rows // 32, ci, device=dev).bfloat16()
    w = (torch.randn(co, ci, device=dev) / ci ** 0.5)
    b = torch.randn(co, device=dev) * 0.1
    wp = ops.pack_conv_weight(w[:, :, None], torch.bfloat16)
    wb = w.bfloat16()
    t_vo = clock(lambda: ops.conv1d(x, wp, b, Co=co, K=1, compute_dtype=torch.bfloat16))
    t_bl = clock(lambda: torch.nn.functional.linear(x, wb, b.bfloat16()))
    y_vo = ops.conv1d(x, wp, b, Co=co, K=1, compute_dtype=torch.bfloat16).float()
    y_bl = torch.nn.functional.linear(x, wb, b.bfloat16()).float()
    rel = ((y_vo - y_bl).norm() / y_bl.norm()).item()
    fl = 2.0 * rows * ci * co
    print(f"rows {rows} {ci:5d} -> {co:5d}: conv1d_kernel {t_vo:7.1f} us ({fl / t_vo / 1e6:6.0f} TF/s)  "
          f"hipBLASLt {t_bl:7.1f} us ({fl / t_bl / 1e6:6.0f} TF/s)  rel {rel:.1e}", flush=True)
