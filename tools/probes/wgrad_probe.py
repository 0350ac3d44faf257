"""Counter / timing probe for the round-6 weight-gradient kernels: the K = 1 kernel on the C4 decoder's q/k/v
shape and the strided multi-tap kernel on the MSD's k = 41 stride-2 grouped layer, 5 calls each
(tools/wgrad_counters.sh runs it under rocprofv3 --pmc)."""

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from visual_onoma_to_wave_amd import ops  # noqa: E402

g = torch.Generator().manual_seed(0)
dev = torch.device("cuda", 0)
x = torch.randn(32, 512, 256, generator=g).bfloat16().to(dev)
gy = torch.randn(32, 512, 768, generator=g).bfloat16().to(dev)
xs = torch.randn(32, 4096, 128, generator=g).bfloat16().to(dev)
gs = torch.randn(32, 2048, 256, generator=g).bfloat16().to(dev)
for _ in range(5):
    ops.conv1d_wgrad(gy, x, 1, with_bias=True)
    ops.conv1d_wgrad(gs, xs, 41, S=2, pad=20, groups=16, with_bias=True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn in (("k1 q/k/v 32x512 256->768", lambda: ops.conv1d_wgrad(gy, x, 1, with_bias=True)),
                 ("mt MSD k41 s2 g16 32x2048", lambda: ops.conv1d_wgrad(gs, xs, 41, S=2, pad=20, groups=16,
                                                                         with_bias=True))):
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    e1.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call (kernel + reduce)", flush=True)
