"""vo_attention bf16 at the decoder shape (B = 32, L = 512, 2 heads of 128): att_cfg 0 vs 1."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402

qkv = torch.randn(32, 512, 768, device="cuda").to(torch.bfloat16)
lens = torch.full((32,), 512, dtype=torch.int32, device="cuda")
fl = 4.0 * 512 * 512 * 128 * 64
for c in (1, 0, 1, 0):
    _lib.lib().vo_tune(b"att_cfg", c)
    for _ in range(3):
        ops.attention(qkv, lens, 2)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        ops.attention(qkv, lens, 2)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print(f"att_cfg {c}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s", flush=True)
