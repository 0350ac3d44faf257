"""Per-conv timeline of the k = 3 ResBlock in the wave-owned-plane form (csrc/resblock_pb3.hip) from s_memtime
stamps.  Diagnostic library built here (never the product one):

    hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=1000000 \\
        -mllvm -amdgpu-mfma-vgpr-form=1 -DVO_PB3_STAMPS \\
        visual_onoma_to_wave_amd/csrc/resblock_pb3.hip visual_onoma_to_wave_amd/csrc/vo_runtime.cpp \\
        -o tools/probes/build/libpb3_stamps.so
    python tools/probes/pb3_stamps.py [C]

Prints, for tiles 1-3 of workgroups 0-15 (median over waves and workgroups), the shader cycles of each conv's
barrier, its phase 0 ("tap 0": tap 0), the two halves of phase 1 ("tap 1", "tap 2": taps 1 and 2 interleaved,
with the epilogues) and its tail.  Ideal tap at C = 128 (14 row tiles): 56 steps x 2 MFMAs x 16 cycles = 1,792.
(The stamped build is not the product code: its extra stores and waits cost ~10 % or more.)
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from visual_onoma_to_wave_amd import ops  # noqa: E402

NSTW, NSTT, NPT = 16, 4, 30


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    L = ctypes.CDLL(os.environ.get("PB3_LIB", os.path.join(ROOT, "tools/probes/build/libpb3_stamps.so")))
    B, T = 32, (32768 if C == 128 else 65536)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    w = [ops.pack_conv_weight(torch.randn(C, C, 3, device="cuda", generator=g) / (C * 3) ** 0.5, torch.bfloat16)
         for _ in range(6)]
    P = ctypes.c_void_p
    arr = lambda ts: (P * 3)(*[t.data_ptr() for t in ts])  # noqa: E731
    w1, w2, bb = arr(w[0::2]), arr(w[1::2]), arr([b, b, b])
    n = NSTW * 4 * NSTT * NPT
    buf = (ctypes.c_ulonglong * n)()
    fn = L.vo_pb3_stamps
    fn.argtypes = [P, P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    fn.restype = ctypes.c_int
    for _ in range(3):  # warm clocks; keep the last
        assert fn(P(x.data_ptr()), w1, bb, w2, bb, P(y.data_ptr()), B, T, C, ctypes.cast(buf, P)) == 0
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(NSTW, 4, NSTT, NPT)[:, :, 1:, :]
    tile = np.median((st[:, :, 1:, 0] - st[:, :, :-1, 0]).reshape(-1)) if NSTT > 2 else 0
    print(f"C = {C}: median tile {tile:.0f} cycles (s_memtime units)")
    for v in range(6):
        nxt = 5 * (v + 1) if v < 5 else None
        seg = [("barrier", 5 * v, 5 * v + 1), ("tap 0", 5 * v + 1, 5 * v + 2), ("tap 1", 5 * v + 2, 5 * v + 3),
               ("tap 2", 5 * v + 3, 5 * v + 4)]
        vals = []
        for name, i0, i1 in seg:
            vals.append((name, float(np.median((st[..., i1] - st[..., i0]).reshape(-1)))))
        if nxt is not None:
            vals.append(("tail", float(np.median((st[..., nxt] - st[..., 5 * v + 4]).reshape(-1)))))
        print(f"conv {v} ({'c1' if v % 2 == 0 else 'c2'} stage {v // 2}): " +
              "  ".join(f"{n} {x:7.0f}" for n, x in vals))


if __name__ == "__main__":
    main()
