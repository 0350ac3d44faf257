"""Per-phase timeline of the C = 128 / 64 wave-owned-plane pair (csrc/resblock_rw.hip) from s_memtime stamps.
Diagnostic library built here (never the product one):

    hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -DVO_PRW_STAMPS \
        visual_onoma_to_wave_amd/csrc/resblock_rw.hip visual_onoma_to_wave_amd/csrc/vo_runtime.cpp \
        -o tools/probes/build/libprw_stamps.so
    python tools/probes/prw_stamps.py [k d [variant]]

Prints, for tiles 1-3 of workgroups 0-15 (median over waves and workgroups), shader cycles spent in the
B0 barrier, each P1 tap, the P1 tail (last row tile's epilogue), the B1 barrier, each P2 tap and the P2
tail.  Ideal tap: 64 steps x 2 MFMAs x 16 cycles = 2,048.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from visual_onoma_to_wave_amd import ops  # noqa: E402

NSTW, NSTT, NPT = 16, 4, 28


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    v = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # bit 2: fragment-ordered weights, bit 3: C = 64, bit 4: no acc
    L = ctypes.CDLL(os.environ.get("PRW_LIB", os.path.join(ROOT, "tools/probes/build/libprw_stamps.so")))
    C, B, T = (64, 32, 65536) if v & 8 else (128, 32, 32768)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    w = [ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
         for _ in range(2)]
    if v & 4:
        w = [ops.pack_frag(q) for q in w]
    for _ in range(5):
        ops.resblock_pair(x, w[0], b, w[1], b, k, d, 0.1, out=y, out_scale=1 / 3, acc=y, frag=bool(v & 4))
    torch.cuda.synchronize()
    n = NSTW * 4 * NSTT * NPT
    buf = (ctypes.c_ulonglong * n)()
    P = ctypes.c_void_p
    fn = L.vo_prw_stamps
    fn.argtypes = [P, P, P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    fn.restype = ctypes.c_int
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for _ in range(3):  # warm clocks; keep the last
        assert fn(ptr(x), ptr(w[0]), ptr(b), ptr(w[1]), ptr(b), ptr(y), ptr(y), B, T, k, d, v,
                  ctypes.cast(buf, P)) == 0
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(NSTW, 4, NSTT, NPT)
    st = st[:, :, 1:, :]  # tiles 1-3 (tile 0 carries the prologue)
    K = k
    names = ["B0"] + [f"P1 tap {i}" for i in range(K)] + ["P1 tail", "B1"] + [f"P2 tap {i}" for i in range(K)] + ["P2 tail"]
    idx = [(0, 1)] + [(2 + i, 3 + i) for i in range(K)] + [(2 + K, 3 + K)] + [(3 + K, 4 + K)]  # B0, P1 taps(+tail)
    # P1 tap i: stamp 2+i .. 3+i (tap K-1 ends at 2+K = end of P1 incl. the last epilogue parts)
    idx = [(0, 1)] + [(2 + i, 2 + i + 1) for i in range(K)] + [(2 + K, 3 + K)] + \
          [(K + 4 + i, K + 5 + i) for i in range(K)] + [(2 * K + 3, 2 * K + 4)]
    names = ["B0 barrier"] + [f"P1 tap {i}" for i in range(K)] + ["B1 barrier"] + \
            [f"P2 tap {i}" for i in range(K)] + ["P2 last tap + tail"]
    # (P1 tap K-1's interval ends at stamp 2+K = end of P1, including the last row tile's epilogue parts;
    #  the B1 interval is 2+K .. 3+K; P2 tap i is K+4+i .. K+5+i; the last one ends at 2K+4 = end of P2)
    tot = np.median((st[..., 2 * K + 4] - st[..., 0]).ravel())
    print(f"C={C} k={k} d={d} v={v}: median tile {tot:.0f} cycles (ideal MFMA {2 * K * 2048 * C // 128})")
    for nm, (i0, i1) in zip(names, idx):
        v = (st[..., i1] - st[..., i0]).ravel()
        print(f"  {nm:22s} median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    # from the end of one tile to the next tile's start (the loop back-edge)
    gap = (st[:, :, 1:, 0] - st[:, :, :-1, 2 * K + 4]).ravel()
    print(f"  {'back-edge':22s} median {np.median(gap):8.0f}")


if __name__ == "__main__":
    main()
