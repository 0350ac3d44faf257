"""Per-slice timeline of the register-streamed C = 128 pair (resblock_rs.hip) from s_memtime stamps:
ablation library, pair_cfg 72 + rs_cfg 9.  Prints the median slice duration per phase and slice index
over workgroups 0-7, tiles 1-2 (wave 0), in shader cycles (ideal: 48 MFMAs x 16 = 768).

    VO_LIB_PATH=visual_onoma_to_wave_amd/lib/libvonoma_abl.so python tools/probes/rs_stamps.py [k d]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    L = _lib.lib()
    L.vo_tune(b"pair_cfg", 72)
    L.vo_tune(b"rs_cfg", 9)
    C, B, T = 128, 32, 32768
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    w = [ops.pack_conv_weight(torch.randn(C, C, k, device="cuda", generator=g) / (C * k) ** 0.5, torch.bfloat16)
         for _ in range(2)]
    for _ in range(5):
        ops.resblock_pair(x, w[0], b, w[1], b, k, d, 0.1, out=y, out_scale=1 / 3, acc=y)
    torch.cuda.synchronize()
    n = 8 * 2 * 2 * 64
    buf = (ctypes.c_ulonglong * n)()
    fn = L.vo_rs_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    assert fn(ctypes.cast(buf, ctypes.c_void_p), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(8, 2, 2, 64)
    NS = 4 * k
    d1 = st[:, :, 0, 1:NS] - st[:, :, 0, :NS - 1]          # P1 slice durations (slices 0..NS-2)
    d2 = st[:, :, 1, 1:NS] - st[:, :, 1, :NS - 1]
    p1_tail = st[:, :, 1, 0] - st[:, :, 0, NS - 1]           # last P1 slice + epilogue
    p2_tail = st[:, :, 1, 63] - st[:, :, 1, NS - 1]          # last P2 slice + y epilogue
    span = st[:, :, 1, 63] - st[:, :, 0, 0]
    print(f"tile span median {np.median(span):.0f} cycles; ideal MFMA {2 * NS * 768}")
    print("P1 slice durations (median over wg/tiles):", " ".join(f"{v:.0f}" for v in np.median(d1.reshape(-1, NS - 1), 0)))
    print("P2 slice durations:", " ".join(f"{v:.0f}" for v in np.median(d2.reshape(-1, NS - 1), 0)))
    print(f"last P1 slice + P1 epilogue {np.median(p1_tail):.0f}, last P2 slice + y epilogue {np.median(p2_tail):.0f}")


if __name__ == "__main__":
    main()
