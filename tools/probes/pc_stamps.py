"""Per-group timeline of the round-4 C = 128 pair kernel from s_memtime stamps (ablation library:
VO_LIB_PATH=visual_onoma_to_wave_amd/lib/libvonoma_abl.so, pc_cfg 12 = full kernel + stamps,
13 = no DMA + stamps).  Prints, for waves 0 (weight role) and 4 (window role) of workgroups 0-7,
tiles 1-3: each group's MFMA-phase length (group start -> after its MFMAs) and the wait to the next
group's start (group-end vmcnt + barrier), in shader cycles.

    python tools/probes/pc_stamps.py 12 [k d]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from visual_onoma_to_wave_amd import _lib, ops  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 11
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    L = _lib.lib()
    L.vo_tune(b"pc_cfg", cfg)
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
    n = 8 * 2 * 4 * 64 * 2
    buf = (ctypes.c_ulonglong * n)()
    fn = L.vo_pc_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    assert fn(ctypes.cast(buf, ctypes.c_void_p), n) == 0
    s = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(8, 2, 4, 64, 2)
    NG = (4 * k) // 4
    tot = {0: [], 1: []}
    for wg in range(8):
        for role in (0, 1):
            for t in (1, 2):
                st = s[wg, role, t]
                starts = [st[g, 0] for g in range(2 * NG)]
                ends = [st[g, 1] for g in range(2 * NG)]
                nxt = starts[1:] + [st[63, 0]]
                mf = [e - a for a, e in zip(starts, ends)]
                wt = [n_ - e for e, n_ in zip(ends, nxt)]
                span = st[63, 0] - starts[0]
                tot[role].append((mf, wt, span, st[60, 0] - ends[NG - 1], st[60, 1] - st[60, 0],
                                  st[63, 0] - st[61, 0]))
    for role in (0, 1):
        mf = np.array([r[0] for r in tot[role]])
        wt = np.array([r[1] for r in tot[role]])
        span = np.array([r[2] for r in tot[role]])
        print(f"== role {'weight' if role == 0 else 'window'} wave: tile span median {np.median(span):.0f} cycles")
        print("   group:       " + " ".join(f"{g:5d}" for g in range(2 * NG)))
        print("   mfma phase:  " + " ".join(f"{v:5.0f}" for v in np.median(mf, axis=0)))
        print("   wait->next:  " + " ".join(f"{v:5.0f}" for v in np.median(wt, axis=0)))
        print(f"   P1 end->epilogue start {np.median([r[3] for r in tot[role]]):.0f}, "
              f"P1 epilogue {np.median([r[4] for r in tot[role]]):.0f}, "
              f"P2 end->tile end {np.median([r[5] for r in tot[role]]):.0f}")
        print(f"   sum mfma phases {np.median(mf.sum(1)):.0f}, sum waits {np.median(wt.sum(1)):.0f}")


if __name__ == "__main__":
    main()
