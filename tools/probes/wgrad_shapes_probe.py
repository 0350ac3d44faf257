"""Per-call time of every weight-gradient launch in one eager C5 (HiFi-GAN) training step:
ops.conv1d_wgrad wrapped with synchronising HIP events; prints (calls, total ms) per shape."""
import os
import sys
from collections import defaultdict

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    from visual_onoma_to_wave_amd import ops
    import bench
    stats = defaultdict(lambda: [0, 0.0])
    orig = ops.conv1d_wgrad

    def timed(a, b, K, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = orig(a, b, K, **kw)
        e.record()
        e.synchronize()
        key = (tuple(a.shape), tuple(b.shape), K, kw.get("S", 1), kw.get("groups", 1), bool(kw.get("transposed")))
        stats[key][0] += 1
        stats[key][1] += s.elapsed_time(e)
        return r
    sys.argv = ["bench.py", "--mode", "gan", "--steps", "1", "--warmup", "1", "--no-graph", "--cpu-seconds", "0"]
    ops.conv1d_wgrad = timed
    a = bench.parse()
    a.ranks_seen = [0]
    dev = torch.device("cuda")
    bench.bench_gan(a, dev, 0, 1, None)
    tot = sum(v[1] for v in stats.values())
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{v[1]:8.3f} ms  {v[0]:3d} calls  A{k[0]} B{k[1]} K={k[2]} S={k[3]} g={k[4]} tr={k[5]}")
    print(f"total {tot:.2f} ms over {sum(v[0] for v in stats.values())} calls (warm-up + 1 step)")


if __name__ == "__main__":
    main()
