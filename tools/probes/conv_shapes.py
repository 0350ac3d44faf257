"""Per-call conv (forward / input-gradient) shapes and times in an eager C4 or C5 step (A/B input for the conv tiles):
wraps ops.conv1d with an event pair per call (synchronised: eager, not the graphed step's clock) and
prints the calls grouped by shape, sorted by time per step.

  python tools/probes/wgrad_shapes.py train|gan [VO_TUNE knobs via the environment]
"""

import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import bench  # noqa: E402
from visual_onoma_to_wave_amd import ops  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "gan"
STEPS = 2
sys.argv = ["bench.py", "--mode", mode, "--no-graph", "--steps", str(STEPS), "--warmup", "1", "--cpu-seconds", "0"]
a = bench.parse()
a.ranks_seen = [0]
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)

calls = collections.defaultdict(lambda: [0, 0.0])
orig = ops.conv1d
active = [False]


def wrapped(x, w_packed, bias, **kw):
    if not active[0]:
        return orig(x, w_packed, bias, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = orig(x, w_packed, bias, **kw)
    e1.record()
    e1.synchronize()
    key = (str(x.dtype).replace("torch.", ""), tuple(x.shape), kw.get("Co"), kw.get("K"), kw.get("stride", 1),
           kw.get("groups", 1), kw.get("dil", 1), kw.get("transposed") is not None, kw.get("variant", 0),
           bias is not None, kw.get("res1") is not None, kw.get("ymask") is not None)
    calls[key][0] += 1
    calls[key][1] += e0.elapsed_time(e1) * 1e3
    return r


ops.conv1d = wrapped
orig_timed = bench.timed


def timed(fn, steps, dist):
    active[0] = True
    try:
        return orig_timed(fn, steps, dist)
    finally:
        active[0] = False


bench.timed = timed
(bench.run_gan if mode == "gan" else bench.run_train)(a, dev, 0, 1, None)
tot = sum(v[1] for v in calls.values()) / STEPS
print(f"{mode}: conv1d {sum(v[0] for v in calls.values()) / STEPS:.0f} calls, {tot:.0f} us per step (eager, synced)")
print("  us/step  calls/step   us/call  dtype x-shape Co K stride groups dil transposed variant bias res1 ymask")
for k, (n, us) in sorted(calls.items(), key=lambda kv: -kv[1][1]):
    print(f"{us / STEPS:9.1f} {n / STEPS:9.1f} {us / n:9.1f}  {k}")
