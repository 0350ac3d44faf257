"""Capture one end-to-end synthesis step (bench.py's workload) in a HIP graph and replay it:
checks capture works (no host sync on the path), that replay output == eager output, and times both."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
import bench  # noqa: E402

dev = torch.device("cuda")
model, gen = bench.build_models(dev, "mixed")
args = bench.make_batch(1234, 32, 12, 512, dev)
with torch.no_grad():
    for _ in range(3):
        ref = bench.step(model, gen, args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        bench.step(model, gen, args)
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / 20
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        bench.step(model, gen, args)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = bench.step(model, gen, args)
    g.replay()
    torch.cuda.synchronize()
    print("replay == eager:", torch.equal(out, ref), float((out - ref).abs().max()))
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / 20
print(f"eager {t_eager * 1e3:.3f} ms/step, graph {t_graph * 1e3:.3f} ms/step")
