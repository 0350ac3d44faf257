"""Minimal check of stream ordering after a HIP-graph replay: capture a chain of N small kernels
whose last one writes `out`, replay it, and read `out` with an ordinary stream-ordered kernel right
after (no host wait).  If the runtime lets that kernel start before the graph has finished, the
read sees the previous contents.

    python tools/probes/graph_order_probe.py [n_kernels] [kernels|memset|memcpy]
"""
import os
import sys

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda")
    x = torch.zeros(1 << 20, device=dev)
    seed = torch.zeros((), device=dev)

    mode = sys.argv[2] if len(sys.argv) > 2 else "kernels"
    lst = [torch.zeros(1000 + 7 * i, device=dev) for i in range(300)]  # multi-tensor-apply operands

    def chain():
        y = x + seed
        for _ in range(n):
            if mode == "memset":       # zero-fill node + accumulate kernel
                z = torch.zeros_like(y)
                z.add_(y)
                y = z
            elif mode == "memcpy":     # device-to-device copy node
                y = y.clone()
            elif mode == "foreach":    # multi-tensor-apply kernels (~4 KB kernel-argument blocks)
                torch._foreach_add_(lst, 1.0)
            y = y * 1.0 + 1.0
        return y

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        chain()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = chain()
    reads = []
    for i in range(8):
        seed.fill_(1000.0 * (i + 1))     # stream-ordered input change
        g.replay()
        reads.append(out[:4].clone())    # stream-ordered read right after the replay
    torch.cuda.synchronize()
    if mode == "foreach":
        sums = sorted(set(float(t.min()) for t in lst) | set(float(t.max()) for t in lst))
        print(f"  foreach operands after warm-up + 8 replays: distinct values {sums[:6]} (want {float(9 * n)})")
    got = [float(r[0]) for r in reads]
    want = [1000.0 * (i + 1) + n for i in range(8)]
    bad = sum(1 for a, b in zip(got, want) if a != b)
    print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'unset')} "
          f"n={n} {mode}: {bad}/8 stream-ordered reads after replay saw stale data; got {got} want {want}", flush=True)


if __name__ == "__main__":
    main()
