"""Locate the first non-finite value of a graph-replayed C4 forward+backward (see
graph_race_probe.py): capture fwd + loss + backward once, replay once, and compare the forward
outputs, the losses and every parameter gradient with the same segment run eagerly.

    python tools/probes/graph_nan_locate.py [mixed|fp32] [B] [T]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden"),
                os.path.dirname(os.path.abspath(__file__))]
from graph_bisect_probe import model_and_batch, rel  # noqa: E402
from visual_onoma_to_wave_amd.model import FastSpeech2Loss  # noqa: E402

NAMES = ["mel", "postnet_mel", "e_pred", "k_pred", "log_d_pred", "d_rounded", "src_masks", "mel_masks",
         "src_lens", "mel_lens"]


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    m, batch, _ = model_and_batch(prec)
    lossf = FastSpeech2Loss()
    names = [n for n, p in m.named_parameters()]
    bufs = {k: v.clone() for k, v in m.named_buffers()}

    def restore():
        for k, v in m.named_buffers():
            v.copy_(bufs[k])

    def body():
        for p in m.parameters():
            p.grad = None
        out = m(*(batch[1:]), True)
        losses = lossf(batch, out)
        losses[0].backward()
        outs = [o for o in out if torch.is_tensor(o)]
        return outs, list(losses), [p.grad for p in m.parameters()]

    restore()
    ro, rl, rg = body()
    ro = [o.detach().clone() for o in ro]
    rl = [x.detach().clone() for x in rl]
    rg = [None if g is None else g.clone() for g in rg]
    restore()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream().wait_stream(side)
    restore()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        go, gl, gg = body()
    restore()
    g.replay()
    torch.cuda.synchronize()
    print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "unset"), prec)
    for n, a, b in zip([n for n in NAMES], go, ro):
        fin = bool(torch.isfinite(a.float()).all()) if a.is_floating_point() else True
        e = rel(a.float(), b.float()) if a.is_floating_point() else float((a != b).sum())
        print(f"  out {n:12s} finite {fin} err {e:.3e}")
    for i, (a, b) in enumerate(zip(gl, rl)):
        print(f"  loss[{i}] graph {float(a):.6f} eager {float(b):.6f}")
    bad = []
    for n, a, b in zip(names, gg, rg):
        if a is None or b is None:
            continue
        e = rel(a, b)
        if not (e < 1e-2):
            bad.append((n, e))
    print(f"  grads: {len(bad)} differ > 1e-2 / non-finite: {bad[:12]}", flush=True)


if __name__ == "__main__":
    main()
