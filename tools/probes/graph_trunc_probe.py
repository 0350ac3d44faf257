"""Truncation bisection of the C4 graph-replay failure.  For each body (fwd | fwd+bwd |
fwd+bwd+clip | fwd+bwd+adam | full step), capture once and replay 4 times; per replay record the
total loss read stream-ordered right after the replay (no host wait) and again after a host
synchronize.  Stale = the two reads differ; NaN = the synced read is not finite.

    python tools/probes/graph_trunc_probe.py [mixed|fp32]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden"),
                os.path.dirname(os.path.abspath(__file__))]
from graph_bisect_probe import model_and_batch  # noqa: E402
from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim  # noqa: E402


def run(kind, prec):
    m, batch, (pc, mc, tc) = model_and_batch(prec)
    opt = ScheduledOptim(m, tc, mc, 0, capturable=True)
    opt._update_learning_rate()
    lossf = FastSpeech2Loss()

    def body():
        out = m(*(batch[1:]), True)
        losses = lossf(batch, out)
        if kind == "fwd":
            return losses[0].detach()
        losses[0].backward()
        params = [p for p in m.parameters() if p.grad is not None]
        if kind in ("clip", "full"):
            torch.nn.utils.clip_grad_norm_(params, 1.0)
        if kind in ("adam", "full"):
            opt._optimizer.step()
        opt._optimizer.zero_grad(set_to_none=True)
        return losses[0].detach()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = body()
    early, late = [], []
    for _ in range(4):
        g.replay()
        early.append(out.clone())
        torch.cuda.synchronize()
        late.append(float(out))
    early = [float(e) for e in early]
    stale = sum(1 for a, b in zip(early, late) if a != b)
    nan = sum(1 for b in late if b != b)
    print(f"{kind:5s} {prec}: stale reads {stale}/4, non-finite {nan}/4; early {early} late {late}", flush=True)


if __name__ == "__main__":
    prec = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "unset"))
    for kind in sys.argv[2:] or ["fwd", "bwd", "clip", "adam", "full"]:
        run(kind, prec)
