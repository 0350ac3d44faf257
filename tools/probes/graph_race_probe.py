"""Diagnose the C4 HIP-graph replay NaN: capture the graphed train step once,
dump the captured graph's topology (node types, roots, leaves, fan-out), then replay it back to
back WITHOUT a host wait and record every step's losses into a device buffer (stream-ordered
copies, one sync at the end).

    python tools/probes/graph_race_probe.py <variant> [steps]
    variant: syncread -- replay only, host wait between the replay and the stream-ordered loss read
             nofence  -- copy batch + LR update + replay, no host wait (the failing pattern)
             static   -- replay only (no inter-replay copy / LR fill)
             fence    -- stream synchronize after every replay (the round-1 workaround)
"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
from helpers import configs, vtts_arrays  # noqa: E402
from weights import load_into  # noqa: E402
from visual_onoma_to_wave_amd import synth  # noqa: E402
from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS  # noqa: E402
from visual_onoma_to_wave_amd.train import GraphedTrainStep  # noqa: E402

TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
         7: "event_record", 8: "sem_signal", 9: "sem_wait", 10: "mem_alloc", 11: "mem_free"}


def topology(graph_handle):
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    g = ctypes.c_void_p(graph_handle)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(ne)) == 0
    src = (ctypes.c_void_p * max(ne.value, 1))()
    dst = (ctypes.c_void_p * max(ne.value, 1))()
    assert hip.hipGraphGetEdges(g, src, dst, ctypes.byref(ne)) == 0
    kinds = collections.Counter()
    tmap = {}
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        kinds[TYPES.get(t.value, t.value)] += 1
        tmap[nd] = TYPES.get(t.value, t.value)
    outd, ind = collections.Counter(), collections.Counter()
    for a, b in zip(src[:ne.value], dst[:ne.value]):
        outd[a] += 1
        ind[b] += 1
    roots = [nd for nd in nodes if ind[nd] == 0]
    leaves = [nd for nd in nodes if outd[nd] == 0]
    fan = [nd for nd in nodes if outd[nd] > 1]
    join = [nd for nd in nodes if ind[nd] > 1]
    print(f"graph: {n.value} nodes, {ne.value} edges, types {dict(kinds)}")
    print(f"  roots {len(roots)} ({collections.Counter(tmap[r] for r in roots)}), "
          f"leaves {len(leaves)} ({collections.Counter(tmap[r] for r in leaves)})")
    print(f"  fan-out nodes {len(fan)} ({collections.Counter(tmap[r] for r in fan)}), join nodes {len(join)}",
          flush=True)


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "nofence"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda")
    pc, mc, tc = configs()
    small = os.environ.get("SMALL") == "1"
    b = synth.acoustic_batch(1234, 8 if small else 32, 12, 256 if small else 512)
    t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
             t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
    torch.manual_seed(0)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision("mixed")
    if os.environ.get("NODROP") == "1":
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        m.postnet.dropout_p = 0.0
        for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
            vp.dropout = 0.0
    opt = ScheduledOptim(m, tc, mc, 0, capturable=True)
    run = GraphedTrainStep(m, opt, FastSpeech2Loss(), warmup=1)
    if os.environ.get("NOOPT") == "1" or os.environ.get("NOCLIP") == "1":
        def body(batch):
            output = m(*(batch[1:]), True)
            losses = FastSpeech2Loss()(batch, output)
            losses[0].backward()
            if os.environ.get("NOCLIP") == "1":
                opt._optimizer.step()
            else:
                params = [p for p in m.parameters() if p.grad is not None]
                torch.nn.utils.clip_grad_norm_(params, 1.0)
            opt._optimizer.zero_grad(set_to_none=True)
            return losses
        run._body = body
    # capture exactly as GraphedTrainStep does, but keep the graph for the topology dump
    run.static = tuple(x.clone() if torch.is_tensor(x) else x for x in batch)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        opt._update_learning_rate()
        run._body(run.static)
    torch.cuda.current_stream().wait_stream(side)
    keep = os.environ.get("NOKEEP") != "1"
    graph = torch.cuda.CUDAGraph(keep_graph=keep)
    with torch.cuda.graph(graph):
        out = run._body(run.static)
    if keep:
        topology(graph.raw_cuda_graph())
        graph.instantiate()
    rec = torch.full((steps, len(out)), float("nan"), device=dev)
    torch.cuda.synchronize()
    for i in range(steps):
        if variant != "static":
            for s, x in zip(run.static, batch):
                if torch.is_tensor(s):
                    s.copy_(x)
            opt._update_learning_rate()
        graph.replay()
        if variant == "syncread":
            torch.cuda.current_stream().synchronize()
        rec[i].copy_(torch.stack([o.detach().float() for o in out]))
        if variant == "fence":
            torch.cuda.current_stream().synchronize()
    torch.cuda.synchronize()
    r = rec.cpu().numpy()
    bad = [i for i in range(steps) if not np.isfinite(r[i]).all()]
    flags = " ".join(f"{k}={os.environ[k]}" for k in ("SMALL", "NODROP", "NOKEEP", "NOOPT", "NOCLIP") if k in os.environ)
    print(f"{variant} [{flags}] (DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'unset')}): "
          f"first non-finite step {bad[0] if bad else None} of {steps}; total loss per step "
          f"{np.round(r[:, 0], 3).tolist()}", flush=True)


if __name__ == "__main__":
    main()
