"""Per-call device time of the C4 training step's HIP weight-gradient and conv launches and of
the PyTorch-side attention backward (eager step, HIP events around each call on the current
stream).  Usage: python tools/probes/train_calls.py"""
import collections
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    sys.path.insert(0, p)
from helpers import configs, vtts_arrays  # noqa: E402
from weights import load_into  # noqa: E402
from visual_onoma_to_wave_amd import autograd as AG, ops, synth  # noqa: E402
from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS  # noqa: E402
from visual_onoma_to_wave_amd.train import train_step  # noqa: E402

REC = collections.defaultdict(lambda: [0, 0.0])
ACTIVE = [False]


def timed(name_fn, fn):
    def w(*a, **k):
        if not ACTIVE[0]:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(*a, **k)
        e1.record()
        e1.synchronize()
        key = name_fn(*a, **k)
        REC[key][0] += 1
        REC[key][1] += e0.elapsed_time(e1) * 1e3
        return r
    return w


ops.conv1d_wgrad = timed(lambda gy, x, K, **k: f"wgrad {x.dtype} rows={x.shape[0]*x.shape[1]} Ci={x.shape[2]} "
                         f"Co={gy.shape[2]} K={K}", ops.conv1d_wgrad)
_ab = AG.AttentionFn.backward
AG.AttentionFn.backward = staticmethod(timed(lambda ctx, go: f"attn_bwd {go.dtype} {tuple(go.shape)}", _ab))
_lb = AG.LayerNormFn.backward
AG.LayerNormFn.backward = staticmethod(timed(lambda ctx, gy: f"ln_bwd {gy.dtype} {tuple(gy.shape)}", _lb))
_lr = AG.LengthRegulateFn.backward
AG.LengthRegulateFn.backward = staticmethod(timed(lambda ctx, go, g2: f"lr_bwd {tuple(go.shape)}", _lr))

dev = torch.device("cuda:0")
pc, mc, tc = configs()
m = vTTS(pc, mc, tc)
load_into(m, vtts_arrays())
m = m.to(dev).train().set_precision("mixed")
opt = ScheduledOptim(m, tc, mc, 0)
b = synth.acoustic_batch(1234, 32, 12, 512)
t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
         t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
for _ in range(3):
    train_step(m, opt, FastSpeech2Loss(), batch)
torch.cuda.synchronize()
ACTIVE[0] = True
train_step(m, opt, FastSpeech2Loss(), batch)
torch.cuda.synchronize()
tot = 0.0
for k, (n, us) in sorted(REC.items(), key=lambda kv: -kv[1][1]):
    tot += us
    print(f"{us:9.1f} us  {n:3d} calls  {us / n:8.1f} us/call  {k}")
print(f"total {tot:.1f} us")
