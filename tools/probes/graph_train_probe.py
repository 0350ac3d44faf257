"""Per-step losses of the C4 train step, eager vs HIP-graph replay (mixed precision, dropout on)."""
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
from visual_onoma_to_wave_amd.train import GraphedTrainStep, train_step  # noqa: E402

dev = torch.device("cuda")
prec = sys.argv[1] if len(sys.argv) > 1 else "mixed"
pc, mc, tc = configs()
b = synth.acoustic_batch(1234, 32, 12, 512)
t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
         t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
for graphed in (False, True):
    torch.manual_seed(0)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision(prec)
    opt = ScheduledOptim(m, tc, mc, 0, capturable=graphed)
    run = GraphedTrainStep(m, opt, FastSpeech2Loss(), warmup=int(os.environ.get("GW", "3"))) if graphed else (
        lambda bt: train_step(m, opt, FastSpeech2Loss(), bt))
    out = []
    nsync = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for i in range(16):
        losses = run(batch)
        if nsync:
            torch.cuda.synchronize()
            out.append(round(float(losses[0].detach()), 4))
    torch.cuda.synchronize()
    out.append(round(float(losses[0].detach()), 4))
    print("graphed" if graphed else "eager  ", out, flush=True)
