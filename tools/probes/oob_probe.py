"""Out-of-bounds write detector for the HIP ops: every tensor the op wrappers allocate
(``torch.empty`` / ``zeros`` / ``*_like`` inside ops.py, gan_ops.py, hifigan/models.py) is placed
between two 1 MiB canary bands; after a C4 train step, a C5 GAN step and an inference pass the
bands are checked.  A kernel writing past its output (or workspace) shows up with the Python
stack of the allocation.

    python tools/probes/oob_probe.py
"""
import math
import os
import sys
import traceback

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden"),
                os.path.dirname(os.path.abspath(__file__))]

G = 1 << 20
PAT = 0xA5


class Guarded:
    def __init__(self):
        self.allocs = []

    def _alloc(self, shape, dtype, device, zero):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
            shape = tuple(shape[0])
        shape = tuple(int(s) for s in shape)
        dtype = dtype or torch.float32
        esz = torch.empty((), dtype=dtype).element_size()
        n = math.prod(shape) * esz
        raw = torch.empty(G + n + G, dtype=torch.uint8, device=device)
        raw.fill_(PAT)
        view = raw[G:G + n].view(dtype).view(shape)
        if zero:
            view.zero_()
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                            for f in reversed(traceback.extract_stack(limit=5)[:-2]))
        self.allocs.append((raw, n, shape, dtype, where))
        return view

    def empty(self, *shape, dtype=None, device=None, **kw):
        return self._alloc(shape, dtype, device, False)

    def zeros(self, *shape, dtype=None, device=None, **kw):
        return self._alloc(shape, dtype, device, True)

    def empty_like(self, t, dtype=None, device=None, **kw):
        return self._alloc(tuple(t.shape), dtype or t.dtype, device or t.device, False)

    def zeros_like(self, t, dtype=None, device=None, **kw):
        return self._alloc(tuple(t.shape), dtype or t.dtype, device or t.device, True)

    def check(self, what):
        torch.cuda.synchronize()
        bad = []
        for raw, n, shape, dtype, where in self.allocs:
            lo = raw[:G] != PAT
            hi = raw[G + n:] != PAT
            if bool(lo.any()) or bool(hi.any()):
                lo_i = torch.nonzero(lo).flatten()
                hi_i = torch.nonzero(hi).flatten()
                bad.append((shape, dtype, where, (G - int(lo_i.min())) if lo_i.numel() else 0,
                            int(hi_i.max()) + 1 if hi_i.numel() else 0, int(lo_i.numel()), int(hi_i.numel())))
        print(f"{what}: {len(self.allocs)} guarded allocations, {len(bad)} with canary damage", flush=True)
        for shape, dtype, where, before, after, nlo, nhi in bad[:20]:
            print(f"   {shape} {dtype}: {nlo} bytes hit up to {before} B before, {nhi} bytes up to {after} B after; "
                  f"allocated at {where}", flush=True)
        self.allocs = []


class Shim:
    def __init__(self, g):
        self._g = g

    def __getattr__(self, name):
        if name in ("empty", "zeros", "empty_like", "zeros_like"):
            return getattr(self._g, name)
        return getattr(torch, name)


def main():
    from helpers import configs, hifigan_arrays, hifigan_h, vtts_arrays
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan, ops, synth
    from visual_onoma_to_wave_amd.hifigan import gan_ops
    from visual_onoma_to_wave_amd.hifigan import models as hmodels
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    g = Guarded()
    shim = Shim(g)
    for mod in (ops, gan_ops, hmodels):
        mod.torch = shim
    dev = torch.device("cuda")
    pc, mc, tc = configs()
    for prec, B, T in (("mixed", 8, 256), ("fp32", 3, 77), ("mixed", 32, 512)):
        b = synth.acoustic_batch(1234, B, 12, T, ragged=True)
        t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
        batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
                 t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
        m = vTTS(pc, mc, tc)
        load_into(m, vtts_arrays())
        m = m.to(dev).train().set_precision(prec)
        out = m(*(batch[1:]), True)
        losses = FastSpeech2Loss()(batch, out)
        losses[0].backward()
        g.check(f"C4 train fwd+bwd {prec} B={B} T={T}")
        m.eval()
        with torch.no_grad():
            out = m(*(batch[1:]), True)
        g.check(f"vTTS inference {prec} B={B} T={T}")
    gen = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(gen, hifigan_arrays())
    gen = gen.to(dev)
    gen_inf = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(gen_inf, hifigan_arrays())
    gen_inf.eval()
    gen_inf.remove_weight_norm()
    gen_inf = gen_inf.to(dev)
    for B, T in ((2, 37), (4, 512)):
        mel = torch.randn(B, 80, T, device=dev)
        with torch.no_grad():
            gen_inf(mel)
        g.check(f"Generator inference B={B} T={T}")
    from visual_onoma_to_wave_amd.hifigan.train import HifiGanTrainer
    h = hifigan.AttrDict(hifigan_h())
    tr = HifiGanTrainer(gen, h, device=dev)
    tr.set_compute_dtype(torch.bfloat16)
    x = torch.randn(4, 32, 80, device=dev)
    y = torch.randn(4, 8192, device=dev).clamp(-1, 1) * 0.3
    tr.step(x, y)
    g.check("C5 GAN step B=4")


if __name__ == "__main__":
    main()
