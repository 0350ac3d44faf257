"""Shared test helpers: golden fixtures and deterministic weights."""

import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
REPO = os.path.dirname(HERE)
DATA = os.path.join(REPO, "visual_onoma_to_wave_amd", "data")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


def spec(which):
    with open(os.path.join(GOLDEN, which + "_spec.json")) as f:
        d = json.load(f)
    return d["seed"], [(k, tuple(s), t) for k, s, t in d["spec"]]


def vtts_arrays():
    from weights import make_state_dict
    seed, sp = spec("vtts")
    return make_state_dict(sp, seed)


def hifigan_arrays():
    from weights import HIFIGAN_UPS_STRIDES, make_state_dict
    seed, sp = spec("hifigan")
    return make_state_dict(sp, seed, HIFIGAN_UPS_STRIDES)


def stats():
    with open(os.path.join(DATA, "stats.json")) as f:
        return json.load(f)


def hifigan_h():
    with open(os.path.join(DATA, "hifigan_config.json")) as f:
        return json.load(f)


def configs():
    """(preprocess, model, train) config dicts pointing at the packaged metadata."""
    import yaml
    out = []
    for n in ("preprocess", "model", "train"):
        with open(os.path.join(DATA, "config", "ICASSP", n + ".yaml")) as f:
            out.append(yaml.load(f, Loader=yaml.SafeLoader))
    out[0]["path"]["preprocessed"] = DATA
    return tuple(out)


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def t(x):
    return torch.from_numpy(np.array(x))


def bf16_bar(ref_fp32, ref_bf16, floor=1e-2, slack=1.0):
    """Tolerance of a bf16 HIP result: the survey's rel-L2 1e-2, or -- where the reference's own
    bf16 autocast on the same weights and input drifts further from its fp32 result (the
    deterministic test weights of weights.py drive the vocoder harder than 1e-2 allows any bf16
    implementation) -- that drift, no slack: no worse than the reference run in bf16."""
    return max(floor, slack * rel_l2(ref_bf16, ref_fp32))


def bf16_grad_check(got, ref, bfs, floor=1e-2, sibling=None, discontinuous=False):
    """The bf16 gradient bar shared by the C4 / C5 step tests.  got / ref: {name: gradient} of the HIP
    path and the fp32 oracle; bfs: the same from the oracle's bf16 arithmetics (oracle/bf16.py:
    autocast and bf16 operands).  Per parameter the oracle's drift D_k = max over bfs of rel-L2(bf, ref).
    * D_k <= floor (signal-dominated): rel-L2(got_k, ref_k) <= floor, per parameter;
    * D_k > floor: the gradient is dominated by the forward's bf16 rounding (L1-loss sign flips,
      BatchNorm batch statistics, cancelling sums) -- two bf16 evaluations are two independent noise
      draws and a per-parameter comparison of one draw with another is a coin toss; over that group,
      RMS_k rel-L2(got_k, ref_k) <= RMS_k D_k (no noisier than the reference's own bf16 arithmetic);
    * discontinuous: every gradient of the set flows through the sign of an L1 term (the HiFi-GAN
      generator: mel and feature-matching losses), so all of them are in the noise-dominated group;
    * sibling(name) -> name of a parameter setting the scale of a structurally-zero gradient:
      ||got_k|| <= max(floor * ||ref_sibling||, the oracle's bf16 ||bf_k||).
    Returns (rows, summary) for printing; asserts."""
    rows, bad, noise_e, noise_d = [], [], [], []
    for k, r in ref.items():
        if k not in got:
            continue
        a = got[k].float()
        sib = sibling(k) if sibling else None
        if sib is not None:  # its scale: floor x the sibling's gradient, or the oracle's own bf16 noise on it
            lim = max([floor * float(ref[sib].norm())] + [float(b[k].norm()) for b in bfs])
            if float(a.norm()) > lim:
                bad.append((k, "structural zero", float(a.norm()), lim))
            continue
        e = rel_l2(a, r)
        d = max(rel_l2(b[k], r) for b in bfs)
        rows.append((e / max(d, floor), k, e, d))
        if d <= floor and not discontinuous:
            if e > floor:
                bad.append((k, e, floor))
        else:
            noise_e.append(e)
            noise_d.append(d)
    rms = lambda v: float(np.sqrt(np.mean(np.square(v)))) if v else 0.0  # noqa: E731
    summary = (len(rows), len(noise_e), rms(noise_e), rms(noise_d))
    assert not bad, bad[:10]
    assert rms(noise_e) <= rms(noise_d), ("noise-dominated group", summary)
    return rows, summary


def oracle_generator_bf16(gsd, mel, h):
    """The oracle Generator under CPU bf16 autocast (the reference's arithmetic in bf16)."""
    import torch
    from oracle import vocoder as V
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        return V.generator(gsd, mel, h).float()
