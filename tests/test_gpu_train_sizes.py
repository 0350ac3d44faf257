"""Training configs at their stated sizes (BASELINE.json C4 / C5) and the GAN trainer's
data-parallel paths on the GPU.

* C4 (``scripts/04_train.py:128-141``): one step at B = 32 utterances, T_src = 12, teacher-forced
  T_mel = 512, fp32 mode: the six FastSpeech2Loss terms and a fixed subset of
  parameter gradients against the CPU oracle's autograd on the same batch.
  Tolerances as test_gpu_train.py: losses rel <= 1e-4, gradients rel-L2 <= 2e-3.
* C5 (HiFi-GAN V1, ``scripts/hifigan/config.json`` batch 16, segment 8192): trainer steps at
  batch 16 in bf16 are finite, and HIP-graph replays equal the eager steps bit for bit.
* ``HifiGanTrainer(distributed=True)`` with two ranks (gloo, CUDA tensors, both on cuda:0): the
  bucket-averaged D and G gradients equal the gradients of one process on the global batch.
* ``HifiGanTrainer(distributed=True, graphed=True)`` on RCCL at world size 1 (fp32 and bf16 on the
  wire): the graph with the captured bucketed all-reduces equals the eager steps bit for bit.
Parity of the HiFi-GAN training side is unpinned (the reference has no training code).
"""

import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import bf16_grad_check, configs, hifigan_arrays, hifigan_h, rel_l2, stats, vtts_arrays
from weights import load_into

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# ------------------------------------------------------------------------------------------- C4

def _c4_batch(dev, seed=4321, B=32, T_src=12, T_mel=512):
    from visual_onoma_to_wave_amd import synth
    b = synth.acoustic_batch(seed, B, T_src, T_mel, ragged=True)
    t = lambda k: torch.from_numpy(np.asarray(b[k])).to(dev)  # noqa: E731
    return (None, t("audiotypes"), t("texts"), t("src_lens"), b["max_src_len"], t("mels"), t("mel_lens"),
            b["max_mel_len"], t("e_targets"), None, t("d_targets"), t("images"), None)


def test_c4_step_full_size_vs_oracle(device):
    from oracle import acoustic as A
    from oracle import training as TR
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    arrays = vtts_arrays()
    m = vTTS(*configs())
    load_into(m, arrays)
    m = m.to(device).train().set_precision("fp32")
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0
    batch = _c4_batch(device)
    assert batch[5].shape == (32, 512, 80) and int(batch[3].max()) == 12
    out = m(*(batch[1:]), True)
    losses = FastSpeech2Loss()(batch, out)
    losses[0].backward()
    got = [float(x) for x in losses]

    torch.set_num_threads(16)
    sd = A.complete_state_dict(arrays, stats()["energy"])
    for k, v in sd.items():
        if v.dtype == torch.float32 and "position_enc" not in k and "bins" not in k and "running" not in k:
            v.requires_grad_(True)
    bc = _c4_batch("cpu")
    ro = A.vtts_forward(sd, *bc[1:12], energy_stats=stats()["energy"], training=True)
    ref = TR.fastspeech2_loss(bc, ro)
    ref[0].backward()
    np.testing.assert_allclose(got, [float(x) for x in ref], rtol=1e-4, atol=1e-6)

    named = dict(m.named_parameters())
    keys = sorted(k for k, v in sd.items() if v.grad is not None and k in named and named[k].grad is not None)
    subset = keys[::5] + [k for k in keys if any(s in k for s in (
        "decoder.layer_stack.5.pos_ffn.w_1", "decoder.layer_stack.0.slf_attn.w_qs", "postnet.convolutions.0",
        "VisualFeatureExtractor.bridge", "energy_predictor.linear_layer", "mel_linear"))]
    bad = []
    for k in sorted(set(subset)):
        gr, p = sd[k].grad, named[k].grad.cpu()
        err = float((p - gr).norm())
        if err > 2e-3 * float(gr.norm()) + 1e-5:
            bad.append((k, err, float(gr.norm())))
    assert not bad, bad[:10]
    assert len(set(subset)) > 50


def _c4_oracle(arrays, bc, bf16_back):
    """(six loss values, {parameter: gradient}) of one oracle step on the CPU; bf16_back: the decoder,
    mel_linear and PostNet under CPU bf16 autocast (the precision split of the HIP "mixed" mode)."""
    from oracle import acoustic as A
    from oracle import training as TR
    sd = A.complete_state_dict(arrays, stats()["energy"])
    for k, v in sd.items():
        if v.dtype == torch.float32 and "position_enc" not in k and "bins" not in k and "running" not in k:
            v.requires_grad_(True)
    ro = A.vtts_forward(sd, *bc[1:12], energy_stats=stats()["energy"], training=True, bf16_back=bf16_back)
    ref = TR.fastspeech2_loss(bc, ro)
    ref[0].backward()
    return [float(x) for x in ref], {k: v.grad for k, v in sd.items() if v.grad is not None}


# gradients that are exactly zero in exact arithmetic (rounding noise on every side), with the sibling
# whose gradient sets their scale: conv biases feeding a train-mode BatchNorm (its beta), and the key
# projection's bias (softmax is invariant to a per-query constant: the query bias of the same layer)
_STRUCTURAL_ZEROS = [(re.compile(r"(.*VisualFeatureExtractor\.embedder\.)([036])\.bias$"),
                      lambda m: f"{m.group(1)}{int(m.group(2)) + 1}.bias"),
                     (re.compile(r"(postnet\.convolutions\.\d+\.)0\.conv\.bias$"), lambda m: f"{m.group(1)}1.bias"),
                     (re.compile(r"(.*slf_attn\.)w_ks\.bias$"), lambda m: f"{m.group(1)}w_qs.bias")]


def _zero_sibling(k):
    for rx, fn in _STRUCTURAL_ZEROS:
        m = rx.match(k)
        if m:
            return fn(m)
    return None


def test_c4_step_mixed_full_size_vs_oracle(device):
    """The bench's C4 precision ("mixed": encoder and variance adaptor fp32, decoder / mel_linear /
    PostNet bf16 -- attention backward v2, step-batched packs, vectorised BatchNorm all on this path)
    at B = 32, T_src = 12, T_mel = 512: the six losses and EVERY parameter gradient against the fp32
    oracle, at the bar of the oracle's own bf16 arithmetic on the same batch and precision split
    (bf16_grad_check; losses per value within max(1e-2, that drift))."""
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    arrays = vtts_arrays()
    m = vTTS(*configs())
    load_into(m, arrays)
    m = m.to(device).train().set_precision("mixed")
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0
    batch = _c4_batch(device)
    out = m(*(batch[1:]), True)
    losses = FastSpeech2Loss()(batch, out)
    losses[0].backward()
    got = [float(x) for x in losses]

    torch.set_num_threads(16)
    bc = _c4_batch("cpu")
    ref, ref_g = _c4_oracle(arrays, bc, False)
    bf = [_c4_oracle(arrays, bc, mode) for mode in ("autocast", "operands")]
    for i, (a, r) in enumerate(zip(got, ref)):
        drift = max(abs(b[0][i] - r) for b in bf)
        assert abs(a - r) <= max(1e-2 * abs(r), drift) + 1e-6, ("loss", i, a, r, drift)

    named = dict(m.named_parameters())
    ours = {k: p.grad.cpu() for k, p in named.items() if p.grad is not None}
    rows, (n, n_noise, rms_e, rms_d) = bf16_grad_check(ours, ref_g, [b[1] for b in bf], sibling=_zero_sibling)
    rows.sort(reverse=True)
    print(f"C4 mixed: {n} gradients; signal-dominated worst error / 1e-2: "
          f"{max(e for _, _, e, d in rows if d <= 1e-2) / 1e-2:.3f}; noise-dominated group of {n_noise}: "
          f"RMS error {rms_e:.3e} vs the oracle's bf16 drift {rms_d:.3e}")
    for row in rows[:8]:
        print("  %.3f %-60s ours %.2e oracle-bf16 %.2e" % row)
    assert n > 180  # every parameter with a gradient but the 13 structural zeros


# ------------------------------------------------------------------------------------------- C5

def _gen(device):
    from visual_onoma_to_wave_amd import hifigan
    g = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(g, hifigan_arrays())
    return g.to(device)


def _c5_batch(B, seed=11):
    gen = torch.Generator().manual_seed(seed)
    t = torch.arange(8192, dtype=torch.float32) / 22050.0
    f0 = 110.0 + 330.0 * torch.rand(B, 1, generator=gen)
    y = (0.3 * torch.sin(2 * np.pi * f0 * t) + 0.05 * torch.randn(B, 8192, generator=gen)).clamp(-1, 1)
    mel = torch.randn(B, 32, 80, generator=gen) - 4.0
    return mel.cuda(), y.cuda()


def test_c5_trainer_batch16_graphed_matches_eager():
    """config.json batch 16 x segment 8192, bf16 compute (the bench's C5 step): three eager steps
    twice (deterministic) and three graph replays from the same state, bit for bit."""
    from visual_onoma_to_wave_amd import hifigan
    h = hifigan.AttrDict(hifigan_h())
    assert h.batch_size == 16 and h.segment_size == 8192
    mel, y = _c5_batch(16)
    finals = []
    for graphed in (False, False, True):
        torch.manual_seed(1234)
        g = _gen("cuda")
        tr = hifigan.HifiGanTrainer(g, h, graphed=graphed, capturable=True).set_compute_dtype(torch.bfloat16)
        for _ in range(3):
            losses = tr.step_graphed(mel, y, warmup=1) if graphed else tr.step(mel, y)
        torch.cuda.synchronize()
        finals.append(({k: float(v) for k, v in losses.items()},
                       torch.cat([p.detach().flatten().cpu() for p in g.parameters()]),
                       torch.cat([p.detach().flatten().cpu() for p in tr.msd.parameters()])))
    (le, ge, de), (l1, g1, d1), (lg, gg, dg) = finals
    assert all(np.isfinite(v) for v in le.values())
    assert torch.equal(g1, ge) and torch.equal(d1, de) and l1 == le, "eager C5 step is not deterministic"
    assert torch.equal(gg, ge) and torch.equal(dg, de) and lg == le, "graph replay differs from the eager steps"


def _grads(tr):
    d = [p.grad.detach().flatten().cpu().clone() for p in list(tr.mpd.parameters()) + list(tr.msd.parameters())
         if p.grad is not None]
    g = [p.grad.detach().flatten().cpu().clone() for p in tr.generator.parameters() if p.grad is not None]
    return torch.cat(d), torch.cat(g)


def _gan_gloo_worker(rank, world, port, out):
    import torch.distributed as dist
    from visual_onoma_to_wave_amd import hifigan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    h = hifigan.AttrDict(dict(hifigan_h(), learning_rate=0.0))  # lr 0: D is unchanged for the G step
    torch.manual_seed(1234)
    tr = hifigan.HifiGanTrainer(_gen("cuda"), h, distributed=True, device=torch.device("cuda", 0))
    tr.set_compute_dtype(torch.float32)
    mel, y = _c5_batch(4)
    sl = slice(2 * rank, 2 * rank + 2)
    tr.step(mel[sl].contiguous(), y[sl].contiguous())
    torch.cuda.synchronize()
    out[rank] = _grads(tr)
    dist.destroy_process_group()


def test_gan_trainer_ddp_two_ranks_matches_global_batch(device):
    """HifiGanTrainer(distributed=True): each rank steps on its half of a batch of 4; the bucketed,
    averaged D and G gradients equal one process's gradients on the whole batch (every HiFi-GAN V1
    loss is a mean over the batch, no batch statistics).  Learning rate 0, so the G step sees the
    same D on both sides."""
    from visual_onoma_to_wave_amd import hifigan
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gan_gloo_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    h = hifigan.AttrDict(dict(hifigan_h(), learning_rate=0.0))
    torch.manual_seed(1234)
    tr = hifigan.HifiGanTrainer(_gen(device), h).set_compute_dtype(torch.float32)
    mel, y = _c5_batch(4)
    tr.step(mel, y)
    torch.cuda.synchronize()
    ref_d, ref_g = _grads(tr)
    for r in range(world):
        d, g = out[r]
        print(f"rank {r}: D {rel_l2(d, ref_d):.2e}  G {rel_l2(g, ref_g):.2e}")
        assert d.shape == ref_d.shape and g.shape == ref_g.shape
        assert rel_l2(d, ref_d) < 1e-5 and rel_l2(g, ref_g) < 1e-5
    torch.testing.assert_close(out[0][0], out[1][0], rtol=0, atol=0)  # every rank holds the same average


def _gan_rccl_graph_worker(rank, world, port, comm, out):
    import torch.distributed as dist
    from visual_onoma_to_wave_amd import hifigan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    h = hifigan.AttrDict(hifigan_h())
    mel, y = _c5_batch(2, seed=3)
    res = []
    for graphed in (False, True):
        torch.manual_seed(1234)
        tr = hifigan.HifiGanTrainer(_gen(dev), h, distributed=True, device=dev, graphed=graphed, capturable=True,
                                    comm_dtype=comm).set_compute_dtype(torch.float32)
        for _ in range(4):
            losses = tr.step_graphed(mel, y, warmup=2) if graphed else tr.step(mel, y)
        torch.cuda.synchronize()
        res.append(({k: float(v) for k, v in losses.items()},
                    torch.cat([p.detach().flatten().cpu() for p in tr.generator.parameters()]),
                    torch.cat([p.detach().flatten().cpu() for p in tr.mpd.parameters()])))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", [None, torch.bfloat16])
def test_gan_graphed_ddp_rccl_matches_eager(device, comm):
    """The HiFi-GAN step with both bucketed RCCL all-reduces captured in its HIP graph (world size
    1: real RCCL launches on the graph's side-stream branch, on the dedicated graph group) against
    eager steps, bit for bit."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gan_rccl_graph_worker, args=(1, _free_port(), comm, out), nprocs=1, join=True)
    (le, ge, de), (lg, gg, dg) = out[0]
    assert all(np.isfinite(v) for v in le.values())
    assert torch.equal(gg, ge) and torch.equal(dg, de) and lg == le
