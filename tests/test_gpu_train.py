"""Training path (C4) on the GPU: teacher-forced forward in train mode (BatchNorm batch
statistics; dropout probabilities set to 0 so both sides are deterministic), FastSpeech2Loss,
backward -- loss terms and parameter gradients against the oracle's autograd on the CPU.

Tolerances: fp32 mode (exact-f32 MFMA forward and HIP dgrad) rel-L2 <= 1e-4 on losses and
<= 2e-3 on gradients (long backward chains through LayerNorm / softmax in a different
summation order); mixed mode loss within 2e-2."""

import numpy as np
import pytest
import torch

from helpers import configs, golden, rel_l2, stats, vtts_arrays
from weights import load_into

pytestmark = pytest.mark.gpu


def _no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0


def _batch(g, dev):
    t = lambda k: torch.from_numpy(np.array(g[k])).to(dev)  # noqa: E731
    return (None, t("in_audiotypes"), t("in_texts"), t("in_src_lens"), int(g["in_max_src_len"]), t("in_mels"),
            t("in_mel_lens"), int(g["in_max_mel_len"]), t("in_e_targets"), None, t("in_d_targets"),
            t("in_images"), None)


def _oracle_grads(arrays, batch_cpu):
    from oracle import acoustic as A
    from oracle import training as TR
    sd = A.complete_state_dict(arrays, stats()["energy"])
    for k, v in sd.items():
        if v.dtype == torch.float32 and "position_enc" not in k and "bins" not in k and "running" not in k:
            v.requires_grad_(True)
    out = A.vtts_forward(sd, *batch_cpu[1:12], energy_stats=stats()["energy"], training=True)
    losses = TR.fastspeech2_loss(batch_cpu, out)
    losses[0].backward()
    return [float(x) for x in losses], {k: v.grad for k, v in sd.items() if v.grad is not None}


@pytest.mark.parametrize("mode", ["fp32", "mixed"])
def test_train_step_grads_vs_oracle(device, mode):
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    arrays = vtts_arrays()
    g = golden("vtts_tf")
    m = vTTS(*configs())
    load_into(m, arrays)
    m = m.to(device).train().set_precision(mode)
    _no_dropout(m)
    batch = _batch(g, device)
    out = m(*(batch[1:]), True)
    losses = FastSpeech2Loss()(batch, out)
    losses[0].backward()
    ref_losses, ref_grads = _oracle_grads(arrays, _batch(g, "cpu"))
    got = [float(x) for x in losses]
    tol = 1e-4 if mode == "fp32" else 2e-2
    np.testing.assert_allclose(got, ref_losses, rtol=tol, atol=1e-6)
    if mode != "fp32":
        return
    named = dict(m.named_parameters())
    checked, bad = 0, []
    for k, gr in ref_grads.items():
        p = named.get(k)
        if p is None or p.grad is None:
            continue
        # conv biases feeding a train-mode BatchNorm have an exactly-zero true gradient
        # (both sides are rounding noise ~1e-8): an absolute floor covers them
        err = float((p.grad.cpu() - gr).norm())
        if err > 2e-3 * float(gr.norm()) + 1e-5:
            bad.append((k, err, float(gr.norm())))
        checked += 1
    assert not bad, bad[:10]
    assert checked > 150


def test_training_reduces_loss(device):
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import train_step
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(device).train()
    opt = ScheduledOptim(m, tc, mc, 0)
    batch = _batch(golden("vtts_tf"), device)
    first = None
    for _ in range(12):
        losses = train_step(m, opt, FastSpeech2Loss(), batch)
        first = first if first is not None else float(losses[0])
    assert float(losses[0]) < 0.8 * first


def test_graphed_train_step_matches_eager(device):
    """train.GraphedTrainStep (HIP-graph replay with the capturable Adam and a device-tensor
    learning rate) against the same number of eager train_step calls (fp32, dropout off).  The
    weight-gradient atomics make two eager runs differ slightly; training amplifies that, so the
    graphed run is held to the spread of a second eager run, not to zero."""
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import GraphedTrainStep, train_step
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["optimizer"] = dict(tc["optimizer"], warm_up_step=10, init_lr=1e-3)  # steps that move the weights
    batch = _batch(golden("vtts_tf"), device)
    finals = []
    for graphed in (False, False, True):
        m = vTTS(pc, mc, tc)
        load_into(m, vtts_arrays())
        m = m.to(device).train().set_precision("fp32")
        _no_dropout(m)
        opt = ScheduledOptim(m, tc, mc, 0, capturable=graphed)
        if graphed:
            run = GraphedTrainStep(m, opt, FastSpeech2Loss(), warmup=1)
            for _ in range(11):  # 1 eager warm-up step + capture, then 11 replays
                losses = run(batch)
        else:
            for _ in range(12):
                losses = train_step(m, opt, FastSpeech2Loss(), batch)
        torch.cuda.synchronize()
        assert opt.current_step == 12
        finals.append((np.array([float(x) for x in losses]),
                       torch.cat([p.detach().flatten().cpu() for p in m.parameters()])))
    (l0, p0), (l1, p1), (lg, pg) = finals
    p_noise = float((p1 - p0).norm() / p0.norm())
    p_err = float((pg - p0).norm() / p0.norm())
    l_noise, l_err = float(np.abs(l1 - l0).max()), float(np.abs(lg - l0).max())
    print(f"graphed vs eager: params {p_err:.2e} (eager spread {p_noise:.2e}), losses {l_err:.2e} "
          f"(eager spread {l_noise:.2e})")
    # twelve Adam steps at lr up to 3e-4 move the weights by ~1e-2 of their norm and the loss
    # 25 -> 7.5: a replay with a stale input / learning rate / packed weight differs at that scale
    assert p_err < max(10 * p_noise, 1e-6) and p_err < 1e-3
    assert l_err < max(10 * l_noise, 1e-4)
