"""Checkpoint interop through the reference's factories (scripts/utils/model.py:10-33,41-98):
reference-layout files written with torch.save -- ``{"model", "optimizer"}`` (248 keys + an Adam
state over every parameter, as scripts/model/optimizer.py:10 builds it) and ``{"generator"}``
(234 weight-normed keys) -- loaded through ``compat.install()`` + ``scripts.utils.model``.

CPU tests: loading, resuming the optimizer, the missing-vocoder error.  GPU tests: the loaded
models against the oracle, and ``vocoder_infer`` (Normalize=False, with lengths)."""

import os
import sys

import numpy as np
import pytest
import torch

from helpers import configs, golden, hifigan_arrays, hifigan_h, rel_l2, stats, vtts_arrays
from weights import load_into

_ROOTS = ("model", "transformer", "hifigan", "utils", "scripts", "audio", "dataset")


@pytest.fixture
def ref_api():
    """The reference's import surface (compat aliases), removed again afterwards."""
    from visual_onoma_to_wave_amd import compat
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in _ROOTS}
    compat.install()
    import scripts.utils.model as um
    try:
        yield um
    finally:
        for k in list(sys.modules):
            if k.split(".")[0] in _ROOTS:
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})


def _reference_like_vtts_ckpt(path, step):
    """What scripts/04_train.py:160-168 writes: model state + Adam(model.parameters()) state."""
    from visual_onoma_to_wave_amd.model import vTTS
    m = vTTS(*configs())
    load_into(m, vtts_arrays())
    opt = torch.optim.Adam(m.parameters(), betas=(0.9, 0.98), eps=1e-9, weight_decay=0.0)
    for p in m.parameters():
        if p.requires_grad:
            p.grad = torch.full_like(p, 1e-3)
    opt.step()
    os.makedirs(path, exist_ok=True)
    torch.save({"model": m.state_dict(), "optimizer": opt.state_dict()}, os.path.join(path, f"{step}.pth.tar"))
    return m, opt


def _arrays_of(m):
    """The module's state as the oracle's input arrays (minus the init-time tensors it computes)."""
    return {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()
            if not (k.endswith("position_enc") or k.endswith("_bins"))}


def _vocoder_ckpt(root):
    """scripts/hifigan/generator_universal.pth.tar relative to the caller's cwd, weight-norm layout."""
    d = os.path.join(root, "scripts", "hifigan")
    os.makedirs(d, exist_ok=True)
    sd = {k: torch.from_numpy(np.array(v)) for k, v in hifigan_arrays().items()}
    torch.save({"generator": sd}, os.path.join(d, "generator_universal.pth.tar"))
    return sd


def _cfgs(tmp_path):
    pc, mc, tc = configs()
    tc = dict(tc)
    tc["path"] = dict(tc["path"], ckpt_path=str(tmp_path / "ckpt"))
    return pc, mc, tc


def test_get_model_resumes_reference_checkpoint(tmp_path, ref_api):
    """get_model(restore_step, train=True) loads model + optimizer state of a reference-layout
    checkpoint (the Adam param group spans every parameter, frozen ones included) and continues
    the schedule from restore_step; the state it would save loads back into a reference-style Adam."""
    cfgs = _cfgs(tmp_path)
    ref_m, ref_opt = _reference_like_vtts_ckpt(cfgs[2]["path"]["ckpt_path"], 300)
    model, optim = ref_api.get_model(300, cfgs, "cpu", train=True)
    assert model.training
    assert len(optim._optimizer.param_groups[0]["params"]) == len(list(ref_m.parameters()))
    for (k, a), b in zip(model.state_dict().items(), ref_m.state_dict().values()):
        assert torch.equal(a, b), k
    st = optim._optimizer.state_dict()["state"]
    rst = ref_opt.state_dict()["state"]
    assert set(st) == set(rst)
    for i in rst:
        assert torch.equal(st[i]["exp_avg"], rst[i]["exp_avg"])
    assert optim.current_step == 300
    optim._update_learning_rate()
    assert optim.current_step == 301
    back = torch.optim.Adam(ref_m.parameters(), betas=(0.9, 0.98), eps=1e-9)
    back.load_state_dict(optim._optimizer.state_dict())
    m_eval = ref_api.get_model(300, cfgs, "cpu", train=False)
    assert not m_eval.training and len(m_eval.state_dict()) == 248


def test_get_vocoder_loads_weight_norm_checkpoint_and_raises_when_missing(tmp_path, ref_api, monkeypatch):
    monkeypatch.chdir(tmp_path)
    mc = configs()[1]
    with pytest.raises(FileNotFoundError):
        ref_api.get_vocoder(mc, "cpu")  # the reference raises here too (torch.load of a missing file)
    sd = _vocoder_ckpt(str(tmp_path))
    voc = ref_api.get_vocoder(mc, "cpu")
    assert not voc.training
    folded = voc.state_dict()
    assert not any(k.endswith(("weight_g", "weight_v")) for k in folded)
    from oracle import vocoder as V
    ref = V.fold_weight_norm(sd)
    for k in ("conv_pre.weight", "ups.0.weight", "resblocks.11.convs2.2.weight", "conv_post.weight"):
        assert rel_l2(folded[k], ref[k]) < 1e-6, k


@pytest.mark.gpu
def test_factories_forward_and_vocoder_infer_vs_oracle(tmp_path, ref_api, monkeypatch):
    """get_model + get_vocoder on reference-layout files, then the notebook's calls
    (prediction.ipynb: model(*(batch[1:]), use_image); vocoder_infer(..., Normalize=False) with
    lengths) against the oracle on the same weights."""
    from oracle import acoustic as A
    from oracle import vocoder as V
    monkeypatch.chdir(tmp_path)
    cfgs = _cfgs(tmp_path)
    saved, _ = _reference_like_vtts_ckpt(cfgs[2]["path"]["ckpt_path"], 200000)
    sd = _vocoder_ckpt(str(tmp_path))
    dev = torch.device("cuda")
    model = ref_api.get_model(200000, cfgs, dev)
    model.set_precision("fp32")
    voc = ref_api.get_vocoder(cfgs[1], dev)
    voc.set_compute_dtype(torch.float32)
    g = golden("vtts_tf")
    t = lambda k: torch.from_numpy(np.array(g[k]))  # noqa: E731
    args = (t("in_audiotypes"), t("in_texts"), t("in_src_lens"), int(g["in_max_src_len"]), t("in_mels"),
            t("in_mel_lens"), int(g["in_max_mel_len"]), t("in_e_targets"), None, t("in_d_targets"),
            t("in_images"))
    with torch.no_grad():
        out = model(*[a.to(dev) if torch.is_tensor(a) else a for a in args], None, True)
    osd = A.complete_state_dict(_arrays_of(saved), stats()["energy"])
    ref = A.vtts_forward(osd, *args, energy_stats=stats()["energy"])
    assert rel_l2(out[1].cpu(), ref[1]) < 1e-4
    mels = out[1].transpose(1, 2).contiguous()
    lengths = (out[9].cpu().numpy() * 256).tolist()
    wavs = ref_api.vocoder_infer(mels, voc, cfgs[1], cfgs[0], lengths=lengths, Normalize=False)
    ref_w = V.generator(V.fold_weight_norm(sd), ref[1].transpose(1, 2), hifigan_h()).squeeze(1).numpy()
    assert len(wavs) == mels.shape[0]
    for i, w in enumerate(wavs):
        assert isinstance(w, np.ndarray) and w.dtype == np.float32 and w.shape == (int(lengths[i]),)
        assert rel_l2(w, ref_w[i][: int(lengths[i])]) < 1e-3
