"""CPU-only checks of the host side: C-ABI library exports, checkpoint-layout compatibility,
config/metadata handling, LR schedule, batch plumbing.  No GPU compute is issued."""

import ctypes
import hashlib
import os
import re

import numpy as np
import pytest
import torch

from helpers import DATA, REPO, configs, meta, spec

LIB = os.path.join(REPO, "visual_onoma_to_wave_amd", "lib", "libvonoma.so")
HEADER = os.path.join(REPO, "include", "vonoma.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(vo_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB), "run `make -C visual_onoma_to_wave_amd` (or __graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/vonoma.h but not exported"
    lib.vo_num_symbols.restype = ctypes.c_int
    lib.vo_symbol_name.restype = ctypes.c_char_p
    listed = {lib.vo_symbol_name(i).decode() for i in range(lib.vo_num_symbols())}
    assert listed == set(syms)


def test_vtts_state_dict_layout_matches_reference():
    from visual_onoma_to_wave_amd.model import vTTS
    m = vTTS(*configs())
    sd = m.state_dict()
    _, ref = spec("vtts")
    assert [k for k, _, _ in ref] == list(sd.keys())
    for k, shape, _ in ref:
        assert tuple(sd[k].shape) == tuple(shape), k
    assert sum(p.numel() for p in m.parameters()) == meta()["n_params"]


def test_generator_state_dict_layout_matches_reference():
    from visual_onoma_to_wave_amd import hifigan
    from helpers import hifigan_h
    g = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    sd = g.state_dict()
    _, ref = spec("hifigan")
    assert [k for k, _, _ in ref] == list(sd.keys())
    for k, shape, _ in ref:
        assert tuple(sd[k].shape) == tuple(shape), k


def test_position_enc_and_bins_bit_exact():
    from visual_onoma_to_wave_amd.model import vTTS
    m = vTTS(*configs())
    pe = m.encoder.position_enc.detach()[0].numpy()
    assert hashlib.sha256(pe.tobytes()).hexdigest() == meta()["position_enc_sha256"]
    assert torch.equal(m.encoder.position_enc, m.decoder.position_enc)
    b = m.variance_adaptor.energy_bins.detach().numpy()
    assert hashlib.sha256(b.tobytes()).hexdigest() == meta()["energy_bins_sha256"]


def test_vocabulary():
    from visual_onoma_to_wave_amd.utils.symbols import get_symbols
    s = get_symbols(DATA)
    assert len(s) == 72 and min(s.values()) == 1


def test_scheduled_optim_lr_matches_reference():
    from visual_onoma_to_wave_amd.model import ScheduledOptim
    pc, mc, tc = configs()
    opt = ScheduledOptim(torch.nn.Linear(2, 2), tc, mc, 0)
    m = meta()
    for s, lr in zip(m["lr_steps"], m["lr_values"]):
        opt.current_step = s - 1
        opt._update_learning_rate()
        assert opt._optimizer.param_groups[0]["lr"] == pytest.approx(lr, rel=1e-12)


def test_to_device_batch_plumbing():
    from visual_onoma_to_wave_amd.utils.tools import to_device
    imgs = [np.full((24, 204), 255, np.uint8), np.zeros((24, 204), np.uint8)]
    batch = (["a", "b"], np.array([1, 2]), np.array([[3, 4], [5, 0]]), np.array([2, 1]), 2,
             np.zeros((2, 10, 80), np.float32), np.array([10, 7]), 10, np.zeros((2, 2), np.float32),
             None, np.array([[4, 6], [7, 0]]), imgs, np.array([None]))
    out = to_device(batch, "cpu")
    assert out[11].shape == (2, 1, 24, 204) and out[11].dtype == torch.float32
    assert float(out[11][0].min()) == 1.0 and float(out[11][1].max()) == 0.0
    assert out[6].dtype == torch.float32 and out[10].dtype == torch.float32
    assert out[12] is None and out[1].dtype == torch.int64


def test_mask_from_lengths_cpu_semantics():
    from visual_onoma_to_wave_amd.utils.tools import get_mask_from_lengths
    from helpers import golden
    g = golden("mask")
    np.testing.assert_array_equal(get_mask_from_lengths(torch.from_numpy(g["lens"])).numpy(), g["mask_none"])
    np.testing.assert_array_equal(get_mask_from_lengths(torch.from_numpy(g["lens"]), 9).numpy(), g["mask_9"])


def test_compat_aliases():
    import sys
    from visual_onoma_to_wave_amd import compat
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k.split(".")[0] in (
        "model", "transformer", "hifigan", "utils", "scripts", "audio")}
    try:
        compat.install()
        from scripts.utils.model import get_model, get_vocoder  # noqa: F401
        import model as m2
        import hifigan as h2
        assert m2.vTTS.__module__.startswith("visual_onoma_to_wave_amd")
        assert h2.Generator.__module__.startswith("visual_onoma_to_wave_amd")
    finally:
        for k in list(sys.modules):
            if k.split(".")[0] in ("model", "transformer", "hifigan", "utils", "scripts", "audio"):
                del sys.modules[k]
        sys.modules.update({k: v for k, v in saved.items() if v is not None})


def test_ops_refuse_cpu_tensors():
    from visual_onoma_to_wave_amd import ops
    x = torch.zeros(1, 4, 8)
    w = torch.zeros(1, 8, 8, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.conv1d(x, w, None, Co=8, K=1)


def test_synthetic_glyphs_shape_and_ink():
    from visual_onoma_to_wave_amd import synth
    img = synth.glyph_images(np.random.default_rng(0), 2, 5)
    assert img.shape == (2, 1, 24, 510) and img.dtype == np.float32
    ink = float((img < 0.5).mean())
    assert 0.05 < ink < 0.25
    d = synth.durations(np.random.default_rng(1), 4, 12, 512)
    assert (d.sum(1) == 512).all() and (d >= 1).all()


def test_vo_tune_rejects_timing_ablations():
    """Kernel configurations that skip loads for timing ablations give wrong results: the shipped
    library refuses to select them (only a -DVO_ABLATIONS build dispatches them)."""
    from visual_onoma_to_wave_amd import _lib
    L = _lib.lib()
    for v in (13, 16, 17, 25):
        assert L.vo_tune(b"pair_cfg", v) != 0
        assert b"ablation" in L.vo_last_error()
    assert L.vo_tune(b"pair_cfg", 0) == 0
