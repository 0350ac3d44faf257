"""Pin the CPU oracle to the reference: oracle vs golden vectors produced by running
the reference itself (tests/golden/make_goldens.py).  CPU only."""

import hashlib

import numpy as np
import pytest
import torch

from helpers import golden, hifigan_arrays, hifigan_h, meta, rel_l2, stats, t, vtts_arrays
from oracle import acoustic as A
from oracle import training as TR
from oracle import vocoder as V

TOL = 1e-5  # fp32 CPU vs fp32 CPU: only op-ordering differences


@pytest.fixture(scope="module")
def sd():
    return A.complete_state_dict(vtts_arrays(), stats()["energy"])


@pytest.fixture(scope="module")
def gsd():
    return V.fold_weight_norm({k: torch.from_numpy(np.array(v)) for k, v in hifigan_arrays().items()})


def test_sinusoid_table_bit_exact():
    pe = A.sinusoid_table(1001, 256).numpy()
    assert hashlib.sha256(pe.tobytes()).hexdigest() == meta()["position_enc_sha256"]


def test_energy_bins_bit_exact():
    b = A.energy_bins(stats()["energy"]).numpy()
    assert hashlib.sha256(b.tobytes()).hexdigest() == meta()["energy_bins_sha256"]


def test_vfe(sd):
    g = golden("vfe")
    out = A.vfe(sd, t(g["images"]))
    assert rel_l2(out, g["out"]) < TOL


@pytest.mark.parametrize("name,prefix", [("fft_enc", "encoder.layer_stack.0"),
                                         ("fft_dec", "decoder.layer_stack.0")])
def test_fft_block(sd, name, prefix):
    g = golden(name)
    L = g["x"].shape[1]
    mask = A.mask_from_lengths(t(g["lens"]), L)
    out, attn = A.fft_block(sd, prefix, t(g["x"]), mask)
    assert rel_l2(out, g["out"]) < TOL
    assert rel_l2(attn, g["attn"]) < TOL


def test_variance_predictors(sd):
    g = golden("var_pred")
    mask = A.mask_from_lengths(t(g["lens"]), 12)
    p = "variance_adaptor."
    assert rel_l2(A.variance_predictor(sd, p + "duration_predictor", t(g["x"]), mask), g["log_d"]) < TOL
    assert rel_l2(A.variance_predictor(sd, p + "energy_predictor", t(g["x"]), mask), g["energy"]) < TOL


def test_bucketize_exact(sd):
    g = golden("bucketize")
    idx = A.bucketize(g["values"], g["bins"])
    np.testing.assert_array_equal(idx, g["index"])
    emb = sd["variance_adaptor.energy_embedding.weight"][torch.from_numpy(idx)]
    np.testing.assert_array_equal(emb.numpy(), g["emb"])


@pytest.mark.parametrize("tag,max_len", [("none", None), ("given", 16), ("crop", 6)])
def test_length_regulator_exact(tag, max_len):
    g = golden("length_regulator")
    out, mel_len, _ = A.length_regulate(t(g["x"]), g["d"], max_len)
    np.testing.assert_array_equal(mel_len.numpy(), g["mel_len_" + tag])
    np.testing.assert_array_equal(out.numpy(), g["out_" + tag])


def test_mask():
    g = golden("mask")
    np.testing.assert_array_equal(A.mask_from_lengths(t(g["lens"])).numpy(), g["mask_none"])
    np.testing.assert_array_equal(A.mask_from_lengths(t(g["lens"]), 9).numpy(), g["mask_9"])


def test_postnet(sd):
    g = golden("postnet")
    assert rel_l2(A.postnet(sd, t(g["x"])), g["out"]) < TOL


def _run_vtts(sd, g, with_targets, ec=1.0, dc=1.0):
    kw = dict(energy_stats=stats()["energy"], e_control=ec, d_control=dc)
    if with_targets:
        return A.vtts_forward(sd, t(g["in_audiotypes"]), t(g["in_texts"]), t(g["in_src_lens"]),
                              int(g["in_max_src_len"]), t(g["in_mels"]), t(g["in_mel_lens"]),
                              int(g["in_max_mel_len"]), t(g["in_e_targets"]), None,
                              t(g["in_d_targets"]), t(g["in_images"]), **kw)
    return A.vtts_forward(sd, t(g["in_audiotypes"]), t(g["in_texts"]), t(g["in_src_lens"]),
                          int(g["in_max_src_len"]), images=t(g["in_images"]), **kw)


NAMES = ["mel", "postnet_mel", "e_pred", "k_pred", "log_d_pred", "d_rounded",
         "src_masks", "mel_masks", "src_lens_out", "mel_lens_out"]


def _check_vtts(out, g):
    for n, o in zip(NAMES, out):
        if o is None:
            assert n not in g
            continue
        if o.dtype in (torch.bool, torch.int64) or n == "d_rounded":
            np.testing.assert_array_equal(o.numpy(), g[n], err_msg=n)
        else:
            assert rel_l2(o, g[n]) < 1e-5, n


def test_vtts_teacher_forced(sd):
    g = golden("vtts_tf")
    _check_vtts(_run_vtts(sd, g, True), g)


@pytest.mark.parametrize("tag", ["inf", "inf_ctrl"])
def test_vtts_inference(sd, tag):
    g = golden("vtts_" + tag)
    sd2 = dict(sd)
    key = "variance_adaptor.duration_predictor.linear_layer.bias"
    sd2[key] = sd[key] + float(g["dur_bias_shift"])
    _check_vtts(_run_vtts(sd2, g, False, float(g["e_control"]), float(g["d_control"])), g)


def test_loss(sd):
    g = golden("vtts_tf")
    out = _run_vtts(sd, g, True)
    batch = (None, t(g["in_audiotypes"]), t(g["in_texts"]), t(g["in_src_lens"]),
             int(g["in_max_src_len"]), t(g["in_mels"]), t(g["in_mel_lens"]),
             int(g["in_max_mel_len"]), t(g["in_e_targets"]), None, t(g["in_d_targets"]),
             t(g["in_images"]), None)
    losses = TR.fastspeech2_loss(batch, out)
    np.testing.assert_allclose([float(x) for x in losses], golden("loss")["values"], rtol=1e-5)


def test_lr_schedule():
    m = meta()
    for s, lr in zip(m["lr_steps"], m["lr_values"]):
        assert TR.lr_at(s) == pytest.approx(lr, rel=1e-12)


def test_weight_norm_fold(gsd):
    g = golden("weightnorm_fold")
    np.testing.assert_allclose(gsd["conv_pre.weight"][:16].numpy(), g["conv_pre_weight_head"],
                               rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_resblocks(gsd, stage):
    g = golden(f"resblock_s{stage}")
    for j, k in enumerate((3, 7, 11)):
        out = V.resblock(gsd, f"resblocks.{3 * stage + j}", t(g["x"]), k)
        assert rel_l2(out, g[f"k{k}"]) < TOL


def test_upsamplers(gsd):
    g = golden("ups")
    h = hifigan_h()
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        out = V.upsample(gsd, i, t(g[f"x{i}"]), k, u)
        assert rel_l2(out, g[f"y{i}"]) < TOL


def test_generator(gsd):
    g = golden("generator")
    assert rel_l2(V.generator(gsd, t(g["mel"]), hifigan_h()), g["wav"]) < TOL


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_mrf_long(gsd, stage):
    """Multi-tile MRF goldens (sum of the stage's three ResBlocks / 3 on T = 600 / 1100 rows,
    B = 2): outputs stored as float16, so the bound is the storage rounding (~3e-4)."""
    g = golden(f"mrf_s{stage}_long")
    out = V.mrf(gsd, stage, t(g["x"]).float(), hifigan_h())
    assert rel_l2(out, g["out"].astype(np.float32)) < 1e-3


def test_generator_long(gsd):
    g = golden("generator_long")
    assert rel_l2(V.generator(gsd, t(g["mel"]), hifigan_h()), g["wav"]) < TOL
