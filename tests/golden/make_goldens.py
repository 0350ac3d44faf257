"""Generate the golden vectors under tests/golden/ from the reference itself.

Runs ONLY in the survey/build container, where the reference is mounted read-only
at /root/reference.  It imports the reference's own Python modules (recipe of
SURVEY.md section 8(c): three unused-on-path modules stubbed in ``sys.modules``,
bytecode writing disabled), fills them with the deterministic weights of
``weights.py`` and records inputs and outputs as small ``.npz`` fixtures.  Only
data is written here -- no reference source travels with the repo.

    python tests/golden/make_goldens.py        # rewrites tests/golden/*.npz|json
"""

import hashlib
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

from weights import HIFIGAN_UPS_STRIDES, load_into, make_state_dict, spec_of  # noqa: E402

VTTS_SEED = 20240
GEN_SEED = 4242
DUR_BIAS_SHIFT = 1.6


def import_reference():
    sys.dont_write_bytecode = True
    os.chdir(REF)
    sys.path.insert(0, os.path.join(REF, "scripts"))

    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Compose:  # torchvision.transforms.Compose stand-in (not on the model path)
        def __init__(self, t):
            self.t = t

    tv = stub("torchvision")
    tv.transforms = stub("torchvision.transforms", Compose=_Compose, ToTensor=lambda: None)
    stub("cv2", normalize=None)
    lb = stub("librosa")
    lb.util = stub("librosa.util", pad_center=None, tiny=None, normalize=None)
    lb.filters = stub("librosa.filters", mel=None)
    import yaml
    cfg = {}
    for n in ("preprocess", "model", "train"):
        with open(os.path.join(REF, "config/ICASSP", n + ".yaml")) as f:
            cfg[n] = yaml.load(f, Loader=yaml.SafeLoader)
    return cfg


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", os.path.relpath(path, REPO), os.path.getsize(path), "bytes")


def t2n(t):
    return None if t is None else t.detach().cpu().numpy()


def main():
    cfg = import_reference()
    import torch
    torch.manual_seed(0)
    from model import vTTS, FastSpeech2Loss, ScheduledOptim
    from model.modules import LengthRegulator
    from transformer.Models import get_sinusoid_encoding_table
    from utils.tools import get_mask_from_lengths
    import hifigan
    from visual_onoma_to_wave_amd import synth

    pc, mc, tc = cfg["preprocess"], cfg["model"], cfg["train"]

    # ---------------- acoustic model ----------------
    model = vTTS(pc, mc, tc)
    spec = spec_of(model.state_dict())
    with open(os.path.join(HERE, "vtts_spec.json"), "w") as f:
        json.dump({"seed": VTTS_SEED, "spec": spec}, f)
    load_into(model, make_state_dict(spec, VTTS_SEED))
    model.eval()

    pe = get_sinusoid_encoding_table(1001, 256).numpy()
    meta = {
        "position_enc_sha256": hashlib.sha256(pe.astype(np.float32).tobytes()).hexdigest(),
        "position_enc_rows": {str(r): pe[r, :8].tolist() for r in (0, 1, 17, 500, 1000)},
        "energy_bins_sha256": hashlib.sha256(t2n(model.variance_adaptor.energy_bins).tobytes()).hexdigest(),
        "n_params": int(sum(p.numel() for p in model.parameters())),
        "n_keys": len(spec),
    }

    rng = np.random.default_rng(7)
    with torch.no_grad():
        # a1: visual feature extractor
        imgs = synth.glyph_images(rng, 2, 3)
        vfe = model.encoder.VisualFeatureExtractor(torch.from_numpy(imgs))
        save("vfe", images=imgs, out=t2n(vfe))

        # a4-a7: FFT blocks (encoder layer 0 at L=12, decoder layer 0 at L=64), ragged masks
        for name, layer, L, lens in (("fft_enc", model.encoder.layer_stack[0], 12, [12, 7]),
                                     ("fft_dec", model.decoder.layer_stack[0], 64, [64, 41])):
            x = rng.normal(0, 1, size=(2, L, 256)).astype(np.float32)
            lens_t = torch.tensor(lens)
            mask = get_mask_from_lengths(lens_t, L)
            out, attn = layer(torch.from_numpy(x), mask=mask,
                              slf_attn_mask=mask.unsqueeze(1).expand(-1, L, -1))
            save(name, x=x, lens=np.array(lens), out=t2n(out), attn=t2n(attn))

        # a9: variance predictors
        x = rng.normal(0, 1, size=(2, 12, 256)).astype(np.float32)
        lens_t = torch.tensor([12, 5])
        mask = get_mask_from_lengths(lens_t, 12)
        va = model.variance_adaptor
        save("var_pred", x=x, lens=np.array([12, 5]),
             log_d=t2n(va.duration_predictor(torch.from_numpy(x), mask)),
             energy=t2n(va.energy_predictor(torch.from_numpy(x), mask)))

        # a10: bucketize against the energy bins (edges included on purpose)
        bins = t2n(va.energy_bins)
        vals = np.concatenate([rng.normal(1.5, 2.5, size=200).astype(np.float32),
                               bins[[0, 1, 17, 128, 253, 254]],
                               np.array([-5, 10, bins[0] - 1e-6, bins[-1] + 1e-6], np.float32)])
        idx = torch.bucketize(torch.from_numpy(vals), va.energy_bins)
        emb = va.energy_embedding(idx)
        save("bucketize", bins=bins, values=vals, index=t2n(idx), emb=t2n(emb))

        # a12: LengthRegulator -- fractional, zero, negative durations; max_len None / given / cropping
        lr = LengthRegulator()
        x = rng.normal(0, 1, size=(3, 7, 8)).astype(np.float32)
        d = np.array([[1.0, 2.7, 0.0, 3.0, 1.2, 0.9, 2.0],
                      [4.0, -1.0, 1.0, 1.0, 0.0, 0.0, 0.0],
                      [0.5, 0.2, 2.9999, 1.0, 5.0, 1.0, 1.0]], np.float32)
        cases = {}
        for tag, ml in (("none", None), ("given", 16), ("crop", 6)):
            out, mel_len = lr(torch.from_numpy(x), torch.from_numpy(d), ml)
            cases["out_" + tag] = t2n(out)
            cases["mel_len_" + tag] = t2n(mel_len)
        save("length_regulator", x=x, d=d, **cases)

        # a13
        lens = torch.tensor([3, 0, 7, 5])
        save("mask", lens=t2n(lens), mask_none=t2n(get_mask_from_lengths(lens)),
             mask_9=t2n(get_mask_from_lengths(lens, 9)))

        # a15: PostNet (eval BatchNorm)
        x = rng.normal(0, 1, size=(2, 32, 80)).astype(np.float32)
        save("postnet", x=x, out=t2n(model.postnet(torch.from_numpy(x))))

        # a16: the whole acoustic model, teacher-forced (training-style inputs) ...
        b = synth.acoustic_batch(99, 2, 6, 40, ragged=True)
        tb = {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
        out = model(tb["audiotypes"], tb["texts"], tb["src_lens"], tb["max_src_len"],
                    tb["mels"], tb["mel_lens"], tb["max_mel_len"], tb["e_targets"], None,
                    tb["d_targets"], tb["images"], None, True)
        names = ["mel", "postnet_mel", "e_pred", "k_pred", "log_d_pred", "d_rounded",
                 "src_masks", "mel_masks", "src_lens_out", "mel_lens_out"]
        res = {n: t2n(o) for n, o in zip(names, out) if o is not None}
        save("vtts_tf", **{"in_" + k: np.asarray(v) for k, v in b.items()}, **res)

        # a22: loss on that output
        batch = (None, tb["audiotypes"], tb["texts"], tb["src_lens"], tb["max_src_len"],
                 tb["mels"], tb["mel_lens"], tb["max_mel_len"], tb["e_targets"], None,
                 tb["d_targets"], tb["images"], None)
        losses = FastSpeech2Loss()(batch, out)
        save("loss", values=np.array([float(l) for l in losses], np.float64))

        # ... and in inference mode (predicted energy + durations), with controls.  With
        # random weights the predicted log-durations sit near 0 (every token rounds to
        # 0 frames and the reference decoder cannot run), so the duration head's bias
        # is shifted by DUR_BIAS_SHIFT for these fixtures; tests apply the same shift.
        model.variance_adaptor.duration_predictor.linear_layer.bias += DUR_BIAS_SHIFT
        for tag, ec, dc in (("inf", 1.0, 1.0), ("inf_ctrl", 1.2, 1.5)):
            b = synth.acoustic_batch(123, 2, 5, 20, ragged=True)
            tb = {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
            out = model(tb["audiotypes"], tb["texts"], tb["src_lens"], tb["max_src_len"],
                        None, None, None, None, None, None, tb["images"], None, True,
                        e_control=ec, d_control=dc)
            res = {n: t2n(o) for n, o in zip(names, out) if o is not None}
            save("vtts_" + tag, **{"in_" + k: np.asarray(v) for k, v in b.items()},
                 e_control=np.float32(ec), d_control=np.float32(dc),
                 dur_bias_shift=np.float32(DUR_BIAS_SHIFT), **res)
        model.variance_adaptor.duration_predictor.linear_layer.bias -= DUR_BIAS_SHIFT

    # a23: learning-rate schedule of ScheduledOptim
    opt = ScheduledOptim(torch.nn.Linear(2, 2), tc, mc, 0)
    steps = [1, 2, 3, 100, 3999, 4000, 4001, 10000, 299999, 300000, 300001, 400001, 500001]
    lrs = []
    for s in steps:
        opt.current_step = s - 1
        opt._update_learning_rate()
        lrs.append(opt._optimizer.param_groups[0]["lr"])
    meta["lr_steps"] = steps
    meta["lr_values"] = lrs

    # ---------------- HiFi-GAN generator ----------------
    with open(os.path.join(REF, "scripts/hifigan/config.json")) as f:
        h = hifigan.AttrDict(json.load(f))
    gen = hifigan.Generator(h)
    gspec = spec_of(gen.state_dict())
    with open(os.path.join(HERE, "hifigan_spec.json"), "w") as f:
        json.dump({"seed": GEN_SEED, "spec": gspec}, f)
    load_into(gen, make_state_dict(gspec, GEN_SEED, HIFIGAN_UPS_STRIDES))
    gen.eval()
    gen.remove_weight_norm()
    meta["gen_n_keys"] = len(gspec)
    rng = np.random.default_rng(11)
    with torch.no_grad():
        folded = {k: t2n(v) for k, v in gen.state_dict().items() if k.startswith("conv_pre")}
        save("weightnorm_fold", conv_pre_weight_head=folded["conv_pre.weight"][:16])
        chans = [256, 128, 64, 32]
        for i, C in enumerate(chans):
            x = rng.normal(0, 1, size=(1, C, 48)).astype(np.float32)
            outs = {}
            for j, k in enumerate((3, 7, 11)):
                outs[f"k{k}"] = t2n(gen.resblocks[3 * i + j](torch.from_numpy(x)))
            save(f"resblock_s{i}", x=x, **outs)
        ups = {}
        for i, Ci in enumerate([512, 256, 128, 64]):
            x = rng.normal(0, 1, size=(1, Ci, 10)).astype(np.float32)
            y = gen.ups[i](torch.nn.functional.leaky_relu(torch.from_numpy(x), 0.1))
            ups[f"x{i}"] = x
            ups[f"y{i}"] = t2n(y)
        save("ups", **ups)
        mel = synth.mels(rng, 2, 12)
        save("generator", mel=mel, wav=t2n(gen(torch.from_numpy(mel))))

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("meta:", {k: v for k, v in meta.items() if "rows" not in k})


def long_goldens():
    """Multi-tile vocoder goldens (round 2): the MRF of every stage (sum of the three ResBlocks / 3,
    hifigan/models.py:155-160) on inputs long enough to cross several 256 / 512-row tiles of the
    fused kernels and two utterances, and the whole Generator at T = 80 mel frames (stage 3 runs
    20,480 rows).  Activations are stored as float16 (inputs drawn fp16-exact, outputs rounded:
    rel-L2 ~3e-4 of storage error, far below the 1e-2 bf16 tolerance they pin)."""
    import torch
    import hifigan
    with open(os.path.join(REF, "scripts/hifigan/config.json")) as f:
        h = hifigan.AttrDict(json.load(f))
    gen = hifigan.Generator(h)
    gspec = spec_of(gen.state_dict())
    load_into(gen, make_state_dict(gspec, GEN_SEED, HIFIGAN_UPS_STRIDES))
    gen.eval()
    gen.remove_weight_norm()
    rng = np.random.default_rng(2024)
    with torch.no_grad():
        for i, (C, T) in enumerate(((256, 600), (128, 1100), (64, 1100), (32, 1100))):
            x = rng.normal(0, 1, size=(2, C, T)).astype(np.float16).astype(np.float32)
            xt = torch.from_numpy(x)
            y = sum(gen.resblocks[3 * i + j](xt) for j in range(3)) / 3
            save(f"mrf_s{i}_long", x=x.astype(np.float16), out=t2n(y).astype(np.float16))
        from visual_onoma_to_wave_amd import synth
        mel = synth.mels(rng, 2, 80)
        save("generator_long", mel=mel, wav=t2n(gen(torch.from_numpy(mel))))


def stft_goldens():
    """Round 3: the reference's own Tacotron STFT front end (scripts/audio/stft.py:52-81 STFT.transform,
    :159-178 TacotronSTFT.mel_spectrogram, audio_processing.py:85-91 dynamic_range_compression) run
    on CPU: ``Tensor.cuda`` is patched to the identity for the call (stft.py:68-69 hard-codes
    ``.cuda()``), ``pad_center`` is the identity (win_length == filter_length, stft.py:41-42), and
    the window is scipy's ``get_window("hann", 1024, fftbins=True)`` as the reference computes it.
    librosa is absent, so the mel basis fed to ``mel_spectrogram`` is the oracle's restatement of
    ``librosa.filters.mel`` (slaney): the basis itself stays parity-unpinned, everything around it
    -- DFT-basis magnitude, basis product, log compression, energy -- is the reference's code.
    Two wav lengths (one full second, one ragged), B = 2, signals in [-1, 1]."""
    import torch
    import audio.stft as ref_stft
    from oracle.mel import librosa_mel
    ref_stft.pad_center = lambda w, size: w if len(w) == size else np.pad(
        w, ((size - len(w)) // 2, size - len(w) - (size - len(w)) // 2))
    ref_stft.librosa_mel_fn = lambda sr, n_fft, n_mels, fmin, fmax: librosa_mel(sr, n_fft, n_mels, fmin, fmax)
    tac = ref_stft.TacotronSTFT(1024, 256, 1024, 80, 22050, 0.0, 8000.0)
    rng = np.random.default_rng(31)
    real_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        for name, N in (("stft_ref_22050", 22050), ("stft_ref_9001", 9001)):
            t = np.arange(N) / 22050.0
            f0 = rng.uniform(80, 2000, size=(2, 1))
            wav = (0.5 * np.sin(2 * np.pi * f0 * t) + 0.2 * np.sin(2 * np.pi * 3.1 * f0 * t)
                   + 0.1 * rng.standard_normal((2, N)))
            wav = np.clip(wav, -1, 1).astype(np.float32)
            with torch.no_grad():
                mag, _ = tac._stft_fn.transform(torch.from_numpy(wav))
                mel, energy = tac.mel_spectrogram(torch.from_numpy(wav))
                drc = ref_stft.dynamic_range_compression(mag)
            save(name, wav=wav, window=np.asarray(ref_stft.get_window("hann", 1024, fftbins=True), np.float32),
                 mel_basis=t2n(tac.mel_basis), magnitude=t2n(mag), log_magnitude=t2n(drc), mel=t2n(mel),
                 energy=t2n(energy))
    finally:
        torch.Tensor.cuda = real_cuda


if __name__ == "__main__":
    if sys.argv[1:] == ["long"]:
        import_reference()
        long_goldens()
    elif sys.argv[1:] == ["stft"]:
        import_reference()
        import utils.tools  # noqa: F401  (imports the reference's audio package as main() does)
        stft_goldens()
    else:
        main()
        long_goldens()
        stft_goldens()
