"""Per-parameter gradient error table of the benched training precisions against the fp32 oracle:
C4 "mixed" (vTTS at B = 32, T_mel = 512) and, with --gan, one bf16 HiFi-GAN step -- next to the oracle's
own bf16-autocast drift on the same quantity (the bar of tests/test_gpu_train_sizes.py /
tests/test_gpu_gan.py).  Prints the rows sorted by error / drift."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    sys.path.insert(0, p)

from helpers import configs, rel_l2, vtts_arrays  # noqa: E402
from weights import load_into  # noqa: E402


def c4():
    import test_gpu_train_sizes as TS
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, vTTS
    arrays = vtts_arrays()
    m = vTTS(*configs())
    load_into(m, arrays)
    m = m.to("cuda").train().set_precision(os.environ.get("MODE", "mixed"))
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0
    batch = TS._c4_batch("cuda")
    out = m(*(batch[1:]), True)
    losses = FastSpeech2Loss()(batch, out)
    losses[0].backward()
    torch.set_num_threads(16)
    bc = TS._c4_batch("cpu")
    ref, rg = TS._c4_oracle(arrays, bc, False)
    refb, bg = TS._c4_oracle(arrays, bc, os.environ.get("BF", "autocast"))
    # forward drift of the two outputs (mel, postnet mel) vs the fp32 oracle
    from oracle import acoustic as A
    from helpers import stats
    sd = A.complete_state_dict(arrays, stats()["energy"])
    with torch.no_grad():
        o32 = A.vtts_forward(sd, *bc[1:12], energy_stats=stats()["energy"], training=True)
        for mode in ("autocast", "operands"):
            ob = A.vtts_forward(sd, *bc[1:12], energy_stats=stats()["energy"], training=True, bf16_back=mode)
            print(f"forward drift {mode}: mel {rel_l2(ob[0], o32[0]):.3e} postnet {rel_l2(ob[1], o32[1]):.3e}")
    print(f"forward drift ours: mel {rel_l2(out[0].detach().float().cpu(), o32[0]):.3e} "
          f"postnet {rel_l2(out[1].detach().float().cpu(), o32[1]):.3e}")
    print("losses ours", [round(float(x), 6) for x in losses])
    print("losses fp32", [round(x, 6) for x in ref])
    print("losses bf16", [round(x, 6) for x in refb])
    named = dict(m.named_parameters())
    rows = []
    for k, r in rg.items():
        p = named.get(k)
        if p is None or p.grad is None:
            continue
        a = p.grad.float().cpu()
        rows.append((rel_l2(a, r) / max(rel_l2(bg[k], r), 1e-2), k, float(r.norm()), rel_l2(a, r), rel_l2(bg[k], r)))
    rows.sort(reverse=True)
    print(f"{'ratio':>7} {'|g|':>10} {'ours':>9} {'bf16':>9}  name")
    for row in rows[:40]:
        print(f"{row[0]:7.3f} {row[2]:10.3e} {row[3]:9.2e} {row[4]:9.2e}  {row[1]}")


def gan():
    import test_gpu_gan as TG
    g, mpd, msd, mel, y = TG._gan_setup()
    dmods = TG._dmods(mpd, msd)
    torch.set_num_threads(16)
    ld_r, gd_r, lg_r, gg_r, _ = TG._oracle_gan_step(g, dmods, mel, y, False)
    ld_b, gd_b, lg_b, gg_b, _ = TG._oracle_gan_step(g, dmods, mel, y, True)
    ld, gd, lg, gg, _ = TG._hip_gan_step(g, mpd, msd, mel, y, torch.bfloat16)
    print(f"L_D ours {ld:.6f} fp32 {ld_r:.6f} bf16 {ld_b:.6f}; L_G ours {lg:.6f} fp32 {lg_r:.6f} bf16 {lg_b:.6f}")
    rows = []
    for i, r in enumerate(gd_r):
        rows.append((rel_l2(gd[i], r) / max(rel_l2(gd_b[i], r), 1e-2), f"D{i} {tuple(r.shape)}", float(r.norm()),
                     rel_l2(gd[i], r), rel_l2(gd_b[i], r)))
    for k, r in gg_r.items():
        rows.append((rel_l2(gg[k], r) / max(rel_l2(gg_b[k], r), 1e-2), k, float(r.norm()), rel_l2(gg[k], r),
                     rel_l2(gg_b[k], r)))
    rows.sort(reverse=True)
    print(f"{'ratio':>7} {'|g|':>10} {'ours':>9} {'bf16':>9}  name")
    for row in rows[:40]:
        print(f"{row[0]:7.3f} {row[2]:10.3e} {row[3]:9.2e} {row[4]:9.2e}  {row[1]}")


if __name__ == "__main__":
    gan() if "--gan" in sys.argv else c4()
