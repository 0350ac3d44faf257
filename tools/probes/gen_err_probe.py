#!/usr/bin/env python3
"""Where the bf16 Generator's error comes from: the HIP path run stage by stage (conv_pre, each
upsampler, each MRF, conv_post), each stage's LOCAL error = HIP stage on the HIP input against the
fp32 oracle stage on that same input, beside the oracle's own CPU bf16-autocast local error, at the
reference's default init (tests/test_gpu_parity.py::test_generator_bf16_reference_init).

Like with like (round 4): the autocast reference gets the stage input as a bf16 TENSOR (the HIP
stage's input is bf16 in HBM).  Given an fp32 tensor, the autocast ResBlock's residual ``xt + x``
promoted to fp32 and its residual stream stayed fp32 through the stage, while the HIP kernels (and
the autocast reference inside a whole-Generator run, where every stage input comes out of a bf16
conv) keep it in bf16.

    python tools/probes/gen_err_probe.py [seed]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
from helpers import hifigan_h, rel_l2  # noqa: E402
from oracle import vocoder as V  # noqa: E402
from visual_onoma_to_wave_amd import hifigan, ops  # noqa: E402
from visual_onoma_to_wave_amd.hifigan.models import LRELU_SLOPE  # noqa: E402


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    h = hifigan_h()
    torch.manual_seed(seed)
    g = hifigan.Generator(hifigan.AttrDict(h))
    sd = V.fold_weight_norm({k: v.detach().clone() for k, v in g.state_dict().items()})
    g.eval()
    g.remove_weight_norm()
    g = g.cuda()
    g.set_compute_dtype(torch.bfloat16)
    gc = torch.Generator().manual_seed(100 + seed)
    mel = torch.clamp(torch.randn(2, 80, 96, generator=gc) * 2.0 - 5.0, -11.513, 2.5)
    dt = torch.bfloat16
    p = g._packed(torch.device("cuda"), g._build)

    def cl(x):  # (B, T, C) cuda -> (B, C, T) cpu fp32
        return x.float().cpu().transpose(1, 2).contiguous()

    def line(name, hip, ref32, ref16):
        print(f"{name:10s} local rel-L2: HIP bf16 {rel_l2(hip, ref32):.2e}   oracle bf16-autocast "
              f"{rel_l2(ref16, ref32):.2e}   |x| {float(ref32.abs().max()):.3g}", flush=True)

    def auto(fn, *a):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            return fn(*a).float()

    with torch.no_grad():
        mel_cl = ops.transpose_bct(mel.cuda(), torch.float32)
        w, b = p["pre"]
        x = ops.conv1d(mel_cl, w, b, Co=w.shape[1], K=7, pad=3, out_dtype=dt, compute_dtype=dt)
        pre = lambda m: torch.nn.functional.conv1d(m, sd["conv_pre.weight"], sd["conv_pre.bias"], padding=3)  # noqa
        line("conv_pre", cl(x), pre(mel), auto(pre, mel))
        for i in range(g.num_upsamples):
            xin = cl(x)
            wu, bu, cout, u, pad = p["ups"][i]
            x = ops.conv1d(x, wu, bu, Co=u * cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=LRELU_SLOPE,
                           transposed=dict(stride=u, pad=pad, cout=cout), out_dtype=dt, compute_dtype=dt)
            k = h["upsample_kernel_sizes"][i]
            line(f"ups{i}", cl(x), V.upsample(sd, i, xin, k, u), auto(V.upsample, sd, i, xin.to(dt), k, u))
            xin = cl(x)
            x = g.mrf(i, x)
            line(f"mrf{i}", cl(x), V.mrf(sd, i, xin, h), auto(V.mrf, sd, i, xin.to(dt), h))
            # each ResBlock alone (local), through the same dispatch as the MRF
            nk = g.num_kernels
            for j in range(nk):
                rb = g.resblocks[i * nk + j]
                rb.compute_dtype = dt
                out = torch.empty_like(x)
                rb.run(xin.transpose(1, 2).contiguous().to(dt).cuda(), out=out, out_scale=1.0)
                key = f"resblocks.{i * nk + j}"
                rk, rd = h["resblock_kernel_sizes"][j], h["resblock_dilation_sizes"][j]
                xin16 = xin.to(dt).float()
                line(f"  rb{j} k{rk}", cl(out), V.resblock(sd, key, xin16, rk, rd),
                     auto(V.resblock, sd, key, xin16.to(dt), rk, rd))
        wk, bp = p["post"]
        xin = cl(x)
        wav = ops.conv_post(x, wk, bp, slope=0.01)

        def post(z):
            z = torch.nn.functional.leaky_relu(z)
            return torch.tanh(torch.nn.functional.conv1d(z, sd["conv_post.weight"], sd["conv_post.bias"], padding=3))
        line("conv_post", wav.float().cpu().reshape(2, 1, -1), post(xin), auto(post, xin.to(dt)))
        ref = V.generator(sd, mel, h)
        print(f"end to end: HIP {rel_l2(wav.float().cpu().reshape(ref.shape), ref):.2e}   oracle bf16-autocast "
              f"{rel_l2(auto(V.generator, sd, mel, h), ref):.2e}")


if __name__ == "__main__":
    main()
