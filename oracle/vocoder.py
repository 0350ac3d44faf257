"""ORACLE (test infrastructure only) -- HiFi-GAN V1 generator restated on the CPU.

Functional fp32 PyTorch-CPU restatement of scripts/hifigan/models.py over a
reference-layout state dict (weight-norm ``weight_g``/``weight_v`` or folded
``weight`` keys).
"""

import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1  # scripts/hifigan/models.py:7


def fold_weight_norm(sd):
    """remove_weight_norm, scripts/hifigan/models.py:105-109,167-174:
    w = g * v / ||v||, the norm over every dim except 0 (C_out for Conv1d,
    C_in for ConvTranspose1d)."""
    out = {}
    for k, v in sd.items():
        if k.endswith("weight_v"):
            p = k[: -len("weight_v")]
            g = sd[p + "weight_g"]
            norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
            out[p + "weight"] = g * v / norm
        elif k.endswith("weight_g"):
            continue
        else:
            out[k] = v
    return out


def get_padding(k, d=1):
    """scripts/hifigan/models.py:16-17."""
    return int((k * d - d) / 2)


def resblock(sd, p, x, k, dilations=(1, 3, 5)):
    """ResBlock.forward (ResBlock1), scripts/hifigan/models.py:96-103."""
    for i, d in enumerate(dilations):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = F.conv1d(xt, sd[f"{p}.convs1.{i}.weight"], sd[f"{p}.convs1.{i}.bias"],
                      padding=get_padding(k, d), dilation=d)
        xt = F.leaky_relu(xt, LRELU_SLOPE)
        xt = F.conv1d(xt, sd[f"{p}.convs2.{i}.weight"], sd[f"{p}.convs2.{i}.bias"],
                      padding=get_padding(k, 1))
        x = xt + x
    return x


def upsample(sd, i, x, k, u):
    """lrelu(0.1) -> ConvTranspose1d(k, stride u, padding (k-u)//2), models.py:124-135,152-153."""
    x = F.leaky_relu(x, LRELU_SLOPE)
    return F.conv_transpose1d(x, sd[f"ups.{i}.weight"], sd[f"ups.{i}.bias"], stride=u,
                              padding=(k - u) // 2)


def mrf(sd, i, x, h):
    """Multi-receptive-field fusion of upsampling stage i: the mean of its num_kernels ResBlocks,
    scripts/hifigan/models.py:155-160."""
    nk = len(h["resblock_kernel_sizes"])
    xs = None
    for j, (rk, rd) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
        r = resblock(sd, f"resblocks.{i * nk + j}", x, rk, rd)
        xs = r if xs is None else xs + r
    return xs / nk


def generator(sd, mel, h):
    """Generator.forward, scripts/hifigan/models.py:149-165 (folded weights)."""
    x = F.conv1d(mel, sd["conv_pre.weight"], sd["conv_pre.bias"], padding=3)
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = upsample(sd, i, x, k, u)
        x = mrf(sd, i, x, h)
    x = F.leaky_relu(x)  # default slope 0.01, models.py:161
    x = F.conv1d(x, sd["conv_post.weight"], sd["conv_post.bias"], padding=3)
    return torch.tanh(x)
