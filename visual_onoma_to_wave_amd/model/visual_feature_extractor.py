"""Visual-glyph encoder front (reference: scripts/model/visual_feature_extractor.py:5-83).

The strip (B, 1, 24, 102*T) is cut into T character slices by the kernel grid itself
(no Python slicing loop, no stacked copies); each slice runs 3 x [Conv2d 3x3 (1 -> 1
channel) -> BatchNorm2d(eval) -> ReLU] in LDS (``vo_vfe_stencil``), then the bridge
Linear(2448 -> 256) + ReLU runs as a K=1 MFMA conv over all B*T slices at once.
"""

import torch
import torch.nn as nn

from .. import ops
from .._base import HipModule, fold_bn


class VisualFeatureExtractor(HipModule):
    def __init__(self, load_scale, slice_width, slice_height, embed_dim, stride, embed_normalize=True,
                 bridge_relu=True, kernel_size=(3, 3), num_convolutions=1):
        super().__init__()
        self.load_scale = load_scale
        self.dim3 = {"gray-scale": 1, "RGB-scale": 3}[load_scale]
        self.slice_width, self.slice_height = slice_width, slice_height
        self.embed_dim, self.stride = embed_dim, stride
        self.embed_normalize, self.bridge_relu = embed_normalize, bridge_relu
        kh, kw = kernel_size
        self.kernel_size = (slice_height, kw) if kh == -1 else (kh, kw)
        if self.kernel_size[0] % 2 == 0 or self.kernel_size[1] % 2 == 0:
            raise AssertionError(f"conv2d kernel {self.kernel_size} must be odd in both dims")
        self.num_convolutions = num_convolutions
        layers = []
        for _ in range(num_convolutions):
            layers.append(nn.Conv2d(self.dim3, self.dim3, kernel_size=self.kernel_size, stride=1,
                                    padding=((kh - 1) // 2, (kw - 1) // 2)))
            if embed_normalize:
                layers.append(nn.BatchNorm2d(self.dim3))
            layers.append(nn.ReLU(inplace=True))
        self.embedder = nn.Sequential(*layers)
        lin = nn.Linear(slice_width * stride * slice_height * self.dim3, embed_dim)
        self.bridge = nn.Sequential(lin, nn.ReLU(inplace=True)) if bridge_relu else lin
        for p in self.parameters():
            nn.init.uniform_(p, -0.08, 0.08)

    def _supported(self):
        if not (self.dim3 == 1 and self.stride == 1 and self.kernel_size == (3, 3) and
                self.embed_normalize and self.bridge_relu):
            raise NotImplementedError("the HIP VFE covers the ICASSP configuration (gray-scale, stride 1, "
                                      "3x3 kernels, BatchNorm, bridge ReLU)")

    def _build(self, device, dtype):
        convs, bns = [], []
        for m in self.embedder:
            if isinstance(m, nn.Conv2d):
                convs.append(torch.cat([m.weight.detach().float().reshape(-1), m.bias.detach().float()]))
            elif isinstance(m, nn.BatchNorm2d):
                s, sh = fold_bn(m)
                bns.append(torch.cat([s, sh]))
        lin = self.bridge[0]
        d = dict(conv=torch.stack(convs).to(device).contiguous(),
                 bn=torch.stack(bns).to(device).contiguous(),
                 w=ops.pack_conv_weight(lin.weight.to(device)[:, :, None], dtype),
                 b=lin.bias.detach().float().to(device).contiguous())
        # the bridge is a 2448-deep reduction over only B * n rows: as one conv each workgroup
        # walks 77 channel chunks in series (90 us at B = 32).  Split-K instead: S channel groups
        # as a grouped conv (group g = input channels [g Ci/S, (g+1) Ci/S) -> its own E outputs),
        # then the S partial sums are added in order (deterministic) -> 5 chunks per workgroup.
        E, Ci = lin.weight.shape
        S = next((s for s in (17, 16, 12, 8, 4, 2) if Ci % s == 0 and (Ci // s) % 8 == 0), 1)
        if S > 1:
            wg = lin.weight.detach().float().to(device).view(E, S, Ci // S).transpose(0, 1).reshape(S * E, Ci // S)
            d.update(split=S, wsplit=ops.pack_grouped_weight(wg[:, :, None], dtype, groups=S))
        return d

    def run(self, images, out_dtype=None):
        self._supported()
        p = self._packed(images.device, self._build)
        flat, n = ops.vfe_stencil(images, p["conv"], p["bn"], self.slice_width, self.compute_dtype)
        B = images.shape[0]
        E = self.embed_dim
        if p.get("split", 1) > 1 and flat.shape[0] <= 4096:
            S = p["split"]
            part = ops.conv1d(flat.unsqueeze(0), p["wsplit"], None, Co=S * E, K=1, groups=S,
                              out_dtype=torch.float32, compute_dtype=self.compute_dtype)
            y = torch.relu(part.view(-1, S, E).sum(1) + p["b"]).to(out_dtype or self.compute_dtype)
            return y.view(B, n, E)
        y = ops.conv1d(flat.unsqueeze(0), p["w"], p["b"], Co=E, K=1,
                       post_act=ops.ACT_RELU, out_dtype=out_dtype or self.compute_dtype,
                       compute_dtype=self.compute_dtype)
        return y.view(B, n, E)

    def train_run(self, images, out_dtype):
        """Training forward (BatchNorm2d uses batch statistics, so the eval-folded stencil kernel
        does not apply): the slices gathered into (B n, 1, 24, 102) maps, then conv (vo_vfe_conv),
        BatchNorm with batch statistics (vo_bn_train_fwd), ReLU, and the bridge on HIP."""
        from .. import autograd as AG
        B, C, H, W = images.shape
        n = int((W - (self.stride // 2) * self.slice_width * 2) / self.slice_width)
        sl = images[..., : n * self.slice_width].reshape(B, C, H, n, self.slice_width)
        x = sl.permute(0, 3, 1, 2, 4).reshape(B * n, C, H, self.slice_width)
        self._supported()
        for m in self.embedder:
            if isinstance(m, nn.BatchNorm2d):
                x = AG.batch_norm_train(x, m, (0, 2, 3))
            elif isinstance(m, nn.ReLU):
                x = torch.relu(x)
            else:
                x = AG.vfe_conv(x, m)
        y = AG.linear(x.reshape(1, B * n, -1).to(out_dtype), self.bridge[0].weight, self.bridge[0].bias,
                      relu=True, compute_dtype=out_dtype)
        return y.view(B, n, self.embed_dim)

    def forward(self, images):
        self._check_inference()
        return self.run(images)
