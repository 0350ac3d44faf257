"""Shared machinery of the HIP-backed nn.Modules.

Each module keeps its parameters in the reference's checkpoint layout (same attribute
names, shapes and state-dict keys) and, on first use on a device, packs them once into
the layout its kernels read (``[K][Co][Ci]``, BatchNorm / weight-norm folded, fused
QKV ...).  The pack is cached per (device, compute dtype) and rebuilt only when a
parameter's version counter moves (load_state_dict, optimizer step) or a HIP-graph replay
has updated the parameters (``invalidate_packs``).

Precision ("compute dtype") is a per-module attribute:
  * torch.float32  -- exact-f32 MFMA everywhere (the parity mode);
  * torch.bfloat16 -- bf16 MFMA with fp32 accumulation, bf16 activations in HBM.
``vTTS.set_precision("mixed")`` (the default) keeps the encoder and variance adaptor in
fp32 -- their outputs feed the discontinuous bucketize / round steps (SURVEY.md section 7,
hard part 1) -- and runs the decoder, PostNet and vocoder in bf16.
"""

import torch
import torch.nn as nn

_GENERATION = [0]


def invalidate_packs(*modules):
    """Drop the packed-weight caches of ``modules`` (and their HIP submodules); with no argument,
    of every module in the process.  HIP-graph replays of a training step update parameters in
    place without bumping their version counters, so the graphed steps call this for the modules
    they train after each replay (and after capture) -- inference modules living in the same
    process (a vocoder, a SynthesisPipeline) keep their packs."""
    if not modules:
        _GENERATION[0] += 1
        return
    for root in modules:
        for m in root.modules():
            if isinstance(m, HipModule):
                m.__dict__["_pack_gen"] = m.__dict__.get("_pack_gen", 0) + 1


class HipModule(nn.Module):
    compute_dtype = torch.bfloat16

    def _params_version(self):
        return tuple(p._version for p in self.parameters()) + tuple(
            b._version for b in self.buffers())

    def _packed(self, device, builder, dtype=None):
        dtype = dtype or self.compute_dtype
        key = (str(device), dtype, _GENERATION[0], self.__dict__.get("_pack_gen", 0), self._params_version())
        cache = self.__dict__.setdefault("_pack_cache", {})
        hit = cache.get("key")
        if hit != key:
            cache.clear()
            cache["key"] = key
            with torch.no_grad():
                cache["val"] = builder(device, dtype)
        return cache["val"]

    f32_split = False

    @property
    def contract_dtype(self):
        """The compute dtype the training path's contractions run in: ops.F32X3 (split-bf16 over fp32
        tensors) for an fp32 module set to f32_split, else compute_dtype."""
        from . import ops
        return ops.F32X3 if (self.f32_split and self.compute_dtype == torch.float32) else self.compute_dtype

    def set_compute_dtype(self, dtype, f32_split=False):
        """f32_split: an fp32 module's TRAINING contractions (train_run) as split-bf16 (ops.F32X3);
        inference (run) stays exact fp32."""
        for m in self.modules():
            if isinstance(m, HipModule):
                m.compute_dtype = dtype
                m.f32_split = bool(f32_split)
        return self

    def _check_inference(self):
        if self._training_path():
            raise NotImplementedError(
                f"{type(self).__name__}.forward: training runs through vTTS.forward (train_run path)")

    def _training_path(self):
        """True when autograd must record the op graph (train mode with grad enabled)."""
        return self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())


def fold_bn(bn):
    """Eval-mode BatchNorm as (scale, shift): y = x * scale + shift."""
    scale = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
    shift = bn.bias.detach().float() - bn.running_mean.detach().float() * scale
    return scale, shift
