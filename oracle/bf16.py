"""ORACLE (test infrastructure only) -- the reference's arithmetic at bf16, two ways.

The parity bar of a bf16 HIP result is the oracle's own drift when it runs at bf16 (helpers.bf16_bar).
Two equally valid bf16 arithmetics of the same functions:

* ``autocast``: torch's CPU bf16 autocast -- contractions on bf16 operands with their OUTPUTS rounded
  to bf16, every following op (norms, activations) on bf16 tensors;
* ``operands`` (``bf16_operands`` below): every dense contraction (conv1d / conv2d / conv_transpose1d /
  linear / bmm) rounds its two operands to bf16 and accumulates in fp32 -- the rounding of an MFMA
  kernel -- and everything else stays fp32.

Their drifts differ from each other by 5-20 % per gradient where the gradient is dominated by the
forward's rounding (L1-loss sign flips, BatchNorm batch statistics): the spread of the reference's own
bf16 arithmetic, which the gradient tests take as their bar.
"""

import contextlib

import torch
import torch.nn.functional as F


class _Shim:
    """A module stand-in: the names in ``over`` replaced, everything else from ``base``."""

    def __init__(self, base, over):
        self._base, self._over = base, over

    def __getattr__(self, k):
        return self._over[k] if k in self._over else getattr(self._base, k)


def _r(t):
    return t.to(torch.bfloat16).float() if torch.is_tensor(t) and t.is_floating_point() else t


def _two(f):
    def g(x, w, *a, **k):
        return f(_r(x), _r(w), *a, **k)
    return g


@contextlib.contextmanager
def bf16_operands(*modules):
    """Inside the block, the oracle ``modules`` (e.g. oracle.acoustic, oracle.vocoder) evaluate their
    dense contractions on bf16-rounded operands with fp32 accumulation; biases and all other ops fp32."""
    over_f = {n: _two(getattr(F, n)) for n in ("conv1d", "conv2d", "conv_transpose1d", "linear")}
    over_t = {"bmm": _two(torch.bmm)}
    saved = []
    for m in modules:
        saved.append((m, m.F, getattr(m, "torch", None)))
        m.F = _Shim(F, over_f)
        if hasattr(m, "torch"):
            m.torch = _Shim(torch, over_t)
    try:
        yield
    finally:
        for m, f, t in saved:
            m.F = f
            if t is not None:
                m.torch = t
