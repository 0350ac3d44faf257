"""Deterministic, realistically scaled parameters for parity tests.

Pretrained checkpoints are not available offline, so every golden vector is
produced with weights drawn here from ``numpy.random.default_rng(seed)``, walking
the state-dict keys in order.  The same function fills the reference model (in
``make_goldens.py``, in the survey container only) and this package's model (in
the tests, here and on the GPU box), so the weights are regenerated, never stored.

Key-name rules (keys and shapes are the reference's checkpoint layout,
SURVEY.md section 8(b)):

* ``position_enc``, ``*_bins``      -> left to the module (computed at init)
* ``num_batches_tracked``           -> 0
* ``running_mean`` / ``running_var``-> N(0, 0.1) / U(0.5, 1.5)
* norm ``weight`` / ``bias``        -> 1 + N(0, 0.1) / N(0, 0.1)
* embedding ``weight``              -> N(0, 1)          (torch default init)
* conv / linear ``weight`` / ``bias`` -> U(-1/sqrt(fan_in), +1/sqrt(fan_in))
* weight-norm ``weight_v`` / ``weight_g`` -> v ~ N(0, 1); g = per-slice gain
  (1 for Conv1d, sqrt(C_out * stride / C_in) for ConvTranspose1d) * U(0.8, 1.2),
  so the folded weight keeps activations O(1) through the vocoder.
"""

import numpy as np

def _is_norm(key, shape):
    if "layer_norm" in key:
        return True
    if "postnet.convolutions." in key and ".1." in key:
        return True
    if "VisualFeatureExtractor.embedder." in key:
        idx = int(key.split("embedder.")[1].split(".")[0])
        return idx % 3 == 1
    return False


def make_state_dict(spec, seed, ups_strides=None):
    """spec: ordered list of (key, shape, dtype-str). Returns {key: np.ndarray}."""
    rng = np.random.default_rng(seed)
    out = {}
    ups_strides = ups_strides or {}
    shapes = {k: tuple(s) for k, s, _ in spec}
    for key, shape, dtype in spec:
        shape = tuple(shape)
        leaf = key.rsplit(".", 1)[-1]
        if key.endswith("position_enc") or key.endswith("_bins"):
            continue
        if leaf == "num_batches_tracked":
            out[key] = np.zeros(shape, dtype=np.int64)
            continue
        if leaf == "running_mean":
            out[key] = rng.normal(0.0, 0.1, size=shape).astype(np.float32)
            continue
        if leaf == "running_var":
            out[key] = rng.uniform(0.5, 1.5, size=shape).astype(np.float32)
            continue
        if _is_norm(key, shape):
            if leaf == "weight":
                out[key] = (1.0 + rng.normal(0.0, 0.1, size=shape)).astype(np.float32)
            else:
                out[key] = rng.normal(0.0, 0.1, size=shape).astype(np.float32)
            continue
        if "emb" in key and leaf == "weight":
            out[key] = rng.normal(0.0, 1.0, size=shape).astype(np.float32)
            continue
        if leaf == "weight_v":
            out[key] = rng.normal(0.0, 1.0, size=shape).astype(np.float32)
            continue
        if leaf == "weight_g":
            prefix = key[: -len("weight_g")]
            if prefix.startswith("ups."):
                i = int(prefix.split(".")[1])
                s = ups_strides.get(i, 1)
                # ConvTranspose1d v: (C_in, C_out, k); norm over all dims but 0
                vshape = shapes[prefix + "weight_v"]
                cin, cout = vshape[0], vshape[1]
                gain = np.sqrt(cout * s / cin)
            else:
                gain = 1.0
            out[key] = (gain * rng.uniform(0.8, 1.2, size=shape)).astype(np.float32)
            continue
        # conv / linear weight and bias
        if leaf == "weight":
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            bound = 1.0 / np.sqrt(fan_in)
            out[key] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
            continue
        if leaf == "bias":
            prefix = key[: -len("bias")]
            wshape = shapes.get(prefix + "weight", shapes.get(prefix + "weight_v"))
            if prefix + "weight_v" in shapes:
                bound = 0.05
            elif wshape is not None and len(wshape) > 1:
                bound = 1.0 / np.sqrt(int(np.prod(wshape[1:])))
            else:
                bound = 0.1
            out[key] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
            continue
        raise KeyError(f"no generation rule for {key} {shape}")
    return out


def spec_of(state_dict):
    """(key, shape, dtype) list from a torch state dict (any implementation)."""
    return [(k, tuple(v.shape), str(v.dtype)) for k, v in state_dict.items()]


def load_into(module, arrays):
    """Copy generated arrays into a torch module (strict on the generated keys)."""
    import torch
    sd = module.state_dict()
    missing = [k for k in arrays if k not in sd]
    if missing:
        raise KeyError(f"generated keys missing in module: {missing[:5]}")
    with torch.no_grad():
        for k, a in arrays.items():
            t = torch.from_numpy(np.array(a, copy=True, order="C"))
            if tuple(sd[k].shape) != tuple(t.shape):
                raise ValueError(f"shape mismatch for {k}: {tuple(sd[k].shape)} vs {tuple(t.shape)}")
            sd[k].copy_(t)
    return module


HIFIGAN_UPS_STRIDES = {0: 8, 1: 8, 2: 2, 3: 2}
