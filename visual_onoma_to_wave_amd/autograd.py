"""Autograd wrappers for the training path (config C4, scripts/04_train.py:128-141).

The forward of every op is the same HIP kernel the inference path runs.  Backward:

* Conv1d / Linear input-gradient: HIP -- the conv kernel itself over dY with the weights
  re-packed taps-reversed / channels-swapped (``vo_pack_weight`` mode DGRAD);
* Conv1d / Linear weight and bias gradients: HIP -- ``vo_conv1d_wgrad`` (MFMA, fragments
  read transposed from LDS) and ``vo_colsum``;
* LayerNorm backward: HIP -- ``vo_layernorm_bwd`` (row-wise input gradient, deterministic
  gamma / beta column sums);
* attention backward: HIP -- ``vo_attention_bwd`` (flash-style: the row log-sum-exp is rebuilt
  from q / k, dQ and dK / dV in two MFMA kernels, nothing of size L x L stored);
* LengthRegulator backward: HIP -- ``vo_length_regulate_bwd`` (segmented frame sums per token,
  deterministic);
* training-mode BatchNorm (PostNet, glyph encoder) forward / backward and the glyph encoder's
  3 x 3 conv forward / backward: HIP -- ``vo_bn_*`` and ``vo_vfe_conv_*`` (train_glue.hip).

All functions take and return channels-last (B, T, C) activations.
"""

import os
import weakref

import torch
import torch.nn.functional as F

from . import ops

# ---------------------------------------------------------------------------- step-batched weight packs
# Every conv of the training forward packs its weight ([K][Co][Ci], compute dtype) and its backward the
# taps-reversed input-gradient layout ([K][Ci][Co]); packed one launch per layer and layout that was
# ~100 launches of 4-7 us per C4 step.  Instead each (weights, compute dtype) the step uses keeps
# persistent pack buffers here, and the first look-up at new parameter versions (after an optimizer
# step, or in each HIP-graph replay) re-packs EVERY stale layout of the store in one vo_pack_batch call
# per dtype (its job table: 32 packs per launch).  The fused q/k/v projection's weights are written by
# three jobs into one [768][256] buffer (no torch.cat per step).  VO_C4_PREPACK=0: per-call packs (A/B).
PREPACK = os.environ.get("VO_C4_PREPACK", "1") != "0"
STATS = {"batches": 0, "packs": 0}


class _PackEntry:
    __slots__ = ("refs", "cdt", "Co", "Ci", "K", "buf", "ver", "need_dgrad")

    def __init__(self, params, cdt):
        self.refs, self.cdt = tuple(weakref.ref(p) for p in params), cdt  # the store keeps no model alive
        self.Co = sum(p.shape[0] for p in params)
        self.Ci = params[0].shape[1]
        self.K = params[0].shape[2] if params[0].dim() == 3 else 1
        self.buf, self.ver, self.need_dgrad = {}, {}, False

    @property
    def params(self):
        return tuple(r() for r in self.refs)

    def alive(self):
        return all(r() is not None for r in self.refs)

    def version(self):
        return tuple(p._version for p in self.params)

    def jobs(self, kind):
        """vo_pack_batch jobs (src, dst, fields, offset) writing this layout from every source."""
        K, Ci, Co = self.K, self.Ci, self.Co
        dst = self.buf[kind]
        out, row0 = [], 0
        for p in self.params:
            co = p.shape[0]
            src = p.detach()
            if kind == "fwd":  # dst[k][r0 + co][ci] = src[co][ci][k]
                f = dict(mode=ops.PJ_GATHER, swap=0, T=K, rows=co, width=Ci, dst_rows=Co, ld=Ci, rpg=co, cpg=0,
                         cig=Ci, K=K, tap0=0, tstep=1, src_rows=co)
                out.append((src, dst, f, row0 * Ci))
            else:  # dgrad: dst[K-1-k][ci][r0 + co] = src[co][ci][k]
                f = dict(mode=ops.PJ_GATHER, swap=1, T=K, rows=Ci, width=co, dst_rows=Ci, ld=Co, rpg=Ci, cpg=0,
                         cig=Ci, K=K, tap0=K - 1, tstep=-1, src_rows=co)
                out.append((src, dst, f, row0))
            row0 += co
        return out


_STORES = ({}, {})  # [capturing]: packs made inside a graph capture live in the graph's own store
# every (weights, dtype) a step has packed, and whether its backward wanted the dgrad layout: a store that
# is empty after reset_packs() is seeded with all of them at its first look-up, so that the step's first
# conv re-packs every layout of the step in one batch (inside a graph capture too: entries discovered one
# conv at a time each packed alone, ~100 launches per captured C4 step)
_KNOWN = {}


def _store():
    return _STORES[1 if torch.cuda.is_current_stream_capturing() else 0]


def reset_packs():
    """Forget every step-batched pack: before and after a graph capture (the capture re-packs inside the
    graph, so every replay packs the weights it is about to read), and after each replay (replays move the
    parameters without bumping their version counters: an eager step afterwards must re-pack)."""
    for st in _STORES:
        st.clear()


def _seed(store):
    for key, (refs, cdt, dgrad) in list(_KNOWN.items()):
        params = tuple(r() for r in refs)
        if any(p is None for p in params):
            del _KNOWN[key]
            continue
        e = store[key] = _PackEntry(params, cdt)
        e.need_dgrad = dgrad


def _packed_weight(params, cdt, kind):
    """The ``kind`` ("fwd" | "dgrad") layout of the conv whose weight is ``params`` concatenated along
    C_out (fp32 (Co_i, Ci, K) or (Co_i, Ci) parameters), packed for compute dtype ``cdt``."""
    store = _store()
    key = (tuple(id(p) for p in params), cdt)
    if not store:
        _seed(store)
    e = store.get(key)
    if e is None or any(a is not b for a, b in zip(e.params, params)):  # new, or ids of dead parameters reused
        e = store[key] = _PackEntry(params, cdt)
        _KNOWN[key] = (e.refs, cdt, False)
    if kind == "dgrad" and not e.need_dgrad:
        e.need_dgrad = True
        _KNOWN[key] = (e.refs, cdt, True)
    if e.ver.get(kind) != e.version():
        _refresh(store)
    return e.buf[kind]


def _refresh(store):
    """Re-pack every stale layout of the store: one vo_pack_batch call per dtype."""
    per_dtype = {}
    for k in [k for k, e in store.items() if not e.alive()]:
        del store[k]
    for e in store.values():
        ver = e.version()
        for kind in ("fwd", "dgrad") if e.need_dgrad else ("fwd",):
            if e.ver.get(kind) == ver:
                continue
            if kind not in e.buf:
                dev = e.params[0].device
                shape = (e.K, e.Co, e.Ci) if kind == "fwd" else (e.K, e.Ci, e.Co)
                e.buf[kind] = torch.empty(shape, dtype=e.cdt, device=dev)
            per_dtype.setdefault(e.cdt, []).extend(e.jobs(kind))
            e.ver[kind] = ver
            STATS["packs"] += 1
    for cdt, jobs in per_dtype.items():
        ops.pack_batch(jobs, cdt)
        STATS["batches"] += 1


def _params_of(w):
    """The fp32 parameter(s) behind a conv weight argument (a Linear's weight[:, :, None] view -> the
    Linear's weight), or None when it is not a plain contiguous fp32 tensor."""
    base = w
    if w._base is not None and w.dim() == 3 and w.shape[2] == 1:
        # only exactly base[:, :, None]: a view that slices Ci or starts at an offset would be packed
        # from the whole base and keyed on its id
        base = w._base
        if tuple(base.shape) != tuple(w.shape[:2]) or w.data_ptr() != base.data_ptr():
            return None
    if base.dtype != torch.float32 or not base.is_contiguous() or base.shape[0] != w.shape[0]:
        return None
    return (base,)


class Conv1dFn(torch.autograd.Function):
    """y = post(conv1d(x, w, b, K, dil, pad)), post in {none, relu}; x (B, T, Ci), w (Co, Ci, K)."""

    @staticmethod
    def forward(ctx, x, w, b, K, dil, pad, relu, compute_dtype, out_dtype, bias_before_bn=False):
        Co = w.shape[0]
        src = _params_of(w) if PREPACK else None
        sd = ops.storage_dtype(compute_dtype)  # ops.F32X3: fp32 tensors and packed weights
        wp = _packed_weight(src, sd, "fwd") if src else ops.pack_conv_weight(w, sd)
        y = ops.conv1d(x.contiguous(), wp, b.detach().float().contiguous() if b is not None else None, Co=Co,
                       K=K, dil=dil, pad=pad, post_act=ops.ACT_RELU if relu else ops.ACT_NONE,
                       out_dtype=out_dtype, compute_dtype=compute_dtype)
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.cfg = (K, dil, pad, relu, compute_dtype, b is not None, bias_before_bn)
        ctx.bias_like = b.detach() if (b is not None and bias_before_bn) else None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        K, dil, pad, relu, cdt, has_b, bias_before_bn = ctx.cfg
        gz = gy.contiguous()
        if relu:
            gz = ops.lrelu_mask(gz, y, 0.0)
        gx = gw = gb = None
        want_b = has_b and ctx.needs_input_grad[2]
        if want_b and bias_before_bn:
            # the output feeds a train-mode BatchNorm, whose batch mean subtracts any per-channel constant: the
            # bias gradient is exactly 0 (the column sums of dY cancel); computed as 0, not as the rounding noise
            # of 16 k bf16 terms
            gb = torch.zeros_like(ctx.bias_like)
            want_b = False
        sd = ops.storage_dtype(cdt)
        if ctx.needs_input_grad[0]:
            src = _params_of(w) if PREPACK else None
            wd = _packed_weight(src, sd, "dgrad") if src else ops.pack_dgrad_weight(w, sd)
            gx = ops.conv1d(gz.to(sd) if gz.dtype != sd else gz, wd, None, Co=w.shape[1], K=K, dil=dil,
                            pad=(K - 1) * dil - pad, T_out=x.shape[1], out_dtype=x.dtype, compute_dtype=cdt)
        if ctx.needs_input_grad[1]:
            if x.dtype in (torch.float32, torch.bfloat16) and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
                # MFMA weight gradient over transposed LDS reads (vo_conv1d_wgrad), in the forward's
                # compute dtype (an fp32 activation feeding a bf16 conv -- PostNet after its fp32
                # BatchNorm -- was contracted in bf16 by the forward too)
                fuse_b = want_b and gz.dtype == sd  # bias = column sums of the same dY (no cast)
                r = ops.conv1d_wgrad(gz.to(sd).contiguous(), x.to(sd).contiguous(), K, dil=dil, pad=pad,
                                     with_bias=fuse_b, split=cdt is ops.F32X3)
                if fuse_b:
                    r, gb = r
                gw = r.to(w.dtype)
            else:
                gw = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), w.shape, gz.float().transpose(1, 2),
                                                 padding=pad, dilation=dil)
        if want_b and gb is None:
            gb = ops.colsum(gz.contiguous())
        return gx, gw, gb, None, None, None, None, None, None, None


def conv1d(x, w, b, K=1, dil=1, pad=0, relu=False, compute_dtype=torch.bfloat16, out_dtype=None, bias_before_bn=False):
    """bias_before_bn: the output feeds a train-mode BatchNorm (PostNet): the bias gradient is exactly 0."""
    return Conv1dFn.apply(x, w, b, K, dil, pad, relu, compute_dtype, out_dtype or x.dtype, bias_before_bn)


def linear(x, weight, bias, relu=False, compute_dtype=torch.bfloat16, out_dtype=None):
    return conv1d(x, weight[:, :, None], bias, 1, 1, 0, relu, compute_dtype, out_dtype)


class QKVLinearFn(torch.autograd.Function):
    """The fused q / k / v projection (SubLayers.py:39-41 as one GEMM): x (B, L, D) -> (B, L, 3D) with
    the three Linears' weights packed side by side by the step's pack batch (no per-step torch.cat of
    the weights); the backward splits dW and db back onto the three Linears."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, bq, bk, bv, compute_dtype):
        params = (wq, wk, wv)
        wp = _packed_weight(params, ops.storage_dtype(compute_dtype), "fwd")
        b = torch.cat([bq.detach(), bk.detach(), bv.detach()]).float()
        y = ops.conv1d(x.contiguous(), wp, b, Co=wp.shape[1], K=1, compute_dtype=compute_dtype,
                       out_dtype=x.dtype)
        ctx.save_for_backward(x, wq, wk, wv)
        ctx.cdt = compute_dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wq, wk, wv = ctx.saved_tensors
        cdt = ctx.cdt
        sd = ops.storage_dtype(cdt)
        gz = gy.contiguous()
        gz = gz.to(sd) if gz.dtype != sd else gz
        gx = None
        if ctx.needs_input_grad[0]:
            wd = _packed_weight((wq, wk, wv), sd, "dgrad")
            gx = ops.conv1d(gz, wd, None, Co=wq.shape[1], K=1, T_out=x.shape[1], out_dtype=x.dtype,
                            compute_dtype=cdt)
        fuse_b = gy.dtype == sd  # bias = column sums of the same dY (no cast), as Conv1dFn
        r = ops.conv1d_wgrad(gz, x.to(sd).contiguous(), 1, with_bias=fuse_b, split=cdt is ops.F32X3)
        gw, gb = r if fuse_b else (r, ops.colsum(gy.contiguous()))
        gw = gw.to(wq.dtype).reshape(gw.shape[0], gw.shape[1])
        n = wq.shape[0]
        return (gx, gw[:n], gw[n:2 * n], gw[2 * n:], gb[:n], gb[n:2 * n], gb[2 * n:], None)


def qkv_linear(x, wq, wk, wv, bq, bk, bv, compute_dtype):
    if not PREPACK:
        w = torch.cat([wq, wk, wv], 0)
        b = torch.cat([bq, bk, bv], 0)
        return linear(x, w, b, compute_dtype=compute_dtype)
    return QKVLinearFn.apply(x, wq, wk, wv, bq, bk, bv, compute_dtype)


class AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, lens, n_head):
        # the row log-sum-exp is kept for the backward (B x H x L fp32): it need not rebuild it
        out, lse = ops.attention(qkv.contiguous(), lens, n_head, with_lse=True)
        ctx.save_for_backward(qkv, lens, out, lse)
        ctx.n_head = n_head
        return out

    @staticmethod
    def backward(ctx, go):
        qkv, lens, out, lse = ctx.saved_tensors
        return ops.attention_bwd(qkv.contiguous(), out, go.to(qkv.dtype).contiguous(), lens, ctx.n_head,
                                 lse=lse), None, None


def attention(qkv, lens, n_head):
    return AttentionFn.apply(qkv, lens, n_head)


class LayerNormFn(torch.autograd.Function):
    """LN(x + res) * g + b with pad rows (t >= lens[b]) zeroed (FFTBlock.masked_fill)."""

    @staticmethod
    def forward(ctx, x, res, g, b, lens):
        ctx.save_for_backward(x, res, g, b, lens)
        return ops.layernorm(x.contiguous(), g.detach().float().contiguous(), b.detach().float().contiguous(),
                             res=res.contiguous() if res is not None else None, lens=lens)

    @staticmethod
    def backward(ctx, gy):
        x, res, g, b, lens = ctx.saved_tensors
        xr = x.contiguous()
        rr = res.contiguous() if res is not None else None
        if rr is not None and rr.dtype != xr.dtype:
            rr = rr.to(xr.dtype)
        gh, gg, gb = ops.layernorm_bwd(xr, gy.contiguous(), g.detach().float().contiguous(), res=rr, lens=lens)
        gr = (gh if res.dtype == gh.dtype else gh.to(res.dtype)) if res is not None else None
        return gh, gr, gg.to(g.dtype), gb.to(b.dtype), None


def layernorm(x, res, g, b, lens=None):
    return LayerNormFn.apply(x, res, g, b, lens)


class LayerNormDualFn(torch.autograd.Function):
    """The mixed training decoder's LayerNorm (round 6): y = LN(x + res) * g + b (pad rows zeroed) with a
    bf16 sublayer output x and the fp32 residual stream res; returns (y fp32 -- the next residual --, its
    bf16 copy y16 -- what the next conv reads and saves).  Forward and backward are one kernel each
    (vo_layernorm_dual / vo_layernorm_bwd_ex: the two incoming gradients are added in the kernel)."""

    @staticmethod
    def forward(ctx, x, res, g, b, lens):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, res, g, lens)
        return ops.layernorm(x.contiguous(), g.detach().float().contiguous(), b.detach().float().contiguous(),
                             res=res.contiguous(), lens=lens, out_dtype=torch.float32, with_bf16=True)

    @staticmethod
    def backward(ctx, gy, gy16):
        x, res, g, lens = ctx.saved_tensors
        if gy is None and gy16 is None:
            return None, None, None, None, None
        if gy is None:  # only the copy was read (the last layer feeds mel_linear its y16)
            gy, gy16 = gy16, None
        gy2 = None if gy16 is None else gy16.contiguous()
        if gy2 is not None and gy2.dtype != torch.bfloat16:
            gy, gy2 = gy + gy2.to(gy.dtype), None
        gh, gh32, gg, gb = ops.layernorm_bwd_ex(x.contiguous(), gy.contiguous(), g.detach().float().contiguous(),
                                                res.contiguous(), lens=lens, gy2=gy2)
        return gh, gh32, gg.to(g.dtype), gb.to(g.dtype), None


def layernorm_dual(x, res, g, b, lens=None):
    return LayerNormDualFn.apply(x, res, g, b, lens)


class LayerNormDropFn(torch.autograd.Function):
    """The training FFT block's sublayer dropout fused into the LayerNorm after it (round 6): y = LN(dropout_p(x) +
    res) * g + b, pad rows zeroed; x the sublayer output (before its dropout), res the residual stream.  dual
    (fp32 res, bf16 compute): returns (y fp32, its bf16 copy y16) as LayerNormDualFn; else y in res's dtype.  The
    mask is vo_dropout's for the same (seed, salt) -- recomputed in the backward kernel, no mask tensor."""

    @staticmethod
    def forward(ctx, x, res, g, b, lens, p, seed, salt, dual):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, res, g, lens, seed)
        ctx.p, ctx.salt, ctx.dual = p, salt, dual
        return ops.layernorm_drop(x.contiguous(), g.detach().float().contiguous(), b.detach().float().contiguous(),
                                  res.contiguous(), p, seed, salt, lens=lens, with_bf16=dual)

    @staticmethod
    def backward(ctx, *grads):
        x, res, g, lens, seed = ctx.saved_tensors
        gy, gy16 = (grads[0], grads[1]) if ctx.dual else (grads[0], None)
        if gy is None and gy16 is None:
            return (None,) * 9
        if gy is None:  # only the copy was read (the last decoder layer feeds mel_linear its y16)
            gy, gy16 = gy16, None
        gy2 = None if gy16 is None else gy16.contiguous()
        if gy2 is not None and (gy2.dtype != torch.bfloat16 or gy.dtype != torch.float32):
            gy, gy2 = gy.float() + gy2.float(), None
        gh, gres, gg, gb = ops.layernorm_bwd_drop(x.contiguous(), gy.contiguous(), g.detach().float().contiguous(),
                                                  res.contiguous(), ctx.p, seed, ctx.salt, lens=lens, gy2=gy2)
        return gh, gres, gg.to(g.dtype), gb.to(g.dtype), None, None, None, None, None


def layernorm_drop(x, res, g, b, lens, p, dual):
    """LN(dropout_p(x) + res) in one kernel each way; dual: (y fp32, y16) as layernorm_dual."""
    seed, salt = _dropout_seed_salt(x.device)
    return LayerNormDropFn.apply(x, res, g, b, lens, float(p), seed, salt, dual)


class DropoutFn(torch.autograd.Function):
    """Training dropout on HIP (vo_dropout): the keep mask is a hash of (seed, site, element index), so
    the backward re-applies it to the gradient from the saved seed -- no mask tensor."""

    @staticmethod
    def forward(ctx, x, p, seed, salt):
        ctx.p, ctx.salt = p, salt
        ctx.save_for_backward(seed)
        return ops.dropout(x, p, seed, salt)

    @staticmethod
    def backward(ctx, gy):
        (seed,) = ctx.saved_tensors
        g = gy.contiguous()
        if g.data_ptr() % 16:
            g = g.clone()
        return ops.dropout(g, ctx.p, seed, ctx.salt), None, None, None


_DROP = {"seed": None, "site": 0}


def begin_dropout_step(device):
    """Draw the step's dropout seed (one int64 from torch's generator, on the device: graph-safe, every
    replay of a captured step draws anew); the step's dropout sites then salt it with their call index.
    Without it each dropout call draws its own seed (one more small kernel per call)."""
    _DROP["seed"] = torch.randint(1, 2 ** 62, (1,), device=device, dtype=torch.int64)
    _DROP["site"] = 0


def dropout(x, p, training=True):
    """F.dropout(x, p, training) for the training forward (scripts/transformer/SubLayers.py:38,87,
    scripts/transformer/Layers.py:129-131, scripts/model/modules.py:52-56): masks differ per step and
    per call as with F.dropout (the draws differ from ATen's)."""
    if not training or p == 0.0:
        return x
    if p == 1.0:  # F.dropout's exact zeros (x * 0 would turn Inf / NaN inputs into NaN)
        return x.masked_fill(torch.ones((), dtype=torch.bool, device=x.device), 0.0)
    xc = x.contiguous()
    if xc.data_ptr() % 16:
        xc = xc.clone()
    seed, salt = _dropout_seed_salt(x.device)
    return DropoutFn.apply(xc, float(p), seed, salt)


def _dropout_seed_salt(device):
    """(device seed, salt) of the next dropout site: the step's seed salted by the site's index, or a fresh seed
    when no step seed is set (begin_dropout_step)."""
    seed = _DROP["seed"]
    if seed is None or seed.device != device:
        return torch.randint(1, 2 ** 62, (1,), device=device, dtype=torch.int64), 0
    _DROP["site"] = _DROP["site"] + 1
    return seed, _DROP["site"]


class LengthRegulateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dur, max_len, out_dtype):
        out, mel_len, _ = ops.length_regulate(x.contiguous(), dur, int(max_len), out_dtype=out_dtype)
        ctx.save_for_backward(dur)
        ctx.shape = x.shape
        ctx.xdtype = x.dtype
        ctx.mark_non_differentiable(mel_len)
        return out, mel_len

    @staticmethod
    def backward(ctx, go, _gm):
        (dur,) = ctx.saved_tensors
        return ops.length_regulate_bwd(go.contiguous(), dur, ctx.shape[1], out_dtype=ctx.xdtype), None, None, None


class BatchNormTrainFn(torch.autograd.Function):
    """nn.BatchNorm* in training mode on HIP (``vo_bn_train_fwd`` / ``vo_bn_bwd``): batch
    statistics per channel, the running-stat update (momentum, unbiased running variance,
    ``num_batches_tracked`` += 1) done by the finalize kernel on the device -- nothing on the
    host, so the step stays graph-capturable."""

    @staticmethod
    def forward(ctx, x, weight, bias, bn):
        xc = x.contiguous()
        track = bn.track_running_stats and bn.running_mean is not None
        y, mr = ops.bn_train_fwd(xc, weight, bias, bn.eps, bn.momentum,
                                 bn.running_mean if track else None, bn.running_var if track else None,
                                 bn.num_batches_tracked if track else None)
        ctx.save_for_backward(xc, weight, mr)
        ctx.has_affine = weight is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, mr = ctx.saved_tensors
        dx, dg, db = ops.bn_bwd(x, gy.contiguous(), w, mr)
        if not ctx.has_affine:
            dg = db = None
        return dx, dg, db, None


def batch_norm_train(x, bn, dims):
    """Training-mode BatchNorm over ``dims`` (batch statistics; the channel is the one dim left):
    channels-last (B, T, C) with dims (0, 1) -- PostNet, no transposes -- or a single-channel
    (N, 1, H, W) map with dims (0, 2, 3) -- the glyph encoder."""
    if bn.momentum is None:
        raise NotImplementedError("batch_norm_train: cumulative-average BatchNorm (momentum=None)")
    if not ((x.dim() == 3 and tuple(dims) == (0, 1)) or (x.dim() == 4 and tuple(dims) == (0, 2, 3) and
                                                           x.shape[1] == 1)):
        raise NotImplementedError(f"batch_norm_train: layout {tuple(x.shape)} over dims {dims}")
    if bn.affine:
        return BatchNormTrainFn.apply(x, bn.weight, bn.bias, bn)
    return BatchNormTrainFn.apply(x, None, None, bn)


class VfeConvFn(torch.autograd.Function):
    """The glyph encoder's Conv2d(1, 1, 3, padding=1) (``vo_vfe_conv_fwd`` / ``vo_vfe_conv_bwd``)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        w10 = torch.cat([weight.detach().reshape(-1).float(), bias.detach().reshape(-1).float()])
        xc = x.contiguous()
        ctx.save_for_backward(xc, w10)
        ctx.wshape = weight.shape
        return ops.vfe_conv_fwd(xc, w10)

    @staticmethod
    def backward(ctx, gy):
        x, w10 = ctx.saved_tensors
        dx, dw = ops.vfe_conv_bwd(x, gy.contiguous(), w10)
        return dx, dw[:9].view(ctx.wshape), dw[9:]


def vfe_conv(x, conv):
    if conv.weight.shape != (1, 1, 3, 3) or conv.bias is None or conv.padding != (1, 1) or conv.stride != (1, 1):
        raise NotImplementedError("vfe_conv: the HIP path covers Conv2d(1, 1, 3, padding=1) with bias")
    return VfeConvFn.apply(x, conv.weight, conv.bias)


def length_regulate(x, dur, max_len, out_dtype=None):
    return LengthRegulateFn.apply(x, dur, max_len, out_dtype or x.dtype)


class BucketEmbedFn(torch.autograd.Function):
    """x + Embedding(table)[bucketize(target, bins)] (scripts/model/modules.py:53-64,101-104, teacher
    forced): forward vo_bucket_embed, backward dx = dy and dtable by vo_embed_bwd (row-ordered sums)."""

    @staticmethod
    def forward(ctx, x, table, target, bins):
        out, idx = ops.bucket_embed(x.contiguous(), target, bins.detach().float().contiguous(),
                                    table.detach().float().contiguous())
        ctx.save_for_backward(idx)
        ctx.n_table = table.shape[0]
        ctx.table_dtype = table.dtype
        ctx.mark_non_differentiable(idx)
        return out, idx

    @staticmethod
    def backward(ctx, go, _gi):
        (idx,) = ctx.saved_tensors
        dt = ops.embed_bwd(go.contiguous(), idx, ctx.n_table) if ctx.needs_input_grad[1] else None
        return go, (dt.to(ctx.table_dtype) if dt is not None else None), None, None


def bucket_embed(x, embedding, target, bins):
    """``x + embedding(torch.bucketize(target, bins))`` on HIP, differentiable in x and the table."""
    return BucketEmbedFn.apply(x, embedding.weight, target, bins)[0]
