"""ctypes binding of lib/libvonoma.so (the C ABI declared in include/vonoma.h).

The product path has NO fallback: if the library is missing or cannot be loaded,
every op raises.  Build it with ``make -C visual_onoma_to_wave_amd -j8`` (or
``python -c "import __graft_entry__ as g; g.build()"``).
"""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VO_LIB_PATH: an alternative build of the same library (A/B timing of two kernel builds in
# tools/); the product path loads lib/libvonoma.so
LIB_PATH = os.environ.get("VO_LIB_PATH") or os.path.join(_HERE, "lib", "libvonoma.so")

VO_F32, VO_BF16, VO_F32X3 = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_LRELU, ACT_TANH = 0, 1, 2, 3
PACK_CONV, PACK_CONVT = 0, 1
HEAD_DURATION, HEAD_ENERGY = 0, 1

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float
c_int64 = ctypes.c_int64


class Conv1dDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("x_dtype", c_int), ("x_bstride", c_int64), ("ldx", c_int),
        ("w", c_void_p), ("bias", c_void_p),
        ("y", c_void_p), ("y_dtype", c_int), ("y_bstride", c_int64), ("ldy", c_int),
        ("res1", c_void_p), ("res2", c_void_p),
        ("B", c_int), ("T_in", c_int), ("T_out", c_int),
        ("Ci", c_int), ("Co", c_int),
        ("K", c_int), ("dil", c_int), ("pad", c_int),
        ("pre_act", c_int), ("pre_slope", c_float),
        ("post_act", c_int), ("post_slope", c_float),
        ("out_scale", c_float),
        ("compute_dtype", c_int),
        ("transposed", c_int), ("up_stride", c_int), ("up_pad", c_int), ("up_cout", c_int),
        ("up_tout", c_int),
        ("variant", c_int),
        ("stride", c_int), ("groups", c_int),
        ("workspace", c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("ymask", c_void_p), ("ymask_slope", c_float),
    ]


class PackJob(ctypes.Structure):
    """VoPackJob (include/vonoma.h, vo_pack_batch)."""
    _fields_ = [("src", c_void_p), ("dst", c_void_p)] + [
        (f, c_int) for f in ("mode", "swap", "T", "rows", "width", "dst_rows", "ld", "rpg", "cpg", "cig", "K", "tap0",
                             "tstep", "src_rows")]


class RemapJob(ctypes.Structure):
    """VoRemapJob (include/vonoma.h, vo_seq_remap2)."""
    _fields_ = [("src", c_void_p), ("src2", c_void_p), ("dst", c_void_p)] + [
        (f, ctypes.c_int64) for f in ("src_rows", "src2_rows", "dst_rows", "Ss", "Ss2")] + [
        (f, c_int) for f in ("Td", "lo", "hi", "shift", "shift2")]


class GanTerm(ctypes.Structure):
    """VoGanTerm (include/vonoma.h, vo_gan_reduce_multi / vo_gan_reduce_grad_multi)."""
    _fields_ = [("kind", c_int), ("a", c_void_p), ("lda", c_int), ("b", c_void_p), ("ldb", c_int),
                ("rows", ctypes.c_int64), ("width", c_int), ("ga", c_void_p), ("ldg", c_int)]


class SnBwdLayer(ctypes.Structure):
    """VoSnBwdLayer (include/vonoma.h, vo_spectral_norm_bwd)."""
    _fields_ = [(f, c_void_p) for f in ("g", "W", "u", "v", "sigma", "gW")] + [("rows", c_int), ("L", c_int)]


class SnLayer(ctypes.Structure):
    """VoSnLayer (include/vonoma.h, vo_spectral_norm)."""
    _fields_ = [(f, c_void_p) for f in ("W", "u", "v", "u_out", "v_out", "vraw", "s", "sigma", "w")] + [
        ("rows", c_int), ("L", c_int)]


class HeadDesc(ctypes.Structure):
    _fields_ = [
        ("kind", c_int),
        ("h", c_void_p), ("h_dtype", c_int),
        ("w", c_void_p), ("b", c_float),
        ("lens", c_void_p),
        ("B", c_int), ("T", c_int), ("D", c_int),
        ("pred", c_void_p),
        ("d_round", c_void_p), ("d_control", c_float),
        ("target", c_void_p),
        ("bins", c_void_p), ("n_bins", c_int),
        ("e_mean", c_float), ("e_std", c_float), ("e_control", c_float),
        ("table", c_void_p),
        ("x", c_void_p), ("x_dtype", c_int),
        ("idx_out", c_void_p),
    ]


_SIGNATURES = {
    "vo_last_error": (ctypes.c_char_p, []),
    "vo_version": (c_int, []),
    "vo_num_symbols": (c_int, []),
    "vo_symbol_name": (ctypes.c_char_p, [c_int]),
    "vo_tune": (c_int, [ctypes.c_char_p, c_int]),
    "vo_resblock_pair": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                 c_int, c_int, c_int, c_int, c_float, c_float, c_void_p]),
    "vo_resblock_pair_frag": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_int, c_int, c_int, c_int, c_float, c_float, c_void_p]),
    "vo_pack_frag": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "vo_resblock3": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                             c_int, c_int, c_float, c_float, c_void_p]),
    "vo_conv1d": (c_int, [ctypes.POINTER(Conv1dDesc), c_void_p]),
    "vo_conv1d_workspace_size": (ctypes.c_int64, [ctypes.POINTER(Conv1dDesc)]),
    "vo_pack_weight": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                               c_void_p, c_int, c_void_p]),
    "vo_layernorm": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                             c_int, c_int, c_float, c_void_p, c_int, c_void_p]),
    "vo_layernorm_dual": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                  c_int, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    "vo_layernorm_bwd_workspace_size": (ctypes.c_int64, [c_int, c_int, c_int]),
    "vo_layernorm_bwd": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                                 c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_layernorm_bwd_ex": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "vo_layernorm_drop": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                  c_int, c_float, c_void_p, c_int, c_void_p, c_float, c_void_p, ctypes.c_uint,
                                  c_void_p]),
    "vo_layernorm_bwd_drop": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                      c_void_p, c_int, c_int, c_int, c_float, c_float, c_void_p, ctypes.c_uint,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_attention": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float,
                             c_void_p, c_void_p]),
    "vo_attention_bwd_workspace_size": (ctypes.c_int64, [c_int, c_int, c_int]),
    "vo_attention_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                 c_void_p, c_void_p, c_void_p]),
    "vo_attention_lse": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                                 c_void_p]),
    "vo_attention_bwd_lse": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                     c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_length_regulate": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                   c_int, c_void_p, c_void_p, c_void_p]),
    "vo_length_regulate_bwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p]),
    "vo_lr_lengths": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "vo_variance_head": (c_int, [ctypes.POINTER(HeadDesc), c_void_p]),
    "vo_bucket_embed": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, ctypes.c_int64,
                                c_int, c_void_p, c_void_p, c_void_p]),
    "vo_adam_multi": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                              c_float, c_float, c_float, c_int, c_void_p]),
    "vo_opt_step_increment": (c_int, [c_void_p, c_void_p]),
    "vo_embed_bwd": (c_int, [c_void_p, c_int, c_void_p, ctypes.c_int64, c_int, c_int, c_void_p, c_void_p]),
    "vo_vfe_stencil": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_int, c_void_p, c_int, c_void_p]),
    "vo_add_pos_class": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                 c_int, c_void_p]),
    "vo_mask_from_lengths": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "vo_conv_post": (c_int, [c_void_p, c_int, c_void_p, c_float, c_int, c_int, c_int, c_int, c_float,
                             c_void_p, c_void_p]),
    "vo_transpose_bct": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "vo_stft_mel": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_float,
                            c_void_p, c_void_p, c_void_p]),
    "vo_stft_mel_ex": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                               c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_conv1d_wgrad_workspace_size": (c_int64, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "vo_conv1d_wgrad": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p, c_void_p]),
    "vo_conv1d_wgrad_grouped": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p,
                                        c_void_p, c_void_p]),
    "vo_conv1d_wgrad_bias": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "vo_lrelu_mask": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, ctypes.c_int64, c_int, c_float,
                              c_void_p, c_int, c_void_p]),
    "vo_colsum_workspace_size": (c_int64, [c_int64, c_int]),
    "vo_colsum": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "vo_char_features": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    "vo_pack_grouped": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "vo_pack_grouped_blocks": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "vo_period_fold": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "vo_wav_cl8": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "vo_avgpool_wav": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "vo_period_fold_bwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "vo_wav_cl8_bwd": (c_int, [c_void_p, c_int, c_int64, c_void_p, c_void_p]),
    "vo_avgpool_wav_bwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "vo_pack_dgrad_phase": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_void_p, c_int, c_void_p]),
    "vo_pack_batch": (c_int, [c_int, c_void_p, c_int, c_void_p]),
    "vo_lrelu_mask_add": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int64, c_int,
                                  c_float, c_void_p, c_int, c_void_p]),
    "vo_lrelu_mask_sum": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int64, c_int,
                                  c_float, c_void_p, c_int, c_void_p]),
    "vo_spectral_norm": (c_int, [c_int, c_void_p, c_int, c_float, c_void_p]),
    "vo_gan_reduce_multi": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_gan_reduce_multi_workspace_size": (c_int64, [c_int]),
    "vo_gan_reduce_grad_multi": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "vo_spectral_norm_bwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p]),
    "vo_spectral_norm_bwd_workspace_size": (c_int64, [c_int, c_void_p]),
    "vo_seq_remap": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int64, c_int, c_int, c_int, c_void_p]),
    "vo_seq_remap2": (c_int, [c_int, c_void_p, c_int, c_int, c_void_p]),
    "vo_weight_norm": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_weight_norm_bwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "vo_gan_reduce": (c_int, [c_int, c_void_p, c_int, c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_void_p,
                              c_void_p]),
    "vo_gan_reduce_grad": (c_int, [c_int, c_void_p, c_int, c_void_p, c_int, c_int64, c_int, c_int, c_void_p,
                                   c_void_p, c_int, c_void_p]),
    "vo_bn_workspace_size": (ctypes.c_int64, [c_int, c_int]),
    "vo_bn_train_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_float, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_bn_bwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p, c_void_p]),
    "vo_dropout": (c_int, [c_void_p, c_int, c_int64, c_float, c_void_p, ctypes.c_uint, c_void_p, c_void_p]),
    "vo_vfe_conv_workspace_size": (ctypes.c_int64, [c_int, c_int, c_int]),
    "vo_vfe_conv_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "vo_vfe_conv_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p]),
    "vo_stft_mel_bwd_workspace_size": (ctypes.c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "vo_stft_mel_bwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_stft_mag": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p]),
    "vo_stft_mag_bwd_workspace_size": (ctypes.c_int64, [c_int, c_int, c_int, c_int]),
    "vo_stft_mag_bwd": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    "vo_stft_loss": (c_int, [c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p]),
    "vo_stft_loss_grad": (c_int, [c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vo_glyph_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                               c_int, c_int, c_void_p, c_void_p]),
}

ABI_VERSION = 2  # include/vonoma.h VO_ABI_VERSION
_lib = None


def lib():
    """Load libvonoma.so once; raise (no fallback) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"visual_onoma_to_wave_amd: HIP library not built ({LIB_PATH} missing); run "
                "`make -C visual_onoma_to_wave_amd -j8` -- there is no CPU fallback")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.vo_version() != ABI_VERSION:  # the signatures above are those of this ABI version
            raise RuntimeError(f"visual_onoma_to_wave_amd: {LIB_PATH} has ABI version {handle.vo_version()}, "
                               f"the bindings expect {ABI_VERSION} (include/vonoma.h VO_ABI_VERSION); rebuild it")
        _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().vo_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")
