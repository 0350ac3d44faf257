/* vonoma.h -- C ABI of the MI355X (gfx950) synthesis-path kernels.
 *
 * Drop-in boundary for the reference's visual-onomatopoeia -> mel -> waveform path
 * (sarulab-speech/visual-onoma-to-wave).  The reference is pure PyTorch: every op on
 * its path is an implicit ATen kernel launched from the nn.Modules cited below.  Each
 * entry point here replaces those ATen calls for one reference function; the Python
 * host layer (visual_onoma_to_wave_amd/, same module/class names as the reference)
 * binds them through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - plain device pointers and sizes; all buffers are caller-owned (no allocation
 *    inside, no host synchronisation: every call is stream-ordered and graph-capturable);
 *  - `stream` is a hipStream_t passed as void*; NULL = the default stream;
 *  - return 0 (VO_OK) on success, VO_ERR_INVALID on a rejected argument, or the
 *    hipError_t of a failed launch; vo_last_error() describes the last failure;
 *  - activations are channels-last ("(B, T, C)", C contiguous) -- the layout the
 *    reference's transformer side already uses (scripts/transformer/SubLayers.py:85-93
 *    transposes to (B, C, T) only to call Conv1d) and the one whose 8 consecutive
 *    channels form one MFMA operand fragment;
 *  - element types: VO_F32 or VO_BF16 for tensor I/O; VO_BF16 compute = bf16 MFMA with
 *    fp32 accumulation, VO_F32 compute = exact-f32 MFMA (the parity mode), VO_F32X3 compute
 *    (fp32 I/O and fp32 packed weights, stride 1, no groups) = split-bf16 contractions: each
 *    fp32 operand as hi + lo bf16, three bf16 MFMAs per product (<= 3 * 2^-18 relative error
 *    per product: fp32-class, not bit-exact fp32; the mixed-precision training step's fp32 side).
 */
#ifndef VONOMA_H_
#define VONOMA_H_

#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define VO_OK 0
#define VO_ERR_INVALID (-1)

enum vo_dtype { VO_F32 = 0, VO_BF16 = 1, VO_F32X3 = 2 /* compute only */ };
enum vo_act { VO_ACT_NONE = 0, VO_ACT_RELU = 1, VO_ACT_LRELU = 2, VO_ACT_TANH = 3 };

/* ------------------------------------------------------------------ runtime */
const char* vo_last_error(void);
/* ABI version of this header; vo_version() returns the library's.  A binding checks they are equal
 * at load time.  2 (round 4): vo_bucket_embed gained n_table (before n), vo_conv1d_desc gained
 * ymask / ymask_slope at its end -- a version-1 binding would pass shifted arguments or leave the
 * new fields uninitialised. */
#define VO_ABI_VERSION 2
int vo_version(void);
/* number of entry points and their names (used by the loader test) */
int vo_num_symbols(void);
const char* vo_symbol_name(int i);
/* kernel-variant knobs for A/B experiments ("pair_cfg", "conv_cfg"; default 0 = shipped
 * configuration); returns VO_OK or VO_ERR_INVALID for an unknown key */
int vo_tune(const char* key, int value);

/* ------------------------------------------------------------------ conv1d (implicit GEMM)
 * y[b, t, co] = post( sum_{k, ci} W[k][co][ci] * pre(x[b, t*1 + k*dil - pad, ci]) + bias[co] )
 *               (+ res1) * out_scale (+ res2)
 * Replaces: nn.Conv1d in PositionwiseFeedForward (scripts/transformer/SubLayers.py:60-93),
 *   PostNet ConvNorm+BatchNorm1d (scripts/transformer/Layers.py:33-137, BN folded),
 *   VariancePredictor Conv (scripts/model/modules.py:216-259), nn.Linear as K=1
 *   (SubLayers.py:18-26, vtts.py:23-26, visual_feature_extractor.py:49-55),
 *   HiFi-GAN conv_pre / ResBlock convs with the lrelu prologue and residual epilogue
 *   (scripts/hifigan/models.py:96-103,150,155-160).
 * transposed != 0: ConvTranspose1d(stride=s, padding=p, K_t = 2s) in its polyphase form
 *   (scripts/hifigan/models.py:124-135,153): W holds the 2-tap phase weights packed by
 *   vo_pack_weight(..., VO_PACK_CONVT, ...), co spans s*C_out phase-major columns and output
 *   row m lands at time m*s - p + phase.
 */
typedef struct vo_conv1d_desc {
  const void* x;      /* input (B, T_in, ldx) channels-last, dtype x_dtype            */
  int x_dtype;
  int64_t x_bstride;  /* elements between batches (usually T_in * ldx)               */
  int ldx;            /* elements between rows (>= Ci, multiple of 8)                */
  const void* w;      /* packed weights [K][Co][Ci], dtype = compute dtype            */
  const float* bias;  /* [Co] or NULL                                                 */
  void* y;            /* output, dtype y_dtype                                        */
  int y_dtype;
  int64_t y_bstride;
  int ldy;
  const void* res1;   /* optional, same layout and dtype as y                        */
  const void* res2;   /* optional, same layout and dtype as y (may alias y)          */
  int B, T_in, T_out; /* T_out = output rows (for transposed: T_in + 1 phase rows)   */
  int Ci, Co;         /* Co = GEMM columns (transposed: s * C_out)                    */
  int K, dil, pad;
  int pre_act;  float pre_slope;
  int post_act; float post_slope;
  float out_scale;
  int compute_dtype;  /* VO_BF16, VO_F32 or VO_F32X3 */
  int transposed, up_stride, up_pad, up_cout, up_tout; /* polyphase ConvTranspose1d */
  int variant;        /* 0 = generic; 1..4 = HiFi-GAN MRF stage 0..3 (bf16 I/O): a kernel
                         instantiation of its own, so profiles attribute the stages   */
  int stride;         /* 0/1 = 1; 2..4: output row o reads input rows o*stride + k*dil - pad
                         (HiFi-GAN MPD Conv2d (k,1)/(s,1) per period column, MSD Conv1d)  */
  int groups;         /* 0/1 = dense; g: grouped conv, w packed dense [K][Co][Ci] with zeros
                         outside the g diagonal blocks (MSD grouped Conv1d)              */
  void* workspace;    /* optional caller-owned device scratch (NULL = none): when it holds
                         vo_conv1d_workspace_size(d) bytes, fp32 convs over short sequences
                         (T_out <= 16: glyph encoder, variance predictors) split their
                         reduction over workgroups and add the fp32 partials in a fixed
                         order (deterministic)                                           */
  int64_t workspace_bytes;
  const void* ymask;  /* optional, y's layout and dtype (bf16 y, no bias / residual / activation):
                         each output is stored as round(round(v) * (ymask > 0 ? 1 : ymask_slope))
                         -- an input gradient masked by the leaky-ReLU output it flows into, as
                         vo_lrelu_mask would mask it (HiFi-GAN discriminators, D step)          */
  float ymask_slope;
} vo_conv1d_desc;
int vo_conv1d(const vo_conv1d_desc* d, void* stream);
/* scratch bytes the split-reduction path of vo_conv1d wants for d (0 = it does not split d) */
int64_t vo_conv1d_workspace_size(const vo_conv1d_desc* d);

/* Weight preparation (load time).  Replaces the weight-norm fold (remove_weight_norm,
 * scripts/hifigan/models.py:105-109,167-174: w = g * v / ||v||, norm over all dims but 0)
 * and the eval-mode BatchNorm fold of PostNet / VFE (Layers.py:129-137), and writes the
 * [K][Co][Ci] compute layout.
 *   mode VO_PACK_CONV : src (Co, Ci, K) -> dst [K][Co][Ci]
 *   mode VO_PACK_CONVT: src (Ci, Co, 2s) (ConvTranspose1d) -> dst [2][s*Co][Ci],
 *                       dst[kk][r*Co + co][ci] = src[ci][co][r + s*(1-kk)]
 *   mode VO_PACK_DGRAD: src (Co, Ci, K) -> dst [K][Ci][Co], dst[K-1-k][ci][co] = src[co][ci][k]
 *                       (the input-gradient of a conv is the conv of dY with these weights,
 *                       padding (K-1)*dil - pad)
 * g (nullable): weight-norm gains, one per src dim-0 slice; row_scale (nullable): per-Co
 * multiplier (BatchNorm gamma / sqrt(var + eps)). */
enum vo_pack_mode { VO_PACK_CONV = 0, VO_PACK_CONVT = 1, VO_PACK_DGRAD = 2 };
int vo_pack_weight(const float* src, const float* g, const float* row_scale, int mode, int Co,
                   int Ci, int K, int stride, void* dst, int dst_dtype, void* stream);

/* ------------------------------------------------------------------ layer norm
 * y[r, :] = LayerNorm(x[r, :] + res[r, :]) * gamma + beta, then zeroed where row r is padding
 * (t >= lens[b], r = b*T + t; lens may be NULL).  eps 1e-5.
 * Replaces: MultiHeadAttention/PositionwiseFeedForward post-LN + residual
 * (scripts/transformer/SubLayers.py:55,91) and FFTBlock.masked_fill (Layers.py:25,28);
 * VariancePredictor LN (modules.py:197-206) with res = NULL, lens = NULL. */
int vo_layernorm(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                 const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y,
                 int y_dtype, void* stream);

/* vo_layernorm with an fp32 y and, in the same pass, its bf16 copy y16 (round to nearest even;
 * pad rows 0 in both).  The mixed-precision decoder keeps its residual stream (y) in fp32, as the
 * reference's bf16 autocast does, while the next conv reads y16 -- the same bits that conv's own
 * fp32 -> bf16 staging would make, at half the bytes.  x / res: both fp32, both bf16, or (round 6,
 * the training decoder: bf16 sublayer output + fp32 residual stream) bf16 x with fp32 res. */
int vo_layernorm_dual(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                      const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y,
                      void* y16, void* stream);

/* Backward of vo_layernorm (training, config C4): gh = dL/d(x + res) (the gradient of both x
 * and res; 0 on pad rows), dgamma / dbeta (fp32, D) summed over the unmasked rows.  x / res /
 * gh share x_dtype.  workspace: vo_layernorm_bwd_workspace_size(B, T, D) bytes (per-workgroup
 * partial column sums, added in a fixed order: deterministic).
 * Replaces: the autograd of nn.LayerNorm + masked_fill (scripts/transformer/SubLayers.py:55,91,
 * scripts/transformer/Layers.py:25,28) under scripts/04_train.py:128-141. */
int64_t vo_layernorm_bwd_workspace_size(int B, int T, int D);
int vo_layernorm_bwd(const void* x, const void* res, int x_dtype, const void* gy, int gy_dtype,
                     const float* gamma, const int32_t* lens, int B, int T, int D, float eps, void* gh,
                     float* dgamma, float* dbeta, void* workspace, void* stream);

/* vo_layernorm_bwd for the backward of vo_layernorm_dual (round 6, mixed-precision training): res may be
 * fp32 beside a bf16 x (res_dtype), gy2 (bf16, may be NULL) is a second incoming gradient -- that of
 * y16 -- added to gy, and gh32 (may be NULL) receives the fp32 gradient of res beside gh (x_dtype).
 * Combinations: bf16 x + fp32 res with fp32 or bf16 gy; or x_dtype == res_dtype with gy2 = gh32 = NULL
 * (then exactly vo_layernorm_bwd).  Same workspace. */
int vo_layernorm_bwd_ex(const void* x, int x_dtype, const void* res, int res_dtype, const void* gy, int gy_dtype,
                        const void* gy2, const float* gamma, const int32_t* lens, int B, int T, int D, float eps,
                        void* gh, float* gh32, float* dgamma, float* dbeta, void* workspace, void* stream);

/* Training FFT blocks (round 6): the sublayer output's dropout (scripts/transformer/SubLayers.py:51,88) fused
 * into the LayerNorm that follows it.  Forward: y = LN(dropout(x) + res) * gamma + beta (pad rows 0), element i
 * of x kept iff it is kept by vo_dropout(p, seed, salt) on the same tensor, scaled by 1 / (1 - p); y16 (may be
 * NULL; fp32 y only) its bf16 copy.  x / res / y: fp32 / fp32 / fp32, bf16 / fp32 / fp32, bf16 / bf16 / bf16.
 * Backward: gh = dL/dx (through the mask, x_dtype), gres = dL/dres (res_dtype), gy2 (bf16, may be NULL) the
 * gradient of y16 added to gy; dgamma / dbeta as vo_layernorm_bwd (same workspace).  B*T*D < 2^32. */
int vo_layernorm_drop(const void* x, int x_dtype, const void* res, int res_dtype, const float* gamma,
                      const float* beta, const int32_t* lens, int B, int T, int D, float eps, void* y, int y_dtype,
                      void* y16, float p, const int64_t* seed, unsigned salt, void* stream);
int vo_layernorm_bwd_drop(const void* x, int x_dtype, const void* res, int res_dtype, const void* gy, int gy_dtype,
                          const void* gy2, const float* gamma, const int32_t* lens, int B, int T, int D, float eps,
                          float p, const int64_t* seed, unsigned salt, void* gh, void* gres, float* dgamma,
                          float* dbeta, void* workspace, void* stream);

/* ------------------------------------------------------------------ attention
 * Scaled dot-product attention with key padding, H heads of d_k = D/H, over the fused
 * qkv activations (B, L, 3D) (columns [q | k | v], head h at h*d_k) -> out (B, L, D)
 * (head-concat columns h*d_k + d).  Keys t >= lens[b] are masked (-inf before softmax).
 * Replaces: MultiHeadAttention split/permute + ScaledDotProductAttention
 * (scripts/transformer/SubLayers.py:39-53, scripts/transformer/Modules.py:14-25).  The
 * probabilities are never materialised (the reference returns them but no caller uses
 * them: Models.py:119-124, 190-195). */
int vo_attention(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                 float scale, void* out, void* stream);

/* Backward of vo_attention (training, config C4): dqkv (B, L, 3D) = [dQ | dK | dV] in the
 * qkv layout, from qkv, the forward output out (B, L, D) and its gradient dout (B, L, D), all in
 * `dtype`.  Flash-style: the row log-sum-exp is rebuilt from qkv, no L x L tensor is stored.
 * workspace: vo_attention_bwd_workspace_size(B, L, H) bytes.  Masked keys get zero dK / dV.
 * Replaces: the autograd of SubLayers.py:39-53 / Modules.py:14-25 under
 * scripts/04_train.py:128-141. */
int64_t vo_attention_bwd_workspace_size(int B, int L, int H);
int vo_attention_bwd(const void* qkv, const void* out, const void* dout, int dtype, const int32_t* lens, int B,
                     int L, int H, int dk, float scale, void* dqkv, void* workspace, void* stream);
/* vo_attention that also writes the row log-sum-exp lse (B, H, L) fp32 (+inf for a row with no key),
 * and the backward that consumes it (bf16: no pass over the keys to rebuild it; every product formed
 * transposed so P / dS stay in registers; fp32: as vo_attention_bwd).  Same reference as above. */
int vo_attention_lse(const void* qkv, int dtype, const int32_t* lens, int B, int L, int H, int dk,
                     float scale, void* out, float* lse, void* stream);
int vo_attention_bwd_lse(const void* qkv, const void* out, const void* dout, int dtype, const int32_t* lens, int B,
                         int L, int H, int dk, float scale, const float* lse, void* dqkv, void* workspace,
                         void* stream);

/* ------------------------------------------------------------------ length regulator
 * out[b, t, :] = x[b, j, :] for cs[j-1] <= t < cs[j] (cs = inclusive cumsum of
 * max(trunc(d[b, j]), 0)), zero for t >= mel_len[b]; mel_len[b] = cs[T_src-1]; rows past
 * max_len are cropped.  index (nullable) receives j (or -1).
 * Replaces: LengthRegulator.LR/expand (scripts/model/modules.py:132-159) + pad
 * (scripts/utils/tools.py:669-687): no per-token device->host sync. */
int vo_length_regulate(const void* x, int x_dtype, const float* dur, int B, int T_src, int D,
                       int max_len, void* out, int out_dtype, int64_t* mel_len, int32_t* index,
                       void* stream);

/* Backward of vo_length_regulate (training, config C4): gx[b, j, :] = sum of go[b, t, :] over
 * the frames t in [cs[j-1], min(cs[j], max_len)) that token j was copied to (frames past the
 * crop get no gradient), summed in frame order (deterministic).  go (B, max_len, D), gx
 * (B, T_src, D); D % 8 == 0.  Replaces: the autograd of LengthRegulator.LR/expand + pad
 * (scripts/model/modules.py:132-159, scripts/utils/tools.py:669-687). */
int vo_length_regulate_bwd(const void* go, int go_dtype, const float* dur, int B, int T_src, int D, int max_len,
                           void* gx, int gx_dtype, void* stream);
/* mel_len only (int64 and int32 copies), so the host can size the output. */
int vo_lr_lengths(const float* dur, int B, int T_src, int64_t* mel_len, int32_t* mel_len32,
                  void* stream);

/* ------------------------------------------------------------------ variance heads
 * Linear(D -> 1) + masked_fill(pad, 0) over h (B*T, D)  (VariancePredictor.linear_layer,
 * scripts/model/modules.py:207-213), then per head:
 *  VO_HEAD_DURATION: pred -> log_d; if d_round != NULL: d_round = clamp(round(exp(log_d)-1)
 *                    * d_control, 0) (modules.py:110-113, round half to even)
 *  VO_HEAD_ENERGY:   pred -> e_pred; idx = bucketize(target or ((pred*std+mean)*control -
 *                    mean)/std, bins) (right=False); x[b, t, :] += table[idx] (modules.py:
 *                    53-64,101-104); e_pred receives the transformed prediction when no
 *                    target is given, as the reference returns it. */
enum vo_head_kind { VO_HEAD_DURATION = 0, VO_HEAD_ENERGY = 1 };
typedef struct vo_head_desc {
  int kind;
  const void* h; int h_dtype;     /* (B*T, D) after the second LayerNorm     */
  const float* w; float b;        /* Linear(D, 1) weight [D] and bias         */
  const int32_t* lens;            /* src lengths [B] (pad mask), nullable     */
  int B, T, D;
  float* pred;                    /* [B*T] log_d or energy prediction         */
  float* d_round; float d_control;/* duration head                            */
  const float* target;            /* energy target [B*T] or NULL              */
  const float* bins; int n_bins;  /* bucket boundaries (n_bins)               */
  float e_mean, e_std, e_control;
  const float* table;             /* embedding (n_bins + 1, D) fp32           */
  void* x; int x_dtype;           /* (B*T, D) hidden state, += table[idx]     */
  int32_t* idx_out;               /* optional bucket indices                  */
} vo_head_desc;
int vo_variance_head(const vo_head_desc* d, void* stream);

/* Training-side energy embedding (config C4, teacher-forced): idx = bucketize(target, bins)
 * (right=False; a NaN target -> n_bins, as torch.bucketize), out = x + table[idx] (out of place),
 * rows = B*T, table (n_table >= n_bins + 1, D) fp32 (VO_ERR_INVALID otherwise);
 * vo_embed_bwd: dtable[e] = sum of dy rows with idx == e, added in row order (deterministic).
 * Replaces: energy_embedding(torch.bucketize(e_target, energy_bins)) and its autograd
 * (scripts/model/modules.py:53-64,101-104). */
int vo_bucket_embed(const void* x, int x_dtype, const float* target, const float* bins, int n_bins,
                    const float* table, int n_table, int64_t rows, int D, void* out, int32_t* idx_out, void* stream);
int vo_embed_bwd(const void* dy, int dy_dtype, const int32_t* idx, int64_t rows, int D, int n_table, float* dtable,
                 void* stream);

/* ------------------------------------------------------------------ encoder glue
 * Visual feature extractor front: for every 24 x W_s slice (b, i) of images (B, 1, 24, W),
 * 3 x [Conv2d 3x3 pad 1 (1 -> 1 ch) -> BatchNorm2d(eval, folded scale/shift) -> ReLU],
 * flattened h*W_s + w into out (B*n, 24*W_s) (then the bridge Linear runs as vo_conv1d K=1).
 * Replaces: VisualFeatureExtractor.forward slicing loop + embedder
 * (scripts/model/visual_feature_extractor.py:60-80).  conv: [n_layers][10] = 9 weights +
 * bias; bn: [n_layers][2] = scale, shift. */
int vo_vfe_stencil(const float* images, int B, int H, int W, int slice_w, int n_slices,
                   const float* conv, const float* bn, int n_layers, void* out, int out_dtype,
                   void* stream);
/* x[b, t, :] += pe[t, :] (pe nullable) + cls[idx, :] (cls nullable) with idx = cls_idx[b]
 * (idx_per_token = 0) or cls_idx[b*T + t] (idx_per_token = 1).
 * Replaces: position_enc add (Models.py:107-116, 184-186), audiotype_emb add (vtts.py:84-85)
 * and the src_word_emb lookup of the use_image=False branch (Models.py:114). */
int vo_add_pos_class(void* x, int x_dtype, const float* pe, const float* cls,
                     const int64_t* cls_idx, int idx_per_token, int B, int T, int D, void* stream);
/* mask[b, t] = t >= lens[b] (True = padding) and/or lens32[b] = (int32) lens[b];
 * lens_dtype: 0 = fp32, 2 = int64, 3 = int32.  Replaces get_mask_from_lengths
 * (scripts/utils/tools.py:164-171). */
int vo_mask_from_lengths(const void* lens, int lens_dtype, int B, int L, bool* mask,
                         int32_t* lens32, void* stream);

/* ------------------------------------------------------------------ vocoder glue
 * conv_post: y[b, t] = tanh(bias + sum_{k<7, c} w[k][c] * lrelu(x[b, t+k-3, c], 0.01))
 * over channels-last x (B, T, C) -> (B, T) fp32.  Replaces Generator.forward tail
 * (scripts/hifigan/models.py:161-163).  w packed [K][C] fp32. */
int vo_conv_post(const void* x, int x_dtype, const float* w, float bias, int B, int T, int C,
                 int K, float slope, float* y, void* stream);
/* Fused ResBlock1 pair for C = 32 / 64 / 128 (bf16, channels-last (B, T, C)):
 *   y = (x + c2(lrelu(c1_dil(lrelu(x, slope)), slope))) * out_scale (+ acc)
 * c1 / c2: K taps, packed [K][C][C] bf16 (vo_pack_weight VO_PACK_CONV), biases fp32;
 * c1 dilation dil, c2 dilation 1, both "same" padding.  The c1 output stays in LDS.
 * acc may alias y (MRF accumulate); y must not alias x.
 * Replaces one (c1, c2) iteration of ResBlock.forward (scripts/hifigan/models.py:96-103)
 * plus the MRF sum / 1/num_kernels of Generator.forward (models.py:155-160). */
int vo_resblock_pair(const void* x, const void* w1, const float* b1, const void* w2,
                     const float* b2, void* y, const void* acc, int B, int T, int C, int K,
                     int dil, float slope, float out_scale, void* stream);
/* vo_resblock_pair for C = 64 / 128, K = 7 / 11 with w1 / w2 in the fragment order that the pair
 * kernel streams into registers (vo_pack_frag of the [K][C][C] pack): every weight load is one
 * contiguous KiB.  C = 128: results equal vo_resblock_pair's on the same weights bit for bit.  Same
 * reference (scripts/hifigan/models.py:96-103, 155-160). */
int vo_resblock_pair_frag(const void* x, const void* w1, const float* b1, const void* w2,
                          const float* b2, void* y, const void* acc, int B, int T, int C, int K,
                          int dil, float slope, float out_scale, void* stream);
/* [K][C][C] bf16 (vo_pack_weight VO_PACK_CONV), C = 64 / 128 -> [K][C/32][C/32][2][64][8] fragment order:
 * dst[k][p][s][t][l][e] = src[k][32p + 8((l & 15) >> 2) + 4t + (l & 3)][32s + 8(l >> 4) + e]. */
int vo_pack_frag(const void* src, void* dst, int C, int K, void* stream);

/* Fused ResBlock1 with K = 3 (bf16, channels-last (B, T, C), C = 32 / 64 / 128): all three
 * (c1_dil[s], c2) iterations in one launch,
 *   x_{s+1} = x_s + c2_s(lrelu(c1_s(lrelu(x_s, slope)), slope))   (s = 0, 1; bf16-rounded)
 *   y = (x_2 + c2_2(lrelu(c1_2(lrelu(x_2))))) * out_scale (+ acc)
 * w1[s] / w2[s]: packed [3][C][C] bf16, b1[s] / b2[s] fp32, dil[s] in [1, 8] with
 * sum_s (dil[s] + 1) <= 12 (HiFi-GAN V1: 1, 3, 5).  x_1, x_2 never leave the chip.  acc may
 * alias y; y must not alias x.  Replaces a whole ResBlock.forward (scripts/hifigan/
 * models.py:96-103) with the MRF sum of Generator.forward (models.py:155-160); results equal
 * three vo_resblock_pair launches up to the fp32 summation order. */
int vo_resblock3(const void* x, const void* const* w1, const float* const* b1, const void* const* w2,
                 const float* const* b2, const int* dil, void* y, const void* acc, int B, int T, int C,
                 float slope, float out_scale, void* stream);

/* (B, C, T) -> (B, T, ldy) with channels C..ldy-1 zero-filled; fp32 in, dtype out. */
int vo_transpose_bct(const float* x, int B, int C, int T, void* y, int y_dtype, int ldy,
                     void* stream);

/* ------------------------------------------------------------------ mel / STFT front-end
 * log-mel (B, n_mels, F) and energy (B, F), F = 1 + N / hop, of wav (B, N) fp32 with
 * torchaudio Spectrogram(n_fft, win=n_fft, hop, power=1, center=True, reflect) +
 * MelScale(fb) + log(clamp_min(., 1e-5)) semantics (scripts/preprocessor/preprocessor.py:
 * 22-36,323-337).  window: (n_fft) fp32; fb: (n_fft/2+1, n_mels) fp32. */
int vo_stft_mel(const float* wav, int B, int N, const float* window, const float* fb, int n_fft,
                int hop, int n_mels, float log_floor, float* mel, float* energy, void* stream);
/* General framing: frame f covers reflect-padded samples [f*hop - pad, f*hop - pad + n_fft),
 * F = 1 + (N + 2*pad - n_fft) / hop; |X| = sqrt(re^2 + im^2 + mag_eps); clip != 0 clamps the
 * input to [-1, 1].  HiFi-GAN's training mel (pad (n_fft - hop)/2, center=False, mag_eps 1e-9,
 * no clip, slaney fb) and vo_stft_mel (pad n_fft/2, eps 0, clip). */
int vo_stft_mel_ex(const float* wav, int B, int N, const float* window, const float* fb, int n_fft,
                   int hop, int n_mels, int pad, float mag_eps, int clip, float log_floor, float* mel,
                   float* energy, float* fstats, void* stream);
/* fstats (nullable, (B, F, 2)): per frame sum_k |X_k|^2 and sum_k log(|X_k|^2 + 1e-8), the
 * power-spectrum statistics of Preprocessor._get_kurtosis. */

/* Character-level acoustic features (Preprocessor._process energy
 * averaging and _get_kurtosis, scripts/preprocessor/preprocessor.py:339-357,395-403): for
 * utterance b with characters j in [char_off[b], char_off[b+1]) of dur[j] frames (consecutive,
 * from frame 0): e_char[j] = mean(energy[b, span]) (0 if dur 0); k_char[j] = (eta+2)(eta+3)/
 * (eta(eta+1)+1e-8), eta = (3 - g + sqrt((g-3)^2 + 24 g)) / (12 g),
 * g = log(mean p + 1e-8) - mean log(p + 1e-8) over the span's n_bins x dur[j] power values. */
int vo_char_features(const float* energy, const float* fstats, int F, const int32_t* dur,
                     const int32_t* char_off, int B, int n_bins, float* e_char, float* k_char,
                     void* stream);

/* ------------------------------------------------------------------ HiFi-GAN training (C5)
 * Discriminator glue (the reference ships no discriminator code, only
 * the training hyper-parameters of scripts/hifigan/config.json):
 *  vo_pack_grouped: (Co, Ci/groups, K) fp32 -> dense [K][Co][Ci_pad] block-diagonal (zeros
 *    outside the groups and for ci >= Ci) for vo_conv1d's groups mode; vo_pack_grouped_blocks
 *    writes the diagonal blocks only (an in-place update of a buffer whose other entries are
 *    already zero);
 *  vo_period_fold: wav (B, T) -> (B*P, ceil(T/P), 8) channels-last, the MPD's reflect pad to a
 *    multiple of P and (T/P, P) view with each period column a separate sequence;
 *  vo_wav_cl8: (B, T) -> (B, T, 8) (channel 0); vo_avgpool_wav: AvgPool1d(4, 2, padding 2),
 *    (B, T) -> (B, T/2 + 1);
 *  vo_gan_reduce: *out += sum over a (rows x width) view of |a-b| (kind 0), (1-a)^2 (kind 1)
 *    or a^2 (kind 2), deterministic (block partials in workspace, >= 512 floats, added in order);
 *    vo_gan_reduce_grad: ga = *scale * d(sum)/da. */
int vo_pack_grouped(const float* src, int Co, int Ci, int K, int groups, int Ci_pad, void* dst,
                    int dst_dtype, void* stream);
int vo_pack_grouped_blocks(const float* src, int Co, int Ci, int K, int groups, int Ci_pad, void* dst,
                           int dst_dtype, void* stream);
/* Input-gradient weights of one stride phase r of a strided / grouped conv: w (Co, Ci/groups, K) fp32
 * -> dst [J][ci_out][co_in], dst[t][ci][co] = w[co][ci mod cig][k_r + S (J - 1 - t)] within a group,
 * 0 elsewhere (blocks_only: the diagonal blocks only, other entries left as they are).  Replaces
 * the transpose / flip / pack chain of the HiFi-GAN discriminators' backward (C5). */
int vo_pack_dgrad_phase(const float* w, int Co, int cig, int K, int groups, int S, int k_r, int J, int ci_out,
                        int co_in, int blocks_only, void* dst, int dst_dtype, void* stream);
/* Many weight packs in one call (hifigan/gan_ops.prepack: the ~270 re-packs after each C5 optimizer
 * step).  Job: for r < rows, j < width, t < T, with cbase(r) = (r / rpg) * cpg,
 *   dst[(t * dst_rows + r) * ld + cbase(r) + j] =
 *     GATHER swap 0: src[r][j][tap0 + tstep t]                    (vo_pack_weight CONV, grouped blocks)
 *     GATHER swap 1: src[cbase(r) + j][r mod rpg][tap0 + tstep t] (DGRAD, vo_pack_dgrad_phase blocks)
 *     CONVT:         src[j][r mod cig][r / cig + tap0 (1 - t)]    (vo_pack_weight CONVT, tap0 = s, K = 2s, T = 2)
 * src (src_rows, cig, K) fp32 contiguous (CONVT: (Ci, Co = cig, K)); other dst entries untouched;
 * a job's tap range (|tstep| (T - 1) + 1, CONVT: K) is at most 48. */
enum vo_pack_job_mode { VO_PJ_GATHER = 0, VO_PJ_CONVT = 1 };
typedef struct vo_pack_job {
  const float* src;
  void* dst;
  int mode, swap, T, rows, width, dst_rows, ld, rpg, cpg, cig, K, tap0, tstep, src_rows;
} VoPackJob;
int vo_pack_batch(int n, const VoPackJob* jobs, int dst_dtype, void* stream);
/* Row remap of channels-last rows (row_bytes, a multiple of 4): dst row r (r < dst_rows; n = r / Td,
 * t = r mod Td) = src row n Ss + t + shift if lo <= t < hi, else zeros.  The joined-sequence layout of
 * the discriminators' short period columns (hifigan/gan_ops._conv_joined) and its adjoint. */
int vo_seq_remap(const void* src, int64_t src_rows, void* dst, int64_t dst_rows, int row_bytes, int Td,
                 int64_t Ss, int lo, int hi, int shift, void* stream);
/* One or two remaps in one launch (rows of whole 16-byte units).  Job: dst row r (n = r / Td, t =
 * r mod Td) = src row n Ss + t + shift [+ src2 row n Ss2 + t + shift2, added in dtype (bf16 / fp32)
 * when src2 is non-NULL] for lo <= t < hi, else zeros; src_rows / src2_rows bound the reads.  One
 * joined discriminator conv feeding the next: the split output and the next joined input from one
 * read, and the backward's two gathers plus autograd's add of them (hifigan/gan_ops.RejoinFn). */
typedef struct vo_remap_job {
  const void* src; const void* src2; void* dst;
  int64_t src_rows, src2_rows, dst_rows, Ss, Ss2;
  int Td, lo, hi, shift, shift2;
} VoRemapJob;
int vo_seq_remap2(int n, const VoRemapJob* jobs, int row_bytes, int dtype, void* stream);
int vo_period_fold(const float* wav, int B, int T, int P, void* out, int dtype, void* stream);
int vo_wav_cl8(const float* wav, int64_t n, void* out, int dtype, void* stream);
int vo_avgpool_wav(const float* x, int B, int T, float* y, void* stream);
/* Their adjoints (dL/dwav, fp32, written): g in the forward's output layout and dtype; the period
 * fold adds the gradient of each right-pad row to the sample it mirrored. */
int vo_period_fold_bwd(const void* g, int dtype, int B, int T, int P, float* gwav, void* stream);
int vo_wav_cl8_bwd(const void* g, int dtype, int64_t n, float* gwav, void* stream);
int vo_avgpool_wav_bwd(const float* g, int B, int T, float* gx, void* stream);

/* Weight normalisation over n layers per call (torch.nn.utils.weight_norm, dim = 0; the HiFi-GAN
 * generator's and discriminators' weight-normed convs in C5 training -- replaces PyTorch's
 * per-layer torch._weight_norm forward / backward kernels, hifigan/models.py:96-103,124-132 and
 * the HiFi-GAN V1 discriminators).  Layer k: fp32 v[k] (rows[k] x len[k], contiguous), g[k]
 * (rows[k]); forward w[k] = v * g / ||v_row||; backward from dw[k]: dv[k], dg[k].  The pointer
 * and size tables are host arrays (copied into the kernel arguments, 24 layers per launch). */
int vo_weight_norm(int n, const void* const* v, const void* const* g, void* const* w, const int* rows,
                   const int* len, void* stream);
int vo_weight_norm_bwd(int n, const void* const* v, const void* const* g, const void* const* dw, void* const* dv,
                       void* const* dg, const int* rows, const int* len, void* stream);
/* Spectral normalisation (torch.nn.utils.spectral_norm: dim 0, one power iteration per training
 * forward; the HiFi-GAN V1 MSD's first scale in C5) for n layers per call.  Layer: W = weight_orig
 * (rows x L fp32), buffers u (rows) / v (L) updated in place when power != 0 (v = normalize(W^T u),
 * u = normalize(W v), normalize(x) = x / max(|x|, eps)), copies of the u / v used written to
 * u_out / v_out, sigma = u . W v, w = W / sigma; vraw (L) and s (rows) are scratch, and so is w
 * until it is written (it must not alias W).  Replaces the
 * per-layer PyTorch hook (two gemv, norms, clamps, divides, clones and a dot per layer). */
typedef struct vo_sn_layer {
  const float* W;
  float *u, *v, *u_out, *v_out, *vraw, *s, *sigma, *w;
  int rows, L;
} VoSnLayer;
int vo_spectral_norm(int n, const VoSnLayer* layers, int power, float eps, void* stream);
/* Its backward (u, v, sigma as the forward used them, held constant, as torch's autograd of the
 * hook does): gW = g / sigma - (sum(g * W) / sigma^2) u v^T for n layers in three launches; the sum
 * in a fixed order (deterministic).  workspace: vo_spectral_norm_bwd_workspace_size bytes. */
typedef struct vo_sn_bwd_layer {
  const float *g, *W, *u, *v, *sigma;
  float* gW;
  int rows, L;
} VoSnBwdLayer;
int64_t vo_spectral_norm_bwd_workspace_size(int n, const VoSnBwdLayer* layers);
int vo_spectral_norm_bwd(int n, const VoSnBwdLayer* layers, float* workspace, void* stream);
int vo_gan_reduce(int kind, const void* a, int lda, const void* b, int ldb, int64_t rows, int width,
                  int dtype, float* out, float* workspace, void* stream);
int vo_gan_reduce_grad(int kind, const void* a, int lda, const void* b, int ldb, int64_t rows,
                       int width, int dtype, const float* scale, void* ga, int ldg, void* stream);
/* Many terms per launch (the C5 G step's feature-matching / adversarial terms, the D step's halves):
 * vo_gan_reduce_multi writes out[i] = sum_i * scale[i] (scale NULL: 1), each sum bit for bit
 * vo_gan_reduce's (workspace: vo_gan_reduce_multi_workspace_size(n) bytes); vo_gan_reduce_grad_multi
 * writes term i's gradient ga_i = scale[i] * d(sum_i)/da_i (ga, ldg per term).  scale: n device floats. */
typedef struct vo_gan_term {
  int kind; const void* a; int lda; const void* b; int ldb; int64_t rows; int width; void* ga; int ldg;
} VoGanTerm;
int64_t vo_gan_reduce_multi_workspace_size(int n);
int vo_gan_reduce_multi(int n, const VoGanTerm* terms, int dtype, const float* scale, float* out, float* workspace,
                        void* stream);
int vo_gan_reduce_grad_multi(int n, const VoGanTerm* terms, int dtype, const float* scale, void* stream);

/* ------------------------------------------------------------------ training backward
 * Weight gradient of a channels-last conv on MFMA (replaces the MIOpen weight pass of the
 * training backward):
 *   dw[(m*N + n)*K + k] = sum_{b, t < T_A} A[b, t, m] * B[b, t*S + k*dil - pad, n]
 * (written in the conv weight's own (M, N, K) order; B rows outside [0, T_B) read as 0;
 * pre_a / pre_b: leaky-ReLU(slope) applied to that operand).
 * Conv1d (Co, Ci, K): A = dY (T_out rows, M = Co), B = pre(x) (T_in rows, N = Ci).
 * ConvTranspose1d (Ci, Co, 2s): A = pre(x) (T_in, M = Ci), B = dY (T_up, N = Co), S = s, pad p.
 * dw fp32.  Deterministic: each row split stores its partial tile into ``workspace``
 * (vo_conv1d_wgrad_workspace_size bytes for the same B, T_A, M, N, K, groups) and a second
 * kernel adds the splits in a fixed order.  dtype: VO_BF16 or VO_F32 for both operands, or VO_F32X3
 * (fp32 operands contracted as split-bf16, see the header note; stride 1, ungrouped).
 * vo_colsum: out[c] = sum_r x[r*ld + c] (bias gradient; block partials in workspace,
 * vo_colsum_workspace_size bytes, added in order). */
int64_t vo_conv1d_wgrad_workspace_size(int B, int T_A, int M, int N, int K, int groups);
int vo_conv1d_wgrad(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B, int M,
                    int N, int K, int S, int dil, int pad, int pre_a, int pre_b, float slope,
                    int dtype, float* dw, float* workspace, void* stream);
/* Grouped conv (groups > 1): M = C_out / groups and N = C_in / groups per group, lda >= groups*M,
 * ldb >= groups*N; group g reads A columns [g*M, (g+1)*M), B columns [g*N, (g+1)*N) and writes
 * rows [g*M, (g+1)*M) of dw laid out (groups*M, N, K).  Replaces MIOpen's grouped weight pass of
 * the multi-scale discriminator (HiFi-GAN V1 MSD). */
int vo_conv1d_wgrad_grouped(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B,
                            int M, int N, int K, int S, int dil, int pad, int groups, int pre_a,
                            int pre_b, float slope, int dtype, float* dw, float* workspace, void* stream);
/* vo_conv1d_wgrad_grouped + the bias gradient in the same launch: db[g*M + m] = sum over all
 * A rows of A[.., g*M + m] (the conv form, A = dY; pre_a must be 0), summed by the tap-0
 * workgroups as they stage A (saves the separate vo_colsum launch). */
int vo_conv1d_wgrad_bias(const void* a, int lda, int T_A, const void* b, int ldb, int T_B, int B,
                         int M, int N, int K, int S, int dil, int pad, int groups, int pre_a,
                         int pre_b, float slope, int dtype, float* dw, float* db, float* workspace,
                         void* stream);
int64_t vo_colsum_workspace_size(int64_t rows, int C);
int vo_colsum(const void* x, int64_t rows, int C, int ld, int dtype, float* out, float* workspace, void* stream);

/* Leaky-ReLU / ReLU backward mask: out[r, c] = g[r, c] * (ref[r, c] > 0 ? 1 : slope) over a
 * (rows x width) view with leading dimensions (out may alias g; ref = the activation's input, or
 * its output when slope > 0).  Replaces the elementwise autograd of F.leaky_relu / F.relu
 * (hifigan/models.py:96-103,155-163, SubLayers.py:85-93) in the training backward. */
int vo_lrelu_mask(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype, int64_t rows,
                  int width, float slope, void* out, int ldo, void* stream);
/* out = round(g * (ref > 0 ? 1 : slope)) + add (the masked gradient plus a residual branch's gradient
 * in one pass; add has g's dtype; rows of 8-element vectors, 16-byte aligned). */
int vo_lrelu_mask_add(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype, const void* add,
                      int lda, int64_t rows, int width, float slope, void* out, int ldo, void* stream);
/* out = round(round(g + add) * (ref > 0 ? 1 : slope)): two gradients of a leaky-ReLU output (the next
 * conv's input gradient and a feature-matching loss's, HiFi-GAN discriminators) summed as autograd
 * sums them and masked in one pass (same layout rules as vo_lrelu_mask_add). */
int vo_lrelu_mask_sum(const void* g, int ldg, int g_dtype, const void* ref, int ldr, int ref_dtype, const void* add,
                      int lda, int64_t rows, int width, float slope, void* out, int ldo, void* stream);

/* ------------------------------------------------------------------ training glue (round 2)
 * BatchNorm with batch statistics over channels-last x (M rows x C channels, VO_F32 / VO_BF16):
 * y = (x - mean) rstd * gamma + beta (gamma / beta may both be NULL), mean_rstd[0..C) = mean,
 * [C..2C) = 1/sqrt(var_biased + eps); running stats (both or neither): r = (1-m) r + m stat with
 * the unbiased variance, *nbt += 1 (NULL: skipped).  workspace: vo_bn_workspace_size bytes.
 * Replaces nn.BatchNorm1d/2d in training mode -- PostNet (scripts/transformer/Layers.py:129-137)
 * and the glyph encoder's single-channel BatchNorm2d (C = 1; scripts/model/
 * visual_feature_extractor.py:40-47).  vo_bn_bwd: dgamma = sum dy xhat, dbeta = sum dy,
 * dx = gamma rstd (dy - dbeta / M - xhat dgamma / M) (dx in x's dtype).  Deterministic. */
int64_t vo_bn_workspace_size(int M, int C);
int vo_bn_train_fwd(const void* x, int dtype, int M, int C, const float* gamma, const float* beta, float eps,
                    float momentum, float* run_mean, float* run_var, int64_t* nbt, float* mean_rstd,
                    float* workspace, void* y, void* stream);
int vo_bn_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype, int M, int C, const float* gamma,
              const float* mean_rstd, float* workspace, float* dgamma, float* dbeta, void* dx, void* stream);

/* Dropout in training (nn.Dropout / F.dropout: scripts/transformer/SubLayers.py:38,87,
 * scripts/transformer/Layers.py:129-131, scripts/model/modules.py:52-56): y[i] = x[i] / (1 - p) when
 * hash(*seed, salt, i) >= p 2^32, else 0 (x, y fp32 / bf16, 16-byte aligned, n < 2^32; y may alias x).
 * The mask depends only on (*seed, salt, i): the backward is the same call on dy.  One device seed per
 * training step, a distinct salt per dropout site of the step. */
int vo_dropout(const void* x, int dtype, int64_t n, float p, const int64_t* seed, unsigned salt, void* y,
               void* stream);

/* Glyph-encoder Conv2d(1, 1, 3, padding=1) on N single-channel H x W maps (fp32), w[0..9) the
 * row-major kernel, w[9] the bias (scripts/model/visual_feature_extractor.py:40-47,60-72):
 * forward, and the backward -> dx and dw[10] (weight + bias gradient; per-block partials summed in
 * a fixed order, workspace: vo_vfe_conv_workspace_size bytes). */
int64_t vo_vfe_conv_workspace_size(int N, int H, int W);
int vo_vfe_conv_fwd(const float* x, int N, int H, int W, const float* w, float* y, void* stream);
int vo_vfe_conv_bwd(const float* x, const float* dy, int N, int H, int W, const float* w, float* dx, float* dw,
                    float* workspace, void* stream);

/* Backward of vo_stft_mel_ex (clip off; the HiFi-GAN V1 training mel-loss front end):
 * gmel (B, n_mels, F) = dL/dlogmel -> dwav (B, N) fp32 (written, not accumulated).  Per frame the
 * spectrum is recomputed; the frame gradients (workspace: vo_stft_mel_bwd_workspace_size bytes)
 * are gathered per sample over the overlapping frames and the reflect-padding mirrors in a
 * fixed order.  n_mels <= 256. */
int64_t vo_stft_mel_bwd_workspace_size(int B, int N, int n_fft, int hop, int pad);
int vo_stft_mel_bwd(const float* wav, int B, int N, const float* window, const float* fb, int n_fft, int hop,
                    int n_mels, int pad, float mag_eps, float log_floor, const float* gmel, float* dwav,
                    float* workspace, void* stream);

/* Multi-resolution STFT loss (the auxiliary spectral loss of BASELINE.json config C5; Parallel
 * WaveGAN's formulation: per resolution spectral convergence ||Y - X||_F / ||Y||_F and mean
 * |log Y - log X| over STFT magnitudes).  vo_stft_mag: torch.stft(center=True, reflect padding
 * n_fft / 2, onesided) of wav (B, N) fp32 with `window` (n_fft samples: the win_len window zero-
 * padded to n_fft, centred, as torch.stft pads it) -> mag (B, 1 + N / hop, n_fft / 2 + 1) =
 * sqrt(max(|X|^2, eps)); vo_stft_mag_bwd: gmag -> dwav (written; workspace
 * vo_stft_mag_bwd_workspace_size bytes; deterministic gather as vo_stft_mel_bwd).
 * vo_stft_loss: out[3] = (sum (y - x)^2, sum y^2, sum |log y - log x|) over n magnitudes
 * (workspace >= 1536 floats); vo_stft_loss_grad: gx = d(w[0] sqrt(out0 / out1) + w[1] out2 / n)/dx with
 * the weights w[2] (the incoming loss gradients) read on the device. */
int vo_stft_mag(const float* wav, int B, int N, const float* window, int n_fft, int hop, float eps, float* mag,
                void* stream);
int64_t vo_stft_mag_bwd_workspace_size(int B, int N, int n_fft, int hop);
int vo_stft_mag_bwd(const float* wav, int B, int N, const float* window, int n_fft, int hop, float eps,
                    const float* gmag, float* dwav, float* workspace, void* stream);
int vo_stft_loss(const float* xm, const float* ym, int64_t n, float* out, float* workspace, void* stream);
int vo_stft_loss_grad(const float* xm, const float* ym, int64_t n, const float* sums, const float* w, float* gx,
                      void* stream);

/* ------------------------------------------------------------------ training input pipeline
 * Glyph batch: B grayscale strips packed in px (strip b at img_off[b],
 * H rows of img_w[b] uint8 columns) -> out (B, 1, H, W_out) fp32 = pixel / 255 with each
 * character j of sample b (char_off[b] <= j < char_off[b+1]: columns [char_start[j],
 * char_start[j] + char_len[j]) of its strip) centred in a `cell`-wide white cell
 * (pleft = (cell-len)/2 + (cell-len)%2), white right-padding to W_out and `margin` white
 * columns on the left.  char_off == NULL: strips copied as they are (already centred).
 * Replaces Dataset.character_padding_forinput (scripts/dataset.py:71-92), pad_2D_gray_image
 * (scripts/utils/tools.py:616-635) and to_device's ToTensor (tools.py:18-20,50-51). */
int vo_glyph_batch(const uint8_t* px, const int64_t* img_off, const int32_t* img_w,
                   const int32_t* char_off, const int32_t* char_start, const int32_t* char_len,
                   int B, int H, int cell, int margin, int W_out, float* out, void* stream);

/* ------------------------------------------------------------------ optimizer
 * Multi-tensor Adam (decoupled = 0: L2 weight decay on the gradient) / AdamW (decoupled = 1) step over
 * nt fp32 tensors (tables of device pointers and element counts, host memory), torch's
 * single-tensor update order; lr and step (the steps taken so far) are device scalars read by the
 * kernels, so the update is graph-capturable.  vo_opt_step_increment(step) advances the counter
 * (after every vo_adam_multi call of a step).  Replaces torch.optim.Adam behind ScheduledOptim
 * (scripts/model/optimizer.py:9-15) and the HiFi-GAN V1 recipe's AdamW. */
int vo_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                  const int64_t* numel, const float* lr, const float* step, float beta1, float beta2, float eps,
                  float weight_decay, int decoupled, void* stream);
int vo_opt_step_increment(float* step, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VONOMA_H_ */
