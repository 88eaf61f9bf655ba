/*
 * libmiattack — C ABI of the MI355X (gfx950 / CDNA4) adversarial-perturbation engine.
 *
 * Hot path (BASELINE.json north_star): PGD/FGSM over  encoder → StyleGAN2 synthesis → VGG feature
 * loss → ∇ wrt pixels → sign-project onto the L∞ ball. The reference has no FFI for this path: it
 * runs PyTorch modules (cuDNN + un-vendored rosinality CUDA ops). Each entry point below replaces
 * one device computation the reference performs, cited as file:line into /root/reference
 * ([ext] = the un-vendored rosinality op the reference calls through net.decoder).
 *
 * Conventions
 *   - All pointers are DEVICE pointers owned by the caller (PyTorch caching allocator).
 *   - Feature maps are NHWC, element type given by `dtype` (MIA_F32 / MIA_F16 / MIA_BF16);
 *     style, demod, bias, noise, reduction buffers and image-space tensors are fp32.
 *     Images at the API boundary are NCHW fp32 in [-1,1].
 *   - `stream` is a hipStream_t; every call is asynchronous on it, stateless and re-entrant.
 *   - Every call returns 0 on success or a negative MIA_E* code; mia_last_error_string() (per
 *     thread) gives detail. No C++ exception crosses the ABI.
 *   - Deterministic reductions: no float atomics. Every per-(image, channel) / per-image sum that
 *     several blocks contribute to (sdot, bab_q, csum, the torgb / bias_act style and q sums,
 *     mia_mse_sum's loss, mia_chan_dot) is written as per-block partials into a device scratch
 *     the library keeps PER STREAM, then added in a fixed order by a finish kernel on the same
 *     stream: results are bit-identical run to run, and an image's sums do not depend on the
 *     other images of the call. The scratch grows on first use (a synchronising hipMalloc; the
 *     old buffer is freed after a stream synchronise); mia_reserve_reduction_scratch pre-sizes
 *     it from the *_workspace_size queries below so that no step allocates.
 */
#ifndef MIATTACK_H
#define MIATTACK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIA_F32 0
#define MIA_F16 1
#define MIA_BF16 2

#define MIA_OK 0
#define MIA_EINVAL (-1)
#define MIA_ELAUNCH (-2)

#define MIA_ACT_NONE 0
#define MIA_ACT_RELU 1
#define MIA_ACT_LRELU_S2 2 /* leaky_relu(v, 0.2) * sqrt(2)  (FusedLeakyReLU) */
#define MIA_ACT_PRELU 3    /* v > 0 ? v : act_slope[co]·v  (PReLU / LeakyReLU; conv act_out only) */

int mia_version(void);
const char* mia_last_error_string(void);

/* ---- reduction scratch (see Conventions) ----------------------------------------------------
 * Upper bounds of the scratch bytes one call needs:
 *   mia_conv_workspace_size — mia_conv3x3 / mia_conv2d / mia_upconv_dgrad* with sdot / bab_q /
 *     csum for N images of an H_out × W_out output with Cout channels (0 without sums);
 *   mia_reduction_workspace_size — the pixel-chunked pointwise reductions (bias_act_bwd,
 *     torgb_bwd[_front], chan_dot: N images of HW pixels × C channels; mse_sum: C = 1).
 * Replaces: nothing in the reference (cuDNN / the rosinality ops allocate their own workspace);
 * the SURVEY.md §8(b) contract's workspace queries. */
int64_t mia_conv_workspace_size(int N, int H_out, int W_out, int Cout, int has_sums);
int64_t mia_reduction_workspace_size(int N, int HW, int C);
/* ensure the stream's scratch holds at least `bytes` (synchronises `stream` if it grows) */
int mia_reserve_reduction_scratch(int64_t bytes, void* stream);
/* bytes the stream's scratch holds now (0 if none) */
int64_t mia_reduction_scratch_bytes(void* stream);
/* free the stream's scratch (synchronises `stream`) */
int mia_release_reduction_scratch(void* stream);

/* ---- kernel-variant switches ------------------------------------------------------------------
 * Every conv launch picks its kernel variant from a table of named switches (MIA_CONV_HALO,
 * MIA_CONV_X6, MIA_HALO_EPI, ... — csrc/reduce.hip g_tune). The defaults are the measured-best
 * choices; the table is read ONCE from the environment at first use, then changed only through
 * mia_set_tuning (the A/B tools and the variant-coverage tests). No launch reads the environment.
 * Replaces: nothing in the reference (cuDNN's algorithm choice is internal). */
int mia_set_tuning(const char* name, int value);   /* MIA_ERR_ARG for an unknown name */
int mia_get_tuning(const char* name, int* value);
/* K-padding the conv weights need for `dtype` (weights are [Cout][Kpad], K = 9*Cin). */
int mia_conv_kpad(int cin, int dtype);

/*
 * Generic 3x3 / stride 1 / pad 1 implicit-GEMM convolution on MFMA (NHWC).
 *   y[n,p,co] = epilogue( Σ_{tap,ci} in(x)[n, p+tap, ci] · w[co][tap*Cin + ci] )
 * Replaces: the cuDNN convs of code/vgg.py:45-62 (VGG fwd and, with flipped/transposed weights,
 * their input-gradient), the grouped conv of ModulatedConv2d [ext] (modulation folded into
 * in_scale, demodulation into out_scale), and the conv_transpose2d + Blur of the up-sampling
 * StyledConv [ext] (4-phase weights + shuffle_out).
 * Prologue on the A operand:  in(x) = act_in(x) * in_scale[n][ci].
 * Epilogue, in this order (each step optional):
 *   sdot[n][co] += acc * act_aux(aux_x[n,p,co])       (style gradient, Σ over pixels)
 *   v = acc * out_scale[n][co % cout_mod]
 *   v += noise_w * noise[pixel_out] ; v += bias[co % cout_mod]
 *   v += tap_coef * (tap_a - tap_t) ; v *= (mask_a > 0) ; v = act_out(v) ; v += y (accumulate)
 *   [fused StyledConv backward front, when bab_demod: with a = aux_x (the stored activation
 *    lrelu(pre)·√2 of the layer below, act_aux = NONE), g = v·lrelu'(a), pre = a / lrelu'(a):
 *    bab_q[n][co] += g·(pre − bab_noise_w·bab_noise[pixel] − bab_bias[co]); v = g·bab_demod[n][co]
 *    — what mia_bias_act_bwd(from_act=1) would compute from this output]
 *   y[...] = v           (pixel-shuffled to (2H, 2W, Cout/4) when shuffle_out)
 */
typedef struct mia_conv_args {
  const void* x;          /* [N][H][W][Cin] */
  const void* w;          /* [Cout][Kpad] */
  void* y;                /* [N][H][W][y_cstride] or shuffled; may be NULL (sdot only) */
  int N, H, W, Cin, Cout, Kpad;
  int y_cstride;          /* channel stride of y (0 → Cout, or Cout/4 when shuffle_out) */
  int act_in;             /* MIA_ACT_* applied to x before in_scale */
  const float* in_scale;  /* [N][Cin] or NULL */
  const float* out_scale; /* [N][cout_mod] or NULL */
  const float* bias;      /* [cout_mod] or NULL */
  const float* noise;     /* [Hout*Wout] or NULL */
  float noise_w;
  int act_out;            /* MIA_ACT_* applied at the end */
  int shuffle_out;        /* 1: Cout = 4*cout_mod phases (py,px) → output (2H,2W,cout_mod) */
  const void* aux_x;      /* [N][H][W][Cout] (same layout as y, un-shuffled) for sdot */
  int act_aux;
  float* sdot;            /* [N][Cout] fp32, accumulated with atomics */
  const void* tap_a;      /* [N][H][W][Cout] */
  const void* tap_t;
  float tap_coef;
  const void* mask_a;     /* [N][H][W][Cout] */
  int accumulate;
  const float* bab_demod; /* [N][Cout] or NULL: fused backward front of the layer below */
  const float* bab_noise; /* [H*W] or NULL */
  float bab_noise_w;
  const float* bab_bias;  /* [Cout] or NULL */
  float* bab_q;           /* [N][Cout] fp32, accumulated with atomics */
  /* encoder (IR-SE50 / e4e) epilogue features, applied in the order of the list above:
   *   mask_slope: the mask step becomes v = mask_a > 0 ? v : mask_slope[co]·v (PReLU backward)
   *   act_slope:  per-channel slope of act_out = MIA_ACT_PRELU
   *   csum:       csum[n][co] += Σ_p y (the stored value; SE average pool) */
  const float* mask_slope; /* [Cout] or NULL (→ 0: ReLU mask) */
  const float* act_slope;  /* [Cout], required by MIA_ACT_PRELU */
  float* csum;             /* [N][Cout] fp32, accumulated with atomics, or NULL */
  /* fp32 only, optional: the same weights pre-split for the bf16 matrix pipe (a = hi + mid + lo,
   * exact; layouts.split_f32): [Cout][Kpad] words, per 4-k quad [hi×4 | mid×4] bf16 (16 B), then
   * [Cout][Kpad] bf16 lo. Lets the stride-1 3×3 layers take the split-once halo kernel
   * (conv_halo_x6.hip); NULL → the kernels split w on the fly. */
  const void* w_split;
} mia_conv_args;

int mia_conv3x3(const mia_conv_args* args, int dtype, void* stream);

/* StyledConv forward on per-image weights (fp16 / bf16; the StyleGAN2 modulated_conv2d of
 * attack_main2.py:619-621, rosinality ModulatedConv2d's own weight path): mia_modulate_weights
 * writes w_mod[n][co][k] = w[co][k]·in_scale[n][ci(k)]·out_scale[n][co] (out_scale may be NULL),
 * k = tap·Cin + ci < 9·Cin, 0 in the Kpad padding; mia_conv3x3_wmod then runs mia_conv3x3 with
 * args->w = w_mod, the images' matrices w_nstride elements apart, and no in_scale / out_scale
 * (folded into the weights). Halo-kernel shapes only (H, W multiples of 16, Cout > 64). */
int mia_modulate_weights(const void* w, const float* in_scale, const float* out_scale,
                         void* w_mod, int N, int Cout, int Cin, int Kpad, int dtype,
                         void* stream);
int mia_conv3x3_wmod(const mia_conv_args* args, int64_t w_nstride, int dtype, void* stream);

/*
 * General form of the same implicit-GEMM conv: 1..4 problems ("groups") over one input x
 * (args->H × args->W) that share the epilogue, each with its own weights [Cout][Kpad]
 * (K = kh·kw·Cin tap-major, Kpad = mia_conv2d_kpad(kh·kw, Cin, dtype)), tap window, padding and
 * output placement: group output (y, x) ∈ [0,ho)×[0,wo) reads input
 * (stride·y + ty − pad_y, stride·x + tx − pad_x) and lands at (ay·y + by, ax·x + bx) of the
 * (N, out_h, out_w, y_cstride) output. Aux operands (mask_a, tap_*, aux_x) are indexed at the
 * placed output pixel with channel stride Cout. args->w and args->Kpad are ignored.
 * Replaces the encoder's strided convolutions and their input gradients (e4e / IR-SE50,
 * un-vendored Encoder4Editing behind net.encoder, code/utils/model_utils.py:24,
 * code/attack/attack_main2.py:597,622): stride-2 3×3 (bottleneck conv2, GradualStyleBlock),
 * 1×1 stride-1/2 (FPN lateral, shortcut), and the 4-phase sub-pixel adjoint of a stride-2 conv.
 */
/* Input gradient of a stride-2, pad-1 3×3 conv as ONE halo-tiled launch (the halo up-conv kernel
 * mirrored; R % 16 == 0, Cg % 64 == 0, Cx % 64 == 0): g (N,R,R,Cg) → gx (N,2R,2R,Cx),
 * gx = mask(Σ ...) (+ gx if accumulate), mask as mia_conv_args.mask_a / mask_slope.
 * w_halo = layouts.s2_dgrad_halo_matrix(W): [Cg/BK][5][2][Cx][BK] (BK = 64, fp32 32). Replaces the same e4e strided
 * conv backward as the mia_conv2d phase groups (bottleneck conv2, GradualStyleBlock convs). */
int mia_conv_s2_dgrad_halo(const void* g, const void* w_halo, void* gx, int N, int R, int Cg,
                           int Cx, const void* mask_a, const float* mask_slope, int accumulate,
                           int dtype, void* stream);
/* The summed input gradients of ng ≤ 8 stride-2 3×3 convs that read the same tensor (the e4e
 * GradualStyleBlocks whose first conv reads one FPN map: 7 heads on p1, 4 on p2, psp_encoders
 * GradualStyleBlock.forward, reached through net.encoder at code/attack/attack_main2.py:597,622)
 * as ONE K loop: g[i] (N,R,R,Cg) are the convs' output gradients, w_halo the heads' packed
 * matrices concatenated along the first dimension ([ng·Cg/BK][5][2][Cx][BK]); gx as
 * mia_conv_s2_dgrad_halo (the sum, masked, + gx if accumulate). w_split (fp32 only, optional):
 * layouts.split_f32(w_halo) — the split-once fp32 kernel (csrc/conv_upconv.hip s2dg_x6_kernel). */
int mia_conv_s2_dgrad_halo_multi(const void* const* g, int ng, const void* w_halo,
                                 const void* w_split, void* gx, int N, int R, int Cg, int Cx,
                                 const void* mask_a, const float* mask_slope, int accumulate,
                                 int dtype, void* stream);

typedef struct mia_conv_group {
  const void* w;
  int kh, kw, pad_y, pad_x, ho, wo, ay, by, ax, bx;
  const void* w_split;  /* as mia_conv_args.w_split, for this group's w (or NULL) */
} mia_conv_group;
int mia_conv2d_kpad(int taps, int cin, int dtype);
int mia_conv2d(const mia_conv_args* args, int stride, const mia_conv_group* groups, int ngroups,
               int out_h, int out_w, int dtype, void* stream);
/* One stride-2 conv whose Cout = P·plane_channels output channels land in P separate planes:
 * channel co of output pixel (n, y, x) at y[(co / plane_channels)·plane_stride +
 * ((n·out_h + y)·out_w + x)·plane_channels + co % plane_channels]. The first convs of the e4e
 * GradualStyleBlocks that read one FPN map (psp_encoders Encoder4Editing.forward: 7 heads on p1,
 * 4 on p2, 3 on c3; called via net.encoder at attack_main2.py:597,622) as ONE launch with the
 * heads' weights / biases concatenated along Cout, each head's output in its slot of the stacked
 * level buffer. plane_channels a multiple of 128; bias / act_out (PReLU: act_slope of Cout)
 * epilogues only. */
int mia_conv2d_planes(const mia_conv_args* args, int stride, const mia_conv_group* groups,
                      int out_h, int out_w, int plane_channels, int64_t plane_stride, int dtype,
                      void* stream);
/* Up to 16 INDEPENDENT convs of one geometry family in one launch (the e4e GradualStyleBlock
 * convs of one resolution level across the style heads, psp_encoders GradualStyleBlock.forward,
 * reached through net.encoder at code/attack/attack_main2.py:597,622): group g is a conv with its
 * own weights (groups[g]) over images batch[g].n_in … + args->N − 1 of args->x, writing images
 * batch[g].n_out … of args->y (aux operands such as mask_a likewise), its per-channel operands
 * (bias, act_slope, mask_slope) read at channel offset batch[g].c_off. x / y / mask_a hold all
 * groups' images stacked along N. No shuffle_out / sdot / bab / csum. */
typedef struct mia_conv_batch {
  int n_in, n_out, c_off;
} mia_conv_batch;
int mia_conv2d_batched(const mia_conv_args* args, int stride, const mia_conv_group* groups,
                       const mia_conv_batch* batch, int ngroups, int out_h, int out_w, int dtype,
                       void* stream);

/* ---- named entry points (thin wrappers over mia_conv3x3) ------------------------------- */
/* ModulatedConv2d + NoiseInjection + FusedLeakyReLU bias, forward [ext]
 * (net.decoder at code/attack/attack_main2.py:619-621). Writes pre = demod·conv(act(x)·s) +
 * noise_w·noise + bias; the lrelu·√2 is applied by the consumer (act_in / act_aux). upsample=1
 * expects 4-phase up-conv weights (Cout = 4*cout) and writes (2H,2W,cout). */
int mia_modconv_fwd(const void* x, const void* w, void* pre, int N, int H, int W, int Cin,
                    int Cout, int Kpad, int act_in, const float* style, const float* demod,
                    const float* noise, float noise_w, const float* bias, int upsample, int dtype,
                    void* stream);
/* Input gradient + style sdot of the modulated conv (K15, no weight gradient). gy is the
 * demod-scaled pre-activation gradient (mia_bias_act_bwd), w_t the flipped/transposed weights
 * ([Cin][Kpad'] over K' = 9*Cout, or 9*4*cout for up-convs), x_fwd/act_x the forward input. */
int mia_modconv_bwd(const void* gy, const void* w_t, void* gx, int N, int H, int W, int Cin_g,
                    int Cout_g, int Kpad, const void* x_fwd, int act_x, const float* style,
                    float* sdot, int dtype, void* stream);
/* VGG conv3x3 + bias + ReLU forward (code/vgg.py:45-62). */
int mia_vgg_conv_relu_fwd(const void* x, const void* w, const float* bias, void* y, int N,
                          int H, int W, int Cin, int Cout, int Kpad, int dtype, void* stream);
/* VGG conv input-gradient with the tap-MSE term and ReLU mask of the layer below fused
 * (code/vgg.py:45-62 backward; feature MSE interpolation.py:786-817). */
int mia_vgg_conv_dgrad(const void* g, const void* w_t, void* gx, int N, int H, int W, int Cin_g,
                       int Cout_g, int Kpad, const void* tap_a, const void* tap_t,
                       float tap_coef, const void* mask_a, int dtype, void* stream);
/* The SURVEY.md §8(b) name of mia_vgg_conv_dgrad (same arguments, same result): the input
 * gradient of a VGG conv3x3 + bias + ReLU block, the ReLU mask of the layer below (mask_a, its
 * stored post-ReLU output) and the tap-MSE term (tap_a, tap_t, tap_coef) fused in the epilogue.
 * Replaces: autograd through code/vgg.py:45-62 and interpolation.py:786-817. */
int mia_vgg_conv_relu_dgrad(const void* g, const void* w_t, void* gx, int N, int H, int W,
                            int Cin_g, int Cout_g, int Kpad, const void* tap_a, const void* tap_t,
                            float tap_coef, const void* mask_a, int dtype, void* stream);

/* Up-sampling StyledConv [ext] as conv_transpose2d(stride 2, pad 0) → Blur (algorithmic FLOPs:
 * 9·Cin·Cout MACs per INPUT pixel). The transposed conv runs as four sub-pixel phase GEMMs in one
 * launch: phase (py,px) has (2−py)×(2−px) taps, w_phase[ph] = [Cout][mia_upconv_kpad(Cin, ph)]
 * with tap (ty,tx) ↔ W[py + 2(kh−1−ty)][px + 2(kw−1−tx)]. Output T: (N, 2R+1, 2R+1, Cout), no
 * demod (applied after the blur, with which it commutes). x: (N,R,R,Cin). */
int mia_upconv_kpad(int cin, int phase, int dtype);
int mia_upconv_fwd(const void* x, const void* const* w_phase, void* t_out, int N, int R, int Cin,
                   int Cout, int act_in, const float* style, int dtype, void* stream);
/* Same result as mia_upconv_fwd from ONE halo-tiled MFMA launch over the interior (input halo
 * staged in LDS once per 64-channel block and read by all 9 (offset, phase) products) plus a
 * generic launch for the last row / column of the even phase grids. w_up: the packed weights
 * [Cin/64][5][2][Cout][64] of layouts.upconv_halo_matrix (K-step st = offset (0,0)·{p0,p1},
 * (0,0)·{p2,p3}, (0,−1)·{p0,p2}, (−1,0)·{p0,p1}, (−1,−1)·{p0}; phase p = 2·py + px; slot weight
 * W[:, :, py + 2·jy, px + 2·jx]). Falls back to mia_upconv_fwd (w_phase) for fp32, R % 16 ≠ 0,
 * Cin % 64 ≠ 0, Cout % 64 ≠ 0 or w_up == NULL. Replaces the same [ext] conv_transpose2d. */
int mia_upconv_fwd_halo(const void* x, const void* const* w_phase, const void* w_up, void* t_out,
                        int N, int R, int Cin, int Cout, int act_in, const float* style,
                        int dtype, void* stream);
/* mia_upconv_fwd_halo with the split_f32 copy of w_up (fp32: the split-once interior kernel,
 * csrc/conv_upconv.hip upconv_x6_kernel; NULL → as mia_upconv_fwd_halo). */
int mia_upconv_fwd_halo_split(const void* x, const void* const* w_phase, const void* w_up,
                              const void* w_up_split, void* t_out, int N, int R, int Cin, int Cout,
                              int act_in, const float* style, int dtype, void* stream);
/* pre = demod·Blur(T) + noise_w·noise + bias, (N, 2R, 2R, C) (rosinality Blur pad (1,1));
 * act_out = MIA_ACT_LRELU_S2 stores the StyledConv activation lrelu(pre)·√2 instead. */
int mia_upconv_blur_fwd(const void* t, void* pre, const float* demod, const float* noise,
                        float noise_w, const float* bias, int N, int R, int C, int act_out,
                        int dtype, void* stream);
/* Adjoint of the blur: gT (N, 2R+1, 2R+1, C) from gy = demod·∂L/∂pre (N, 2R, 2R, C). */
int mia_upconv_blur_bwd(const void* gy, void* gt, int N, int R, int C, int dtype, void* stream);
/* Input gradient of the transposed conv = stride-2, pad-0 3×3 conv over gT with w_t =
 * [Cin][9·Cout] (W[co][ci][ky][kx] at (ky·3+kx)·Cout + co, no flip); epilogue gx = acc·style and
 * sdot[n][ci] += Σ_p acc·act(x_fwd). gx: (N,R,R,Cin). */
int mia_upconv_dgrad(const void* g_t, const void* w_t, void* gx, int N, int R, int Cout, int Cin,
                     const void* x_fwd, int act_x, const float* style, float* sdot, int dtype,
                     void* stream);
/* The same with the fused backward front of the layer below (see mia_conv_args: gx += (torgb
 * part, accumulate), then bab_* on x_fwd = that layer's stored activation) — gx receives that
 * layer's demod-scaled pre-activation gradient directly. */
int mia_upconv_dgrad_fused(const void* g_t, const void* w_t, void* gx, int N, int R, int Cout,
                           int Cin, const void* x_fwd, const float* style, float* sdot,
                           int accumulate, const float* bab_demod, const float* bab_noise,
                           float bab_noise_w, const float* bab_bias, float* bab_q, int dtype,
                           void* stream);
/* mia_upconv_dgrad_fused with the split_f32 copy of w_t (fp32: the X6B tile, weights pre-split,
 * csrc/conv_mfma.hip; NULL → as mia_upconv_dgrad_fused). */
int mia_upconv_dgrad_fused_split(const void* g_t, const void* w_t, const void* w_t_split, void* gx,
                                 int N, int R, int Cout, int Cin, const void* x_fwd,
                                 const float* style, float* sdot, int accumulate,
                                 const float* bab_demod, const float* bab_noise, float bab_noise_w,
                                 const float* bab_bias, float* bab_q, int dtype, void* stream);

/* ---- elementwise / reduction kernels ----------------------------------------------------- */
/* FusedLeakyReLU + NoiseInjection forward, standalone (K4): y = lrelu(x + nw·noise + b)·√2 (NHWC). */
int mia_bias_act_fwd(const void* x, const float* noise, float noise_w, const float* bias,
                     void* y, int N, int H, int W, int C, int dtype, void* stream);
/* StyledConv backward front (K4 bwd + demod): from g_a = ∂L/∂a and pre:
 *   g_pre = g_a·lrelu_s2'(pre); q[n][c] += Σ_p g_pre·(pre − nw·noise − b); gy = g_pre·demod[n][c]
 * gy is written un-shuffled (N,H/2,W/2,4C) when unshuffle=1 (up-conv dgrad input).
 * from_act=1: the stored tensor is the activation a = lrelu(pre)·√2 (pre is recovered as
 * a / lrelu'(a), the sign of a and pre being equal). */
int mia_bias_act_bwd(const void* g_a, const void* pre, const float* noise, float noise_w,
                     const float* bias, const float* demod, void* gy, float* q, int N, int H,
                     int W, int C, int unshuffle, int from_act, int dtype, void* stream);
/* upfirdn2d (K3) on fp32 NCHW planes, separable 1-D kernel (taps ≤ 8):
 * zero-insert `up`, pad (pad0,pad1), correlate with the flipped kernel, keep every `down`-th. */
int mia_upfirdn2d_fwd(const float* x, float* y, int planes, int H, int W, const float* k1d,
                      int ktaps, int up, int down, int pad0, int pad1, void* stream);
int mia_upfirdn2d_bwd(const float* gy, float* gx, int planes, int H, int W, const float* k1d,
                      int ktaps, int up, int down, int pad0, int pad1, void* stream);
/* ToRGB (K5): rgb = Σ_ci act_in(x)·wr[c][ci]·s[n][ci] + bias[c] (+ upfirdn2d(skip, up 2, pad (2,1)))
 * pre NHWC (dtype), rgb/skip fp32 NCHW (N,3,H,W)/(N,3,H/2,W/2). */
int mia_torgb_fwd(const void* pre, const float* style, const float* wr, const float* bias,
                  const float* skip, float* rgb, int N, int H, int W, int Cin, int act_in,
                  int dtype, void* stream);
/* ToRGB backward: u = Σ_c g[c]·wr[c][ci]; g_a (+)= s·u; gs[n][ci] += Σ_p act(pre)·u. */
int mia_torgb_bwd(const float* g_rgb, const void* pre, const float* style, const float* wr,
                  void* g_a, float* gs, int N, int H, int W, int Cin, int accumulate, int act_in,
                  int dtype, void* stream);
/* ToRGB backward for the topmost StyledConv (its activation gradient is this ToRGB's alone),
 * fused with that conv's backward front (mia_bias_act_bwd, from_act=1): gy = demod·g·lrelu'(a),
 * q += Σ_p g·lrelu'(a)·(pre − noise_w·noise − bias); gs as mia_torgb_bwd. act: stored
 * activation (N,H,W,Cin). */
int mia_torgb_bwd_front(const float* g_rgb, const void* act, const float* style, const float* wr,
                        void* gy, float* gs, int N, int H, int W, int Cin, const float* demod,
                        const float* noise, float noise_w, const float* bias, float* q, int dtype,
                        void* stream);
/* MaxPool 2x2/2 (K8) NHWC, ceil_mode for odd sizes (code/vgg.py:14,18,24). */
int mia_maxpool2_fwd(const void* x, void* y, int N, int H, int W, int C, int ceil_mode,
                     int dtype, void* stream);
/* MaxPool backward per input pixel (first-max tie rule) + optional tap-MSE term and ReLU mask:
 *   g_in = [p is argmax]·g_out + tap_coef·(x − tap_t);  g_in *= (x > 0) if mask. */
int mia_maxpool2_bwd(const void* x, const void* g_out, void* g_in, int N, int H, int W, int C,
                     int ceil_mode, const void* tap_t, float tap_coef, int mask, int dtype,
                     void* stream);
/* avg_pool2d(k) on fp32 NCHW (K9; attack_main2.py:590-591) and its backward. */
int mia_avgpool_fwd(const float* x, float* y, int planes, int H, int W, int k, void* stream);
int mia_avgpool_bwd(const float* gy, float* gx, int planes, int H, int W, int k, int accumulate,
                    void* stream);
/* NCHW fp32 image (N,3,S,S) → avg_pool(pf) → NHWC (N,S/pf,S/pf,cpad) dtype, channels ≥3 zero. */
int mia_image_to_nhwc(const float* x, void* y, int N, int S, int pf, int cpad, int dtype,
                      void* stream);
/* coef·Σ over an image of (a − b)² for a [n][len] pair (dtype), into loss[n] (+=). K10 value. */
int mia_mse_sum(const void* a, const void* b, float* loss, int n, int64_t len, float coef,
                int dtype, void* stream);
/* K10 gradient for flat fp32 tensors: g (+)= coef·(a − b). */
int mia_mse_grad_f32(const float* a, const float* b, float* g, int64_t len, float coef,
                     int accumulate, void* stream);
/* The SURVEY.md §8(b) K10 pair in one call: loss[i] (+)= coef_loss·Σ_j (a − b)[i][j]² over the n
 * rows of len elements (mia_mse_sum; loss may be NULL) and g (+)= coef_grad·(a − b) (g may be
 * NULL; fp32: mia_mse_grad_f32, accumulate allowed; fp16 / bf16: mia_tap_grad without a mask,
 * accumulate = 0 only, else MIA_ERR_ARG). Replaces: F.mse_loss(reduction='mean') and its autograd
 * backward (interpolation.py:786-817; coef_loss = 1/len, coef_grad = 2/len for a mean). */
int mia_mse_fwd_bwd(const void* a, const void* b, float* loss, void* g, int n, int64_t len,
                    float coef_loss, float coef_grad, int accumulate, int dtype, void* stream);
/* Tap-MSE seed for the deepest VGG tap: g = coef·(a − t)·[a > 0 if mask] (dtype, flat). */
int mia_tap_grad(const void* a, const void* t, void* g, int64_t len, float coef, int mask,
                 int dtype, void* stream);
/* d(image) of the reconstruction: g_img = coef·(rec − t) + unpool_pf(g_vgg[n,y,x,c]) (fp32 NCHW). */
int mia_image_grad(const float* rec, const float* t, const void* g_vgg, float* g_img, int N,
                   int S, int pf, int cpad, float coef, int dtype, void* stream);
/* Sign-project step (K11, interpolation.py:92-94, cost = −L):
 *   g = unpool_pf(g_vgg)/pf² + coef_img·(x − x0) + unpool(g_enc)/(pool_enc²)   [fp32]
 *   adv = x + a·sign(−g); δ = clamp(adv − x0, −e, e); x = clamp(x0 + δ, lo, hi)   (in place)
 * g_vgg may be NULL; g_enc may be NULL (else (N,3,enc_res,enc_res) fp32).
 * nonfinite: NULL or int[N]; set to 1 for every image with a non-finite gradient element (an
 * fp16 loss-scale overflow: the host lowers the scale and re-runs). */
int mia_pgd_update(float* x, const float* x0, const void* g_vgg, const float* g_enc, int N,
                   int S, int pf, int cpad, int enc_res, float coef_img, float a, float e,
                   float lo, float hi, int* nonfinite, int dtype, void* stream);
/* PGD random start (torchattacks PGD.forward, interpolation.py:73-76): x = clamp(x0 + e·u, lo, hi),
 * u = host-seeded U(-1,1) draws. */
/* ∇_x L as an fp32 image: scale·(coef_img·(x − x0) + avg_pool adjoints of the VGG input-path
 * gradient g_vgg (N,S/pf,S/pf,cpad; dtype) and of the encoder gradient g_enc (N,3,enc_res²)).
 * The gradient the fused PGD update (mia_pgd_update) projects, materialised for the Adam
 * (optimize_vgg, interpolation.py:767,822) and C&W modes. */
int mia_grad_assemble(const float* x, const float* x0, const void* g_vgg, const float* g_enc,
                      float* g, int N, int S, int pf, int cpad, int enc_res, float coef_img,
                      float scale, int* nonfinite, int dtype, void* stream);
/* C&W L2 in tanh space (torchattacks CW, interpolation.py:98-193), images in [-1,1]:
 * w = atanh(x) (x clamped to ±(1 − 2^-20)); adv = tanh(w);
 * g_w = (½(adv − x) + c·scale·g_f)·(1 − adv²) for cost = Σ‖(adv − x)/2‖² + c·Σ f(adv);
 * select: per image n, if f[n] < f0[n] and l2_scale·sq[n] < best_l2[n], best_adv[n] = adv[n]. */
int mia_cw_init(const float* x, float* w, int64_t len, void* stream);
int mia_cw_tanh(const float* w, float* adv, int64_t len, void* stream);
int mia_cw_grad(const float* adv, const float* x, const float* g_f, float* g_w, int64_t len,
                float c, float scale, void* stream);
int mia_cw_select(const float* adv, float* best_adv, const float* sq, float* best_l2,
                  const float* f, const float* f0, int N, int64_t plane, float l2_scale,
                  void* stream);
int mia_random_start(float* x, const float* x0, const float* u, int64_t len, float e, float lo,
                     float hi, void* stream);
/* K11 alone, given a full fp32 gradient (bit-exact contract vs torch fp32). */
int mia_sign_project(float* x, const float* x0, const float* g, int64_t len, float a, float e,
                     float lo, float hi, void* stream);
/* Adversarial patch step (code/attack/patch/adversarial_patch.py:131-134): patch −= g;
 * adv = clamp((1 − mask)·img + mask·patch, lo, hi), lo / hi = min / max of the clean images
 * (:134). g = NULL: the composite only (patch_white_box, attack_main2.py:413-420). mask / patch
 * have img's shape (shared = 0) or one image's shape broadcast over the batch (shared = its
 * numel; composite only). Bit-exact vs torch fp32 ops. */
int mia_patch_update(float* patch, const float* g, const float* img, const float* mask,
                     float* adv, int64_t len, int64_t shared, float lo, float hi, void* stream);
/* Adam on pixels (K12, optim.Adam at interpolation.py:767,822): fp32 state, step t ≥ 1. */
int mia_adam_step(float* p, const float* g, float* m, float* v, int64_t len, float lr,
                  float beta1, float beta2, float eps, int t, void* stream);

/* ---- small fp32 linear algebra (styles, demod, encoder) ----------------------------------- */
/* C[m,n] = alpha·Σ_k A[m*sam + k*sak]·B[k*sbk + n*sbn] + beta·C[m*scm + n*scn] + bias[n] */
int mia_gemm_f32(int M, int Nn, int K, float alpha, const float* A, int64_t sam, int64_t sak,
                 const float* B, int64_t sbk, int64_t sbn, float beta, float* C, int64_t scm,
                 int64_t scn, const float* bias, void* stream);
/* Grouped form: up to any number of independent fp32 products in as few launches as possible
 * (12 groups per launch). Group g computes C = alpha·Σ_{s<nseg} A_s·B_s + beta·C + bias with
 * strided operands as in mia_gemm_f32; nseg ≤ 2 sums two K-ranges (e.g. the two modulated layers
 * that read one W+ latent row, K6 backward). `groups` is a HOST array; its pointers are device
 * pointers. Groups must not alias each other's C. */
typedef struct mia_gemm_seg {
  const float* A;
  const float* B;
  int64_t sam, sak, sbk, sbn;
  int K;
} mia_gemm_seg;
typedef struct mia_gemm_group {
  float* C;
  const float* bias; /* [N] or NULL */
  int64_t scm, scn;
  int M, N;
  float alpha, beta;
  int nseg;
  mia_gemm_seg seg[2];
} mia_gemm_group;
int mia_gemm_f32_grouped(const mia_gemm_group* groups, int ngroups, void* stream);
/* y[n][d] = Σ_s x[n][s][d] (fp32): e4e's latent-gradient rows that all read style 0
 * (Encoder4Editing: w[:, i] = style_0(c3) + delta_i, so ∂style_0 = Σ_i ∂w[:, i]). */
int mia_sum_slices(const float* x, float* y, int N, int S, int D, void* stream);
/* demod[n][co] = rsqrt(scale2·Σ_ci s[n][ci]²·wsq[co][ci] + 1e-8)  (ModulatedConv2d demod [ext]) */
int mia_style_demod(const float* s, const float* wsq, float* demod, int N, int Cin, int Cout,
                    float scale2, void* stream);
/* gs[n][ci] += −scale2·s[n][ci]·Σ_co q[n][co]·demod[n][co]²·wsq[co][ci] */
int mia_demod_bwd(const float* q, const float* demod, const float* wsq, const float* s, float* gs,
                  int N, int Cin, int Cout, float scale2, void* stream);
/* Mapping-network plumbing for the fusion entry point (style_fusion_simple.py:110-142 via the
 * rosinality Generator [ext]): PixelNorm y = x / sqrt(mean_row(x²) + eps) (fp32 [rows][cols]);
 * truncation out = mean + psi·(w − mean) with mean [cols] broadcast over rows. */
int mia_pixel_norm(const float* x, float* y, int rows, int cols, float eps, void* stream);
int mia_truncate(const float* w, const float* mean, float psi, float* out, int rows, int cols,
                 void* stream);
/* dst[i*bytes .. ] = src for i < count (broadcast the constant input over the batch). */
int mia_repeat(const void* src, void* dst, int64_t bytes, int count, void* stream);

/* ---- e4e encoder (Encoder4Editing(50, 'ir_se'), un-vendored; code/utils/model_utils.py:24) --
 * NHWC dtype feature maps, fp32 per-(n,c) vectors. Eval-mode BatchNorm is a per-channel affine
 * y = x·g + b folded on the host. SEModule(C, 16) of bottleneck_IR_SE:
 *   mia_se_fwd:  avg = csum/hw; u = relu(W1·avg) (N,C/16); s = sigmoid(W2·u) (N,C)
 *                W1 [C/16][C], W2 [C][C/16] fp32.
 *   mia_se_apply: out = r·s[n][c] + sc  (sc: NHWC (N, H·ss, W·ss, C) read at (ss·y, ss·x), ss = 1
 *                 or 2 = MaxPool2d(1, 2) shortcut; NULL → none; s NULL → 1); xb = out·g[c] + b[c]
 *                 (the next unit's BatchNorm, optional); out may be NULL when only xb is wanted.
 *   mia_chan_dot: gs[n][c] (+)= Σ_p a·b  (fp32 out)
 *   mia_se_bwd:  from gs = ∂L/∂s: gz = gs·s(1−s); gu = (W2ᵀ gz)·[u > 0]; gavg = W1ᵀ gu / hw
 *   mia_se_fwd_parts / mia_se_bwd_parts: the same, with csum / gs given as mia_chan_sum's nch
 *                 ordered pixel-chunk partials (mia_chan_sum with out NULL) and summed in chunk
 *                 order inside the kernel: bit-identical to mia_chan_sum + mia_se_fwd / _bwd, one
 *                 launch fewer per SE module
 *   mia_se_grad_scale: g_r = gamma[c]·(g_out·s[n][c] + gavg[n][c])  (gamma NULL → 1)
 *   mia_prelu_bwd_scale: g = g_a·(a > 0 ? 1 : slope[c])·gamma[c]  (gamma NULL → 1); `a` is the
 *                 stored activation when every slope is ≥ 0, else the pre-activation
 *   mia_prelu_fwd: a = pre > 0 ? pre : slope[c]·pre (the e4e units with a negative PReLU slope,
 *                 whose conv writes pre for the backward's branch mask; round 6)
 *   mia_cast: y = scale·x converted between dtypes (x, y: flat, n elements)
 *   mia_subsample_add: gx[n][2y][2x][c] += g[n][y][x][c]   (MaxPool2d(1,2) adjoint)
 *   mia_bilinear_fwd/bwd: F.interpolate(mode='bilinear', align_corners=True) (N,Hi,Wi,C) →
 *                 (N,Ho,Wo,C) and its adjoint (gather form, no atomics); accumulate adds to out. */
int mia_se_fwd(const float* csum, const float* w1, const float* w2, float* u, float* s, int N,
               int C, int Cr, float inv_hw, void* stream);
int mia_se_apply(const void* r, const float* s, const void* sc, int ss, void* out,
                 const float* g, const float* b, void* xb, int N, int H, int W, int C, int dtype,
                 void* stream);
int mia_chan_dot(const void* a, const void* b, float* gs, int N, int HW, int C, int accumulate,
                 int dtype, void* stream);
/* Deterministic per-(image, channel) sums over the pixels of (N, HW, C) NHWC tensors:
 * out[n][c] (+)= Σ_p a·b (b given: the SE gate gradient Σ ∂out·r, as mia_chan_dot) or Σ_p a
 * (b NULL: the SE average pool's sum, psp_encoders SEModule AdaptiveAvgPool2d, reached through
 * net.encoder at code/attack/attack_main2.py:597,622). Fixed-order reduction through `part`
 * (fp32 scratch of N · mia_chan_sum_parts(N, HW) · C floats): bit-reproducible run to run.
 * out NULL (accumulate 0): only the partials part[(n·nch + q)·C + c] are written. */
int mia_chan_sum_parts(int N, int HW);
int mia_chan_sum(const void* a, const void* b, float* part, float* out, int N, int HW, int C,
                 int accumulate, int dtype, void* stream);
int mia_se_bwd(const float* gs, const float* s, const float* u, const float* w1, const float* w2,
               float* gavg, int N, int C, int Cr, float inv_hw, void* stream);
int mia_se_fwd_parts(const float* part, int nch, const float* w1, const float* w2, float* u,
                     float* s, int N, int C, int Cr, float inv_hw, void* stream);
int mia_se_bwd_parts(const float* part, int nch, const float* s, const float* u, const float* w1,
                     const float* w2, float* gavg, int N, int C, int Cr, float inv_hw,
                     void* stream);
int mia_se_grad_scale(const void* g_out, const float* s, const float* gavg, const float* gamma,
                      void* g_r, int N, int HW, int C, int dtype, void* stream);
int mia_prelu_bwd_scale(const void* g_a, const void* a, const float* slope, const float* gamma,
                        void* g, int64_t pixels, int C, int dtype, void* stream);
int mia_prelu_fwd(const void* pre, const float* slope, void* a, int64_t pixels, int C, int dtype,
                  void* stream);
int mia_subsample_add(const void* g, void* gx, int N, int H, int W, int C, int dtype,
                      void* stream);
int mia_cast(const void* x, int xdtype, void* y, int ydtype, int64_t n, float scale,
             void* stream);
int mia_bilinear_fwd(const void* x, void* y, int N, int Hi, int Wi, int Ho, int Wo, int C,
                     int accumulate, int dtype, void* stream);
int mia_bilinear_bwd(const void* gy, void* gx, int N, int Hi, int Wi, int Ho, int Wo, int C,
                     int accumulate, int dtype, void* stream);
int mia_memset(void* dst, int value, int64_t bytes, void* stream);

/* ---- fusion evaluation (§8f rank 2): cal_SSMI / cal_result, interpolation.py:903-919,1076-1091 -
 * SSIM of ref (3,H,W) against each of imgs (N,3,H,W), fp32 NCHW, the way cal_SSMI calls
 * skimage.metrics.structural_similarity on rgb2gray images (7×7 uniform window, sample
 * covariance, K1 0.01, K2 0.03, border of 3 cropped). work: device scratch of
 * work_bytes ≥ mia_ssim_workspace_size(N, H, W) bytes (one fp64 partial per image and 32×32
 * output tile, summed in tile order: deterministic, batch-independent); a smaller work_bytes is
 * MIA_ERR_ARG. (Replaces round 3's size-less mia_ssim, whose scratch contract changed.) */
int64_t mia_ssim_workspace_size(int N, int H, int W);
int mia_ssim2(const float* ref, const float* imgs, int N, int H, int W, float data_range,
              double* work, int64_t work_bytes, float* ssim_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MIATTACK_H */
