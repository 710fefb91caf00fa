/*
 * audiolcm_hip.h — C-ABI of libaudiolcm_hip.so, the MI355X (gfx950) hot path of
 * AudioLCM text-to-audio inference.
 *
 * Conventions:
 *   - every entry point is `extern "C" int fn(...)`: 0 on success, a negative
 *     ALCM_E* code otherwise; alcm_last_error() returns a thread-local message;
 *   - every tensor argument is a caller-allocated DEVICE pointer (typically a
 *     torch tensor's data_ptr()) in the reference's own layout unless stated,
 *     fp32, contiguous; sizes are explicit;
 *   - work is enqueued on the caller's hipStream_t (torch.cuda.current_stream());
 *     no call allocates device memory except the *_create loaders, no call
 *     synchronises the host;
 *   - concurrency: calls on one model handle from different host threads and/or
 *     different caller streams may overlap, provided each concurrent call has its
 *     own workspace and output buffers.  The handle's packed weights are read-only
 *     after *_create; the only per-handle mutable state is the set of auxiliary
 *     streams/events alcm_bigvgan_forward forks its resblock chains onto, which is
 *     kept per CALLER stream (created under a lock on that stream's first call), so
 *     concurrent calls never share an event.  alcm_model_set_precision /
 *     alcm_model_set_resblock_streams must not race with calls on the same handle.
 *     Two calls on the SAME caller stream are ordered by that stream;
 *   - no torch types cross the boundary.
 *
 * Reference interfaces replaced (paths under the reference checkout):
 *   alcm_dit_*          ConcatDiT2MLP.forward          ldm/modules/diffusionmodules/concatDiT.py:282-304
 *                       (called as LCM_audio.apply_model, ldm/models/diffusion/lcm_audio.py:479-502)
 *   alcm_lcm_step       LCMSampler.step (eps branch)   ldm/models/diffusion/scheduling_lcm.py:410-496
 *   alcm_*_embedding    get_guidance_scale_embedding   scheduling_lcm.py:87-113
 *                       TimestepEmbedder.timestep_embedding  concatDiT.py:49-67
 *   alcm_vae_*          LCM_audio.decode_first_stage   lcm_audio.py:392-406 -> AutoencoderKL.decode
 *                       autoencoder1d.py:59-62, Decoder1D.forward autoencoder1d.py:484-517
 *   alcm_bigvgan_*      BigVGAN.forward                vocoder/bigvgan/models.py:181-203
 *                       (VocoderBigVGAN.vocode, models.py:406-411)
 *   alcm_activation1d   Activation1d.forward           vocoder/bigvgan/alias_free_torch/act.py:23-27
 *   alcm_gemm           aten conv1d / conv_transpose1d / linear / bmm on the path (SURVEY.md §2 kernel inventory)
 */
#ifndef AUDIOLCM_HIP_H
#define AUDIOLCM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* alcm_stream_t; /* hipStream_t */

enum {
  ALCM_OK = 0,
  ALCM_E_INVALID = -1,  /* bad argument / shape */
  ALCM_E_HIP = -2,      /* HIP runtime error */
  ALCM_E_MISSING = -3,  /* required weight tensor missing */
  ALCM_E_WORKSPACE = -4 /* workspace too small */
};

/* ---------------------------------------------------------------- misc */
const char* alcm_last_error(void);
int alcm_version(void);
/* device properties check: returns 0 if device `dev` is gfx950 */
int alcm_check_device(int dev);

/* ---------------------------------------------------------------- generic MFMA GEMM / implicit-GEMM conv1d
 * C[m][n] = epilogue( sum_k A[m][k] * B[n][k] ), MFMA with fp32 accumulate.  Operand precision `prec`:
 *   ALCM_PREC_BF16  (0) one v_mfma_f32_16x16x32_bf16 (operands rounded to bf16)
 *   ALCM_PREC_SPLIT (1) 3-term bf16 split (hi*hi + hi*lo + lo*hi): fp32-level accuracy, 3x the MFMA work
 *   ALCM_PREC_F16   (2) one v_mfma_f32_16x16x32_f16 (operands rounded to fp16)
 *   ALCM_PREC_F16W2 (3) fp16 activation x fp16 hi+lo weight, 2 MFMAs (alcm_opconv only) */
enum { ALCM_PREC_BF16 = 0, ALCM_PREC_SPLIT = 1, ALCM_PREC_F16 = 2, ALCM_PREC_F16W2 = 3 };
enum { ALCM_OPND_ACT = 0, ALCM_OPND_ACT_T = 1, ALCM_OPND_WEIGHT = 2 };

typedef struct alcm_operand {
  int kind;
  const void* ptr;
  /* ACT: element (b, t, c) at ptr + b*sb + t*st + c*sc; K index k = tap*Cpad + ci, source time
   *      t_src = t + tap*dil - pad (up == 2: nearest-x2 upsampled input, t_up = t + tap*dil - pad,
   *      t_src = t_up/2), zero outside [0, T_in) / ci >= C_in / k >= ksize*Cpad.
   * ACT_T: element (n, k) at ptr + k*st + n*sc, valid k < T_in, n < rows.
   * WEIGHT: packed [rows][Kpad] planes: bf16 hi at ptr, bf16 lo at ptr + w_lo_off, fp16 hi at
 *         ptr + 2*w_lo_off, fp16 lo at ptr + 3*w_lo_off (elements; w_lo_off = rows*Kpad as written by
 *         alcm_pack_conv_weight). */
  int64_t sb, st, sc;
  int T_in, C_in, Cpad, ksize, dil, pad, up;
  int rows_per_batch; /* ACT: rows m -> (b = m / rows_per_batch, t = m % rows_per_batch) */
  int rows;           /* ACT_T / WEIGHT: number of valid rows */
  int64_t zs1, zs2;   /* batched offset (z / zdiv)*zs1 + (z % zdiv)*zs2 */
  /* ACT prologue, applied to valid (non-padding) elements: v = (v - mean[b*T_in+t_src]) * rstd[...]
   * (if pro_mean), v = v*pro_scale[b*pro_sb+c] + pro_shift[...] (if pro_scale), v = act(v)
   * with pro_act 0 (none) or 1 (SiLU); other codes are rejected with ALCM_E_INVALID */
  const float* pro_scale;
  const float* pro_shift;
  int64_t pro_sb;
  const float* pro_mean;
  const float* pro_rstd;
  int pro_act;
  int64_t w_lo_off;
} alcm_operand;

typedef struct alcm_gemm_args {
  int M, N, Kpad; /* Kpad: multiple of 32 covering the real K */
  int batch, zdiv;
  alcm_operand a, b;
  /* activation codes: 0 none, 1 SiLU, 2 GELU (erf), 3 GELU (tanh), 4 tanh
   * epilogue: v = acc*acc_scale + bias[n]; v = act(v) (geglu 1: v_even * gelu_erf(v_odd) -> column n/2,
 *           geglu 2: v_even * gelu_tanh(v_odd), T5's gated-gelu with (wi_1, wi_0) rows interleaved);
   *           v += res[...]; v *= out_scale; if accumulate v += out[...]; out[...] = v
   * output row m -> (b, t), stored at out + zoff + b*o_sb + (t*out_step + out_off)*o_st + n*o_sc */
  const float* bias;
  float acc_scale, out_scale;
  int act, accumulate, geglu;
  const float* res;
  int64_t r_sb, r_st, r_sc, r_zs1, r_zs2;
  float* out;
  int64_t o_sb, o_st, o_sc, o_zs1, o_zs2;
  int out_rows_per_batch, out_step, out_off;
  int prec;           /* ALCM_PREC_* */
  int disable_window; /* 1: never use the window-conv kernel (testing / A-B timing) */
  int tile_n;         /* 0: automatic; 64 / 128: force the N tile of the window-conv kernel */
} alcm_gemm_args;

int alcm_gemm(const alcm_gemm_args* args, alcm_stream_t stream);

/* pack a conv/linear weight W[co][ci][k] (fp32, DEVICE) into four [Cout][Kpad] planes (bf16 hi, bf16 lo,
 * fp16 hi, fp16 lo) with K index = tap*Cpad + ci. transposed=1 takes a ConvTranspose1d weight [ci][co][k]
 * and a phase (stride s, phase r) selecting taps j = r + s*(Q-1-tap), Q = k/s. out must hold 4*Cout*Kpad u16. */
int alcm_pack_conv_weight(const float* w, int c_out, int c_in, int k, int cpad, int kpad, int transposed,
                          int stride, int phase, void* out, alcm_stream_t stream);

/* ---------------------------------------------------------------- normalisation / elementwise
 * Layout of x for the norm kernels: element (b, t, c) at x + b*sb + t*st + c (channels contiguous). */
int alcm_group_norm_affine(const float* x, int B, int T, int C, int64_t sb, int64_t st, int groups,
                           float eps, const float* gamma, const float* beta, float* scale_out,
                           float* shift_out, alcm_stream_t stream);
int alcm_row_stats(const float* x, int rows, int C, int64_t ld, float eps, float* mean, float* rstd,
                   alcm_stream_t stream);
int alcm_layer_norm(const float* x, int rows, int C, int64_t ld_in, float eps, const float* gamma,
                    const float* beta, const float* add, int64_t ld_add, float* y, int64_t ld_out,
                    alcm_stream_t stream);
int alcm_softmax_rows(float* x, int rows, int n, int64_t ld, alcm_stream_t stream);
/* LayerNorm of rows (row stride ld) written as an MFMA operand plane [rows][C] (prec PREC_F16 (2) or
 * PREC_BF16 (0)) for alcm_opconv (the DiT feed-forward input, concatDiT.py:120-125) */
int alcm_layer_norm_plane(const float* x, int rows, int C, int64_t ld, float eps, const float* gamma,
                          const float* beta, void* plane, int prec, alcm_stream_t stream);
/* fused Activation1d(SnakeBeta): x,y DEVICE (b,t,c) channels-last, not in place; alpha_exp = exp(alpha),
 * inv_beta = 1/(exp(beta)+1e-9) per channel (DEVICE); up_filter/down_filter: HOST arrays of 12 taps */
int alcm_activation1d(const float* x, float* y, int B, int T, int C, int64_t sb, int64_t st,
                      const float* alpha_exp, const float* inv_beta, const float* up_filter,
                      const float* down_filter, alcm_stream_t stream);

/* ---------------------------------------------------------------- operand-format AMPBlock path
 * (vocoder/bigvgan/models.py:72-81 as Activation1d -> conv, alcm_opconv.hip)
 * alcm_activation1d_op: Activation1d of x (B,T,C) fp32 channels-last DEVICE into MFMA operand planes
 *   y [B][T][Cp] of 2-byte elements (Cp = multiple of 32 >= C, channels >= C written as 0): prec
 *   ALCM_PREC_F16 / F16W2 -> one fp16 plane; BF16 -> one bf16 plane; SPLIT -> bf16 hi plane at y and
 *   bf16 lo plane at y + B*T*Cp.  alpha_exp / inv_beta DEVICE, filters HOST (12 taps). */
int alcm_activation1d_op(const float* x, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                         const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                         alcm_stream_t stream);
/* alcm_activation1d_op_f16in: alcm_activation1d_op (alias_free_torch/act.py:23-27) of an fp16 plane x16 [B][T][C]
 *   DEVICE — the BigVGAN AMPBlock conv1 output written by alcm_opconv's out_plane epilogue (vocoder/bigvgan/
 *   models.py:74-79: that conv's only consumer is this activation) — into fp16 planes y [B][T][C].  Only the shapes
 *   whose FIR input alcm_activation1d_op rounds to fp16 anyway: prec ALCM_PREC_F16, C >= 192, C % 64 == 0, Cp == C,
 *   16-byte aligned x16 / y; the result equals alcm_activation1d_op on the fp32 conv output bit for bit.
 *   ALCM_E_INVALID otherwise. */
int alcm_activation1d_op_f16in(const void* x16, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                               const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                               alcm_stream_t stream);
/* alcm_opconv: out (B,T,N) = conv_{ksize,dil}(a) with same-length zero padding (2*pad == (ksize-1)*dil)
 * on operand planes a (as written by alcm_activation1d_op, lo plane a_lo_off elements after hi), weights
 * packed by alcm_pack_conv_weight with cpad = Cp; epilogue as alcm_gemm: v = acc + bias[n];
 * v = act(v); v += res; v *= out_scale; if accumulate v += out.  prec: BF16 / SPLIT / F16 / F16W2
 * (must match the planes a holds); C = real input channels (cost accounting). */
/* Zero-initialise the whole struct (memset / `= {0}`) before setting fields: optional trailing fields (act_*, geglu_plane,
 * out_stride / out_offset / out_rows, out_plane) are read as "off" only when zero, and later versions append more. */
typedef struct alcm_opconv_args {
  const void* a;
  int64_t a_lo_off;
  int B, T, C, Cp;
  int ksize, dil, pad;
  const void* w;
  int64_t w_lo_off;
  int kpad, N;
  const float* bias;
  const float* res;
  float* out;
  int out_act, accumulate;
  float out_scale;
  int prec;
  /* optional fused Activation1d epilogue (alias_free_torch/act.py:23-27 applied to v = conv + bias (+ res)):
   * when act_plane != NULL the kernel also writes Activation1d(v) as MFMA operand planes [B][T][Cp'] with
   * Cp' = round_up(N, 32), in the format `prec` reads (SPLIT: lo plane act_plane_lo_off elements after hi),
   * ready for the next conv.  `out` may then be NULL (no fp32 output).  Tiles recompute 8 halo rows, so
   * `out` must not overlap `res`.  alpha_exp / inv_beta are device arrays of N (exp(alpha),
   * 1/(exp(beta)+1e-9)); the 12-tap filters are HOST arrays.  Requires out_act == 0 and N even. */
  void* act_plane;
  int64_t act_plane_lo_off;
  const float* act_alpha_exp;
  const float* act_inv_beta;
  const float* act_up_filter;
  const float* act_down_filter;
  /* optional GEGLU epilogue (new_attention.py:48-55 with value/gate rows interleaved: output columns 2j, 2j+1
   * = value j, gate j): when geglu_plane != NULL the kernel writes (v_2j + b_2j) * gelu_erf(v_2j+1 + b_2j+1)
   * as an operand plane [B][T][N/2] in the format of `prec` (F16 / BF16) instead of the fp32 output; needs
   * res == NULL, out_act == 0 and the wide-layer kernel (N % 128 == 0, Cp % 64 == 0). */
  void* geglu_plane;
  /* optional strided output (one phase of a ConvTranspose1d, vocoder/bigvgan/models.py:160-165): when
   * out_stride > 0, output row t of batch b is row t * out_stride + out_offset of an fp32 [B][out_rows][N]
   * `out`, and `pad` may be any value in [0, (ksize-1)*dil] (input row t - pad + tap*dil, zero outside).
   * Needs F16/BF16, N % 192 == 0, Cp % 64 == 0 and no res / accumulate / out_act / act / GEGLU.
   * 0 (the zero-initialised default): same-length conv, out is [B][T][N]. */
  int out_stride, out_offset, out_rows;
  /* optional operand-plane output: when out_plane != NULL the kernel writes conv + bias as an F16 / BF16 plane
   * [B][T][N] (the format of `prec`) instead of the fp32 `out` (which may be NULL) — for a consumer that rounds to
   * that format anyway (the DiT q/k/v projection feeding the fused attention).  Needs the wide-layer kernel
   * (F16 / BF16, N % 4 == 0, Cp % 64 == 0) and no res / accumulate / out_act / act / GEGLU / strided output. */
  void* out_plane;
  /* optional K-split workspace (fp32, 16-byte aligned, ksplit_ws_floats floats): where the persistent wide-layer
   * kernel's grid would not fill the chip (the DiT FFN down-projection: 192 tiles of 256 x 192 on 256 CUs), the
   * library may split the 64-channel K chunks into P parts (P * B * T * N <= ksplit_ws_floats), write P fp32
   * partial slices here and reduce them in part order with the bias / residual / scale / accumulate epilogue (a
   * second launch on the same stream): deterministic, not bit-identical to the unsplit sum.  NULL: never split. */
  float* ksplit_ws;
  int64_t ksplit_ws_floats;
} alcm_opconv_args;
int alcm_opconv(const alcm_opconv_args* args, alcm_stream_t stream);
/* alcm_opconv_sum: out = (sum over i < n of conv_i(args[i].a) + args[i].bias + args[i].res) * args[0].out_scale
 *   (+ out when args[0].accumulate), 1 <= n <= 3 — the mean over a BigVGAN stage's resblocks (vocoder/bigvgan/
 *   models.py:190-199: xs += resblock_j(x); x = xs / num_kernels) taken at the chains' last conv2 + residual
 *   (models.py:76-80), so the stage output is written once instead of read and rewritten per chain.  Each term is
 *   an alcm_opconv same-length conv with its own planes, weights, ksize / pad, bias and residual; the terms share B,
 *   T and N, and only args[0]'s out / out_scale / accumulate are read (another term's out must be NULL or the same).
 *   Three F16 / BF16 terms of dilation 1 with Cp % 64 == 0 and N % 192 == 0 run as one launch summing all taps in one
 *   fp32 accumulator; otherwise the terms run in order, each accumulating into out (the same value up to fp32
 *   rounding order).  No activation / plane / GEGLU / strided outputs. */
int alcm_opconv_sum(const alcm_opconv_args* args, int n, alcm_stream_t stream);
/* alcm_opconv_dense: the narrow AMPBlock conv of BigVGAN stages 3-5 (vocoder/bigvgan/models.py:72-81, C = N in
 * {24, 48} at F16 / F16W2, 96 at F16; ksize <= 11, (ksize-1)*dil <= 64) with the weights resident in LDS: same
 * arguments as alcm_opconv except that w is packed by alcm_pack_conv_weight with cpad = C (dense K = tap*C + c,
 * kpad = round_up(ksize*C, 32)); the planes a may be wider (Cp > C: channels >= C are ignored) and the fused
 * Activation1d writes only channels < N of its planes.  Epilogues: act (conv1), res + out + act (conv2), res + out
 * with out_scale and accumulate, no act (a resblock's last conv2).  ALCM_E_INVALID for anything else. */
int alcm_opconv_dense(const alcm_opconv_args* args, alcm_stream_t stream);

/* alcm_flash_attention: multi-head self-attention of the DiT (CrossAttention with context = x,
 * ldm/modules/new_attention.py:89-130, the q/k/v projections already applied):
 * out[b, i, h*dh:(h+1)*dh] = softmax_j(q_i . k_j * dh^-1/2) v_j per head, scores kept on chip.
 * qkv: (B, L, 3H) fp32 DEVICE rows [q | k | v] (16-byte aligned), out: (B, L, H) fp32; dh = H / heads <= 72;
 * prec: ALCM PREC_F16 (2) or PREC_BF16 (0) operand rounding of q, k, v and the probabilities. */
int alcm_flash_attention(const float* qkv, float* out, int B, int L, int H, int heads, int prec, alcm_stream_t stream);

/* ---------------------------------------------------------------- LCM scheduler pieces */
/* coeffs (HOST array of 6): {sqrt_a, sqrt_b, c_out, c_skip, sqrt_a_prev, sqrt_b_prev};
 * noise may be NULL (final step: prev_out = denoised) */
int alcm_lcm_step(const float* x, const float* eps, const float* noise, const float* coeffs,
                  float* prev_out, float* denoised_out, int64_t n, alcm_stream_t stream);
/* classifier-free-guidance variant (config 4): eps = eps_uncond + cfg_scale*(eps_cond - eps_uncond)
 * (plms.py:184-186 / ddim.py:203-205) fused into the same step */
int alcm_lcm_step_cfg(const float* x, const float* eps_cond, const float* eps_uncond, float cfg_scale,
                      const float* noise, const float* coeffs, float* prev_out, float* denoised_out, int64_t n,
                      alcm_stream_t stream);
/* out[b] = [f(v[b]*vscale*freqs[i]) ...]: cos_first ? [cos | sin] (TimestepEmbedder, concatDiT.py:49-67)
 *                                                   : [sin | cos] (get_guidance_scale_embedding, w*1000).
 * freqs: the reference's fp32 frequency table (half entries, device pointer) */
int alcm_sincos_embedding(const float* v, float vscale, const float* freqs, int B, int half, int cos_first,
                          float* out, alcm_stream_t stream);

/* ---------------------------------------------------------------- models
 * Weights are host fp32 tensors named by the reference state_dict keys. */
typedef struct alcm_named_tensor {
  const char* name;
  const float* data; /* HOST pointer, contiguous fp32 */
  int ndim;
  int64_t shape[4];
} alcm_named_tensor;

typedef struct alcm_model alcm_model;

/* kind: 0 = ConcatDiT2MLP, 1 = AutoencoderKL (decoder; + Encoder1D when encoder.* tensors are given), 2 = BigVGAN,
 * 3 = FrozenCLAPFLANEmbedder text encoders, 4 = log-mel front-end (NAT_mel.MelNet).
 * iconfig/fconfig: see DESIGN.md §C-ABI (hyper-parameters from configs/audiolcm.yaml / bigvgan json) */
enum { ALCM_MODEL_DIT = 0, ALCM_MODEL_VAE = 1, ALCM_MODEL_BIGVGAN = 2, ALCM_MODEL_TEXT = 3, ALCM_MODEL_MEL = 4 };
/* policy: ALCM_POLICY_* (below) */
int alcm_model_create(int kind, const int* iconfig, int n_iconfig, const alcm_named_tensor* tensors,
                      int n_tensors, int policy, alcm_model** out);
int alcm_model_destroy(alcm_model* m);
size_t alcm_model_weight_bytes(const alcm_model* m);
int alcm_model_set_split(alcm_model* m, int split);
/* per-layer precision policy: ALCM_POLICY_BF16 every contraction bf16; ALCM_POLICY_SPLIT every contraction
 * bf16x3 (fp32 parity); ALCM_POLICY_MIXED fp16 single MFMA on the layers the parity budget allows
 * (DiT GEGLU FFN convs, VAE k3 ResnetBlock/upsample convs, BigVGAN stage 0-2 AMPBlock convs: DESIGN.md §3),
 * bf16x3 elsewhere.  alcm_model_set_split(m, s) == set_precision(m, s ? SPLIT : BF16). */
enum { ALCM_POLICY_BF16 = 0, ALCM_POLICY_SPLIT = 1, ALCM_POLICY_MIXED = 2 };
int alcm_model_set_precision(alcm_model* m, int policy);
/* BigVGAN: run the three resblock chains of a stage concurrently on auxiliary streams forked from the caller's
 * stream (1, the default unless ALCM_SERIAL_RESBLOCKS is set at load) or serially on the caller's stream (0:
 * per-kernel timing, bench.py's roofline pass) */
int alcm_model_set_resblock_streams(alcm_model* m, int concurrent);
/* re-read the ALCM_* diagnostic environment switches (they are read once at library load) */
int alcm_reload_knobs(void);
/* diagnostics: the BigVGAN tail-conv phase trace (ALCM_TCONV_TRACE=1, which selects the tail convs' diagnostics
 * instantiations): shader-clock cycles summed over waves and tiles for [window + first slices, K loop, post-loop
 * barrier, staging, residual + state, Activation1d, final barrier] and the wave-tile count, since the last reset;
 * reset != 0 zeroes it.  The first call allocates the trace buffer and returns zeros (launches after it are traced).
 * Synchronizes the device.  ALCM_E_INVALID for a null out8. */
int alcm_debug_tconv_trace(unsigned long long* out8, int reset);
/* diagnostics: workgroup residency records of the last traced resident-weight tail conv (ALCM_TCONV_TRACE=1): per
 * workgroup [entry s_memrealtime, exit s_memrealtime, HW_ID, XCC_ID] into out (4 x n_wg values, at most 2048
 * workgroups); returns the count copied (0 before the first alcm_debug_tconv_trace call).  Synchronizes the device. */
int alcm_debug_tconv_wg_times(unsigned long long* out, int n_wg);

/* DiT.  x (B,C_lat,T) NCT, t (B,) int64, ctx (B,154,1024), w_emb (B,256) -> eps (B,C_lat,T) NCT.
 * cemb_cache: (B,154,hidden) device buffer filled by alcm_dit_embed_context (step-invariant, hoisted). */
size_t alcm_dit_workspace_bytes(const alcm_model* m, int B, int T);
int alcm_dit_embed_context(alcm_model* m, const float* ctx, int B, float* cemb_cache, void* ws,
                           size_t ws_bytes, alcm_stream_t stream);
int alcm_dit_forward(alcm_model* m, const float* x, const int64_t* t, const float* cemb_cache,
                     const float* w_emb, float* eps_out, int B, int T, void* ws, size_t ws_bytes,
                     alcm_stream_t stream);

/* VAE decode_first_stage. z (B,20,T) NCT -> mel (B,80,2T) NCT */
size_t alcm_vae_workspace_bytes(const alcm_model* m, int B, int T);
int alcm_vae_decode(alcm_model* m, const float* z, float inv_scale_factor, float* mel_out, int B, int T,
                    void* ws, size_t ws_bytes, alcm_stream_t stream);

/* VAE encode_first_stage (AutoencoderKL.encode, autoencoder1d.py:54-58 -> Encoder1D :319-413 + quant_conv):
 * mel (B,80,M) NCT -> posterior moments (B, 2*embed_dim, To) NCT = [mean | logvar] before the clamp,
 * To = alcm_vae_encode_len(m, M) (M/2 for audiolcm.yaml).  Needs a model created with encoder.* tensors. */
size_t alcm_vae_encode_workspace_bytes(const alcm_model* m, int B, int M);
int alcm_vae_encode(alcm_model* m, const float* mel, float* moments_out, int B, int M, void* ws, size_t ws_bytes,
                    alcm_stream_t stream);
int alcm_vae_encode_len(const alcm_model* m, int M);

/* Log-mel front-end (ldm/data/preprocess/NAT_mel.py:66-85, MelNet.forward with center=False): wav (B, L) fp32,
 * L % hop == 0 -> mel (B, n_mels, L/hop) NCT = log10(clamp(mel_basis @ |STFT(reflect_pad(clamp(wav)))|, 1e-5)).
 * Model kind ALCM_MODEL_MEL, iconfig {n_fft, hop, win, n_mels}, tensors "window" (win) and "mel_basis"
 * (n_mels, n_fft/2+1). */
size_t alcm_mel_workspace_bytes(const alcm_model* m, int B, int L);
int alcm_mel_spectrogram(alcm_model* m, const float* wav, float* mel_out, int B, int L, void* ws, size_t ws_bytes,
                         alcm_stream_t stream);

/* BigVGAN. mel (B,80,M) NCT -> wav (B,1,256*M) */
size_t alcm_bigvgan_workspace_bytes(const alcm_model* m, int B, int M);
int alcm_bigvgan_forward(alcm_model* m, const float* mel, float* wav_out, int B, int M, void* ws,
                         size_t ws_bytes, alcm_stream_t stream);

/* Text conditioning: FrozenCLAPFLANEmbedder.encode (ldm/modules/encoders/modules.py:567-582) from token ids.
 * clap_ids / t5_ids (B, L) int64 DEVICE (the CLAP-BERT and T5 tokenizers' input_ids, L <= max_len = 77,
 * ids in [0, vocab): out-of-range ids embed as zero rows) -> out (B, 2L, 1024) fp32 DEVICE =
 * [Projection(BERT(clap_ids)) | T5Encoder(t5_ids)], no attention mask (as the reference).
 * iconfig (14 ints): bert vocab, hidden, layers, heads, intermediate, max_position, projection out,
 * t5 vocab, d_model, d_kv, heads, d_ff, layers, max_len.  Tensors: caption_encoder.base.* (BertModel),
 * caption_encoder.projection.*, t5_transformer.* (T5EncoderModel) plus "_alcm.t5_rel_buckets" (max_len x
 * max_len, the bidirectional relative-position bucket of j - i as float). */
size_t alcm_text_workspace_bytes(const alcm_model* m, int B, int L);
int alcm_text_encode(alcm_model* m, const int64_t* clap_ids, const int64_t* t5_ids, float* out, int B, int L,
                     void* ws, size_t ws_bytes, alcm_stream_t stream);

/* ---------------------------------------------------------------- live kernel timing (bench.py roofline)
 * Between begin/end every kernel launch is bracketed by hipEvents on its stream; end synchronises
 * and returns per-kernel aggregates keyed by the demangled kernel name rocprofv3 reports.
 * flops/bytes are ALGORITHMIC (2*M*N*K for GEMMs; unique input + weight + output bytes). */
typedef struct alcm_prof_entry {
  char name[128];
  int64_t launches;
  double total_ms;
  double flops;
  double bytes;
  double roof_ms; /* sum over launches of max(flops/peak_flops, bytes/peak_bw) */
  /* the HBM-bound launches of this entry (algorithmic flops/bytes below peak_flops/peak_bw) */
  int64_t hbm_launches;
  double hbm_ms;
  double hbm_bytes;
} alcm_prof_entry;
int alcm_profile_begin(double peak_flops, double peak_bytes_per_s);
int alcm_profile_end(alcm_prof_entry* out, int max_entries, int* n_entries);

#ifdef __cplusplus
}
#endif
#endif /* AUDIOLCM_HIP_H */
