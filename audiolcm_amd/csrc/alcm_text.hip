// Small kernels of the text-conditioning encoders (FrozenCLAPFLANEmbedder, ldm/modules/encoders/modules.py:567-582):
// token-embedding gather, T5 RMSNorm statistics / apply, and the row softmax with T5's additive relative
// position bias.  The contractions (q/k/v/o projections, FFNs, attention QK^T / PV) run on the MFMA GEMM
// (alcm_gemm.hip).
#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

// out[r][:] = table[ids[r]][:] (+ add[(r % L)][:]); one 256-thread block per row, float4 lanes.
// Rows whose id is outside [0, vocab) are written as zeros (the host validates ids before upload).
__global__ __launch_bounds__(256) void embed_gather_kernel(const int64_t* __restrict__ ids,
                                                           const float* __restrict__ table, int64_t vocab, int D,
                                                           const float* __restrict__ add, int L,
                                                           float* __restrict__ out) {
  const int r = blockIdx.x;
  const int64_t id = ids[r];
  const bool ok = id >= 0 && id < vocab;
  const float4* src = reinterpret_cast<const float4*>(table + (ok ? id : 0) * (int64_t)D);
  const float4* ad = add ? reinterpret_cast<const float4*>(add + (int64_t)(r % L) * D) : nullptr;
  float4* dst = reinterpret_cast<float4*>(out + (int64_t)r * D);
  for (int c = threadIdx.x; c < D / 4; c += 256) {
    float4 v = ok ? src[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (ad) {
      const float4 a = ad[c];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    dst[c] = v;
  }
}

int embed_gather(const int64_t* ids, int rows, const float* table, int64_t vocab, int D, const float* add, int L,
                 float* out, hipStream_t s) {
  if (!ids || !table || !out || rows <= 0 || D <= 0 || D % 4 || L <= 0)
    return set_error(ALCM_E_INVALID, "embed_gather: bad arguments");
  hipLaunchKernelGGL(embed_gather_kernel, dim3(rows), dim3(256), 0, s, ids, table, vocab, D, add, L, out);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// T5LayerNorm statistics (no mean subtraction, no bias): mean[r] = 0, rstd[r] = 1/sqrt(mean(x^2) + eps),
// accumulated in fp32 as the reference (variance in float32).  One wave per row.
__global__ __launch_bounds__(256) void rms_stats_kernel(const float* __restrict__ x, int rows, int C, float eps,
                                                        float* mean, float* rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c] * xr[c];
  s = wave_sum(s);
  if (lane == 0) {
    mean[row] = 0.f;
    rstd[row] = 1.0f / sqrtf(s / (float)C + eps);
  }
}

int rms_stats(const float* x, int rows, int C, float eps, float* mean, float* rstd, hipStream_t s) {
  if (!x || !mean || !rstd || rows <= 0 || C <= 0) return set_error(ALCM_E_INVALID, "rms_stats: bad arguments");
  hipLaunchKernelGGL(rms_stats_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, eps, mean, rstd);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// y = weight * x * rsqrt(mean(x^2) + eps), row r written at out + (r / L) * out_sb + (r % L) * C
__global__ __launch_bounds__(256) void rms_norm_kernel(const float* __restrict__ x, int rows, int C, float eps,
                                                       const float* __restrict__ w, int L, int64_t out_sb,
                                                       float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c] * xr[c];
  const float r = 1.0f / sqrtf(wave_sum(s) / (float)C + eps);
  float* o = out + (int64_t)(row / L) * out_sb + (int64_t)(row % L) * C;
  for (int c = lane; c < C; c += 64) o[c] = w[c] * (xr[c] * r);
}

int rms_norm(const float* x, int rows, int C, float eps, const float* w, int L, int64_t out_sb, float* out,
             hipStream_t s) {
  if (!x || !w || !out || rows <= 0 || C <= 0 || L <= 0) return set_error(ALCM_E_INVALID, "rms_norm: bad arguments");
  hipLaunchKernelGGL(rms_norm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, eps, w, L, out_sb, out);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// T5LayerNorm straight into an MFMA operand plane (F16 / BF16, [rows][C]): the A operand of the following
// q/k/v or wi projection on the plane conv (alcm_opconv), instead of an fp32 prologue inside the GEMM
template <int PREC>
__global__ __launch_bounds__(256) void rms_plane_kernel(const float* __restrict__ x, int rows, int C, float eps,
                                                        const float* __restrict__ w, u16* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c] * xr[c];
  const float r = 1.0f / sqrtf(wave_sum(s) / (float)C + eps);
  u16* o = out + (int64_t)row * C;
  for (int c = 2 * lane; c < C; c += 128) {
    const float a = w[c] * (xr[c] * r), b = w[c + 1] * (xr[c + 1] * r);
    if constexpr (PREC == PREC_F16) {
      o[c] = __builtin_bit_cast(u16, (_Float16)a);
      o[c + 1] = __builtin_bit_cast(u16, (_Float16)b);
    } else {
      o[c] = __builtin_bit_cast(u16, (__bf16)a);
      o[c + 1] = __builtin_bit_cast(u16, (__bf16)b);
    }
  }
}

int rms_norm_plane(const float* x, int rows, int C, float eps, const float* w, void* out, int prec, hipStream_t s) {
  if (!x || !w || !out || rows <= 0 || C <= 0 || C % 2 || (prec != PREC_F16 && prec != PREC_BF16))
    return set_error(ALCM_E_INVALID, "rms_norm_plane: bad arguments");
  if (prec == PREC_F16)
    hipLaunchKernelGGL(rms_plane_kernel<PREC_F16>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, eps, w, (u16*)out);
  else
    hipLaunchKernelGGL(rms_plane_kernel<PREC_BF16>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, eps, w, (u16*)out);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// T5 gated-GELU from the interleaved wi GEMM output y [rows][2F] (column 2j = wi_1 j, column 2j + 1 = wi_0 j):
// out [rows][F] = y_2j * gelu_tanh(y_2j+1) — the same expression as the GEMM's geglu == 2 epilogue
__global__ __launch_bounds__(256) void geglu_pairs_kernel(const float2* __restrict__ y, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float2 v = y[i];
  out[i] = v.x * alcm_act(v.y, ACT_GELU_TANH);
}

// the same product written as bf16 hi / lo operand planes (hi = bf16(v), lo = bf16(v - hi); lo plane lo_off
// elements after hi): the A operand of the bf16x3 wo projection, which needs the fp32 range (T5 v1.1 FFN
// activations exceed fp16 on real weights)
__global__ __launch_bounds__(256) void geglu_split_kernel(const float2* __restrict__ y, int64_t n, u16* __restrict__ hi,
                                                          int64_t lo_off) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float2 v = y[i];
  const float p = v.x * alcm_act(v.y, ACT_GELU_TANH);
  const __bf16 h = (__bf16)p;
  hi[i] = __builtin_bit_cast(u16, h);
  hi[i + lo_off] = __builtin_bit_cast(u16, (__bf16)(p - (float)h));
}

int geglu_split_planes(const float* y, int64_t rows, int F, void* plane, int64_t lo_off, hipStream_t s) {
  if (!y || !plane || rows <= 0 || F <= 0 || lo_off < rows * F || (((uintptr_t)y) & 7))
    return set_error(ALCM_E_INVALID, "geglu_split_planes: bad arguments");
  const int64_t n = rows * F;
  hipLaunchKernelGGL(geglu_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float2*>(y), n, (u16*)plane, lo_off);
  ALCM_HIP(hipGetLastError());
  return 0;
}

int geglu_pairs(const float* y, int64_t rows, int F, float* out, hipStream_t s) {
  if (!y || !out || rows <= 0 || F <= 0 || (((uintptr_t)y) & 7)) return set_error(ALCM_E_INVALID, "geglu_pairs: bad arguments");
  const int64_t n = rows * F;
  hipLaunchKernelGGL(geglu_pairs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float2*>(y), n, out);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// In-place row softmax over scores S[z][i][0..n) (row stride ld) with an additive per-head bias
// bias[(h * bld + i) * bld + j], h = z % heads (T5Attention: scores += position_bias, then softmax in fp32);
// zeroes the K padding [n, ld) that the P.V GEMM reads.
__global__ __launch_bounds__(256) void softmax_bias_kernel(float* x, int rows, int n, int64_t ld, int L, int heads,
                                                           const float* __restrict__ bias, int bld) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int z = row / L, i = row - z * L, h = z % heads;
  float* xr = x + (int64_t)row * ld;
  const float* br = bias + ((int64_t)h * bld + i) * bld;
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) {
    const float v = xr[c] + br[c];
    xr[c] = v;
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float sum = 0.f;
  for (int c = lane; c < n; c += 64) sum += expf(xr[c] - m);
  const float inv = 1.0f / wave_sum(sum);
  for (int c = lane; c < n; c += 64) xr[c] = expf(xr[c] - m) * inv;
  for (int c = n + lane; c < ld; c += 64) xr[c] = 0.f;
}

int softmax_rows_bias(float* x, int rows, int n, int64_t ld, int L, int heads, const float* bias, int bld,
                      hipStream_t s) {
  if (!x || !bias || rows <= 0 || n <= 0 || ld < n || L <= 0 || heads <= 0 || bld < n)
    return set_error(ALCM_E_INVALID, "softmax_rows_bias: bad arguments");
  hipLaunchKernelGGL(softmax_bias_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, n, ld, L, heads, bias, bld);
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm
