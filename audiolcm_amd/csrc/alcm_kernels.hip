// Bandwidth-bound kernels of the AudioLCM hot path (gfx950): norm statistics, softmax,
// the fused anti-aliased SnakeBeta activation (Activation1d), the LCM step and the
// sinusoidal embeddings.  All tensors are fp32; activations are channels-last (b, t, c).
#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

// ---------------------------------------------------------------- block reduction helpers
template <typename T>
__device__ __forceinline__ T wave_sum_t(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T>
__device__ T block_sum(T v, T* sh) {  // blockDim.x == 256
  v = wave_sum_t(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T r = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------- GroupNorm -> per-(b,c) affine
// torch.nn.GroupNorm (Normalize, new_attention.py:85-86 / autoencoder1d.py:168-169, and the
// DiT final GN16): biased variance over (C/G channels x T), y = (x-mean)*rstd*gamma + beta.
// Emitted as scale = rstd*gamma, shift = beta - mean*scale, consumed by the next GEMM's prologue.
__global__ __launch_bounds__(256) void gn_affine_kernel(const float* __restrict__ x, int T, int C, int64_t sb,
                                                        int64_t st, int groups, float eps,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float* scale, float* shift,
                                                        FastDiv cgdiv) {
  __shared__ double sh[4];
  const int g = blockIdx.x, b = blockIdx.y;
  const int cg = C / groups;
  const float* base = x + (int64_t)b * sb + g * cg;
  const int64_t n = (int64_t)cg * T;
  // one pass over the group: fp64 sum and sum of squares (53-bit accumulation of fp32 inputs, so
  // E[x^2] - mean^2 keeps fp32-level accuracy for any mean/std ratio these activations reach)
  double s = 0.0, q = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    uint32_t t, c;
    cgdiv.divmod((uint32_t)e, t, c);
    const double x1 = (double)base[(int64_t)t * st + c];
    s += x1;
    q += x1 * x1;
  }
  const double mean = block_sum(s, sh) / (double)n;
  const double var = fmax(block_sum(q, sh) / (double)n - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float fmean = (float)mean;
  for (int c = threadIdx.x; c < cg; c += 256) {
    const int ch = g * cg + c;
    const float sc = rstd * gamma[ch];
    scale[(int64_t)b * C + ch] = sc;
    shift[(int64_t)b * C + ch] = beta[ch] - fmean * sc;
  }
}

// the same statistics read as float4 pieces (C / groups % 4 == 0, 16-B aligned rows): a quarter of the load
// instructions and index divisions; the fp64 sums see the same values in another order (53-bit accumulation of the
// fp32 inputs: the fp32 mean / rstd it rounds to are unaffected in practice)
__global__ __launch_bounds__(256) void gn_affine4_kernel(const float* __restrict__ x, int T, int C, int64_t sb,
                                                         int64_t st, int groups, float eps,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* scale, float* shift,
                                                         FastDiv cg4div) {
  __shared__ double sh[4];
  const int g = blockIdx.x, b = blockIdx.y;
  const int cg = C / groups;
  const float* base = x + (int64_t)b * sb + g * cg;
  const int64_t n4 = (int64_t)(cg / 4) * T;
  double s = 0.0, q = 0.0;
  for (int64_t e = threadIdx.x; e < n4; e += 256) {
    uint32_t t, c4;
    cg4div.divmod((uint32_t)e, t, c4);
    const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)t * st + 4 * c4);
    const double a0 = v.x, a1 = v.y, a2 = v.z, a3 = v.w;
    s += (a0 + a1) + (a2 + a3);
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const double n = (double)cg * T;
  const double mean = block_sum(s, sh) / n;
  const double var = fmax(block_sum(q, sh) / n - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float fmean = (float)mean;
  for (int c = threadIdx.x; c < cg; c += 256) {
    const int ch = g * cg + c;
    const float sc = rstd * gamma[ch];
    scale[(int64_t)b * C + ch] = sc;
    shift[(int64_t)b * C + ch] = beta[ch] - fmean * sc;
  }
}

int group_norm_affine(const float* x, int B, int T, int C, int64_t sb, int64_t st, int groups, float eps,
                      const float* gamma, const float* beta, float* scale, float* shift, hipStream_t s) {
  if (!x || !gamma || !beta || !scale || !shift || B <= 0 || T <= 0 || groups <= 0 || C % groups)
    return set_error(ALCM_E_INVALID, "group_norm_affine: bad arguments");
  const int cg = C / groups;
  if (cg % 4 == 0 && st % 4 == 0 && sb % 4 == 0 && !(((uintptr_t)x) & 15))
    hipLaunchKernelGGL(gn_affine4_kernel, dim3(groups, B), dim3(256), 0, s, x, T, C, sb, st, groups, eps, gamma, beta,
                       scale, shift, FastDiv((uint32_t)(cg / 4)));
  else
    hipLaunchKernelGGL(gn_affine_kernel, dim3(groups, B), dim3(256), 0, s, x, T, C, sb, st, groups, eps, gamma, beta,
                       scale, shift, FastDiv((uint32_t)cg));
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- LayerNorm (per-row statistics)
// nn.LayerNorm(576), eps 1e-5 (concatDiT.py:114-116, 97-99).  One wave per row, two-pass.
template <bool APPLY>
__global__ __launch_bounds__(256) void ln_kernel(const float* __restrict__ x, int rows, int C, int64_t ld, float eps,
                                                 float* mean_out, float* rstd_out, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, const float* __restrict__ add,
                                                 int64_t ld_add, float* y, int64_t ld_out, int rpb, int64_t out_bs) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ld;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  const float mean = wave_sum(s) / (float)C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = xr[c] - mean;
    v += d * d;
  }
  const float var = wave_sum(v) / (float)C;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (!APPLY) {
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
    return;
  }
  // rpb > 0: rows come in batches of rpb; the add row is the row within its batch, output batch bb starts at row
  // bb * out_bs (the DiT condition tokens: one launch for every clip, written into the [B][CT] token rows)
  int64_t arow = row, orow = row;
  if (rpb > 0) {
    const int bb = row / rpb, t = row - bb * rpb;
    arow = t;
    orow = (int64_t)bb * out_bs + t;
  }
  float* yr = y + orow * ld_out;
  const float* ar = add ? add + arow * ld_add : nullptr;
  for (int c = lane; c < C; c += 64) {
    float o = (xr[c] - mean) * rstd * gamma[c] + beta[c];
    if (ar) o += ar[c];
    yr[c] = o;
  }
}

int row_stats(const float* x, int rows, int C, int64_t ld, float eps, float* mean, float* rstd, hipStream_t s) {
  if (!x || !mean || !rstd || rows <= 0 || C <= 0) return set_error(ALCM_E_INVALID, "row_stats: bad arguments");
  hipLaunchKernelGGL(ln_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld, eps, mean, rstd,
                     nullptr, nullptr, nullptr, (int64_t)0, nullptr, (int64_t)0, 0, (int64_t)0);
  ALCM_HIP(hipGetLastError());
  return 0;
}

int layer_norm(const float* x, int rows, int C, int64_t ld_in, float eps, const float* gamma, const float* beta,
               const float* add, int64_t ld_add, float* y, int64_t ld_out, hipStream_t s, int rpb, int64_t out_bs) {
  if (!x || !y || !gamma || !beta || rows <= 0 || C <= 0 || rpb < 0) return set_error(ALCM_E_INVALID, "layer_norm: bad arguments");
  hipLaunchKernelGGL(ln_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld_in, eps, nullptr, nullptr,
                     gamma, beta, add, ld_add, y, ld_out, rpb, out_bs);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// LayerNorm straight into an MFMA operand plane (fp16 or bf16 [rows][C]) for a conv that reads planes
// (DiT Conv1dFeedForward input, concatDiT.py:120-125 / new_attention.py:48-74)
template <int PREC>
__global__ __launch_bounds__(256) void ln_plane_kernel(const float* __restrict__ x, int rows, int C, int64_t ld,
                                                       float eps, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, u16* __restrict__ y) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ld;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  const float mean = wave_sum(s) / (float)C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = xr[c] - mean;
    v += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)C + eps);
  u16* yr = y + (int64_t)row * C;
  for (int c = lane; c < C; c += 64) {
    const float o = (xr[c] - mean) * rstd * gamma[c] + beta[c];
    yr[c] = PREC == PREC_F16 ? __builtin_bit_cast(u16, (_Float16)o) : __builtin_bit_cast(u16, (__bf16)o);
  }
}

int layer_norm_plane(const float* x, int rows, int C, int64_t ld, float eps, const float* gamma, const float* beta,
                     void* plane, int prec, hipStream_t s) {
  if (!x || !plane || !gamma || !beta || rows <= 0 || C <= 0 || (prec != PREC_F16 && prec != PREC_BF16))
    return set_error(ALCM_E_INVALID, "layer_norm_plane: bad arguments");
  if (prec == PREC_F16)
    hipLaunchKernelGGL(ln_plane_kernel<PREC_F16>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld, eps, gamma,
                       beta, (u16*)plane);
  else
    hipLaunchKernelGGL(ln_plane_kernel<PREC_BF16>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld, eps, gamma,
                       beta, (u16*)plane);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// GroupNorm affine (+ swish) straight into an MFMA operand plane, optionally nearest-upsampled along t:
// plane[b][t'][c] = act(x[b][t'/up][c] * scale[b][c] + shift[b][c]).  The VAE decoder's
// norm -> nonlinearity -> conv k3 (ResnetBlock1D, autoencoder1d.py:212-235) and Upsample1D's
// interpolate(nearest) -> conv (autoencoder1d.py:291-295) then run on the wide-layer conv kernel.
// One workgroup per output row, 4 channels per thread (C % 4 == 0, contiguous (B, T, C) input).
template <int PREC, bool SILU>
__global__ __launch_bounds__(256) void affine_plane_kernel(const float* __restrict__ x, int T, int C, int up,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, u16* __restrict__ y) {
  const int row = blockIdx.x;  // b * (T * up) + t'
  const int To = T * up;
  const int b = row / To, to = row - b * To;
  const float4* xr = reinterpret_cast<const float4*>(x + ((int64_t)b * T + to / up) * C);
  const float4* sc = scale ? reinterpret_cast<const float4*>(scale + (int64_t)b * C) : nullptr;
  const float4* sh = scale ? reinterpret_cast<const float4*>(shift + (int64_t)b * C) : nullptr;
  uint2* yr = reinterpret_cast<uint2*>(y + (int64_t)row * C);
  auto cv = [](float o) -> uint32_t {
    if (SILU) o = o / (1.0f + __expf(-o));
    return PREC == PREC_F16 ? (uint32_t)__builtin_bit_cast(u16, (_Float16)o)
                            : (uint32_t)__builtin_bit_cast(u16, (__bf16)o);
  };
  for (int c = threadIdx.x; c < C / 4; c += 256) {
    float4 v = xr[c];
    if (sc) {
      const float4 a = sc[c], h = sh[c];
      v.x = v.x * a.x + h.x; v.y = v.y * a.y + h.y; v.z = v.z * a.z + h.z; v.w = v.w * a.w + h.w;
    }
    yr[c] = make_uint2(cv(v.x) | (cv(v.y) << 16), cv(v.z) | (cv(v.w) << 16));
  }
}

int affine_plane(const float* x, int B, int T, int C, int up, const float* scale, const float* shift, int silu,
                 void* plane, int prec, hipStream_t s) {
  if (!x || !plane || B <= 0 || T <= 0 || C <= 0 || C % 4 || up < 1 || (scale && !shift) ||
      (prec != PREC_F16 && prec != PREC_BF16) || (((uintptr_t)x) & 15) || (((uintptr_t)plane) & 7) ||
      (scale && ((((uintptr_t)scale) & 15) || (((uintptr_t)shift) & 15))) || (int64_t)B * T * up >= (1ll << 31))
    return set_error(ALCM_E_INVALID, "affine_plane: bad arguments");
  const dim3 grid((unsigned)(B * T * up)), blk(256);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, blk, 0, s, x, T, C, up, scale, shift, (u16*)plane); };
  if (prec == PREC_F16) {
    if (silu) go(affine_plane_kernel<PREC_F16, true>);
    else go(affine_plane_kernel<PREC_F16, false>);
  } else {
    if (silu) go(affine_plane_kernel<PREC_BF16, true>);
    else go(affine_plane_kernel<PREC_BF16, false>);
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- row softmax (in place)
// sim.softmax(dim=-1) (new_attention.py:121) and AttnBlock1D's softmax(dim=2) (autoencoder1d.py:270).
__global__ __launch_bounds__(256) void softmax_kernel(float* x, int rows, int n, int64_t ld) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* xr = x + (int64_t)row * ld;
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, xr[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < n; c += 64) s += expf(xr[c] - m);
  s = wave_sum(s);
  const float inv = 1.0f / s;
  for (int c = lane; c < n; c += 64) xr[c] = expf(xr[c] - m) * inv;
  for (int c = n + lane; c < ld; c += 64) xr[c] = 0.f;  // zero the K-padding the P.V GEMM reads
}

int softmax_rows(float* x, int rows, int n, int64_t ld, hipStream_t s) {
  if (!x || rows <= 0 || n <= 0 || ld < n) return set_error(ALCM_E_INVALID, "softmax_rows: bad arguments");
  hipLaunchKernelGGL(softmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, n, ld);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- fused Activation1d (SnakeBeta)
// UpSample1d (resample.py:25-33) -> SnakeBeta (activations.py:107-119) -> DownSample1d
// (filter.py:86-94) in one pass, no intermediate 2T signal in HBM.
//   up[m]  = 2 * sum_{k = m+1 (mod 2)} f_up[k] * x[clamp((m + 5 - k)/2)],   m in [0, 2T)
//   s[m]   = up[m] + inv_beta[c] * sin(up[m] * alpha_exp[c])^2
//   out[j] = sum_k f_dn[k] * s[clamp(2j + k - 5, 0, 2T-1)]
// Each thread owns one channel and R consecutive outputs; the input window x[j0-6, j0+R+6)
// and the 2R+10 snake samples stay in registers (compile-time indices).  Lanes run along
// channels (coalesced).  The 12+12 filter taps are kernel arguments (SGPR operands).
constexpr int A1D_R = 16;
constexpr int A1D_W = A1D_R + 12;
constexpr int A1D_S = 2 * A1D_R + 10;

struct Taps12 {
  float up[12], dn[12];
};

// sin(x)^2 with a quadrant reduction (Cody-Waite, 3-term pi/2) and the cephes single-precision
// minimax kernels on |r| <= pi/4: ~1 ulp for |x| < 1e4, no libm call, no branches.
__device__ __forceinline__ float sin_sq(float x) {
  const float k = rintf(x * 0.63661977236758134f);
  float r = fmaf(-k, 1.5703125f, x);
  r = fmaf(-k, 4.837512969970703125e-4f, r);
  r = fmaf(-k, 7.54978995489188216e-8f, r);
  const float z = r * r;
  const float sn = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
  const float cs = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                  4.166664568298827e-2f), z, -0.5f), z, 1.0f);
  const float v = (((int)k) & 1) ? cs : sn;
  return v * v;
}

__device__ __forceinline__ float snake(float u, float ea, float ib) { return u + ib * sin_sq(u * ea); }

// interior runs: every index compile-time, all values in registers
__device__ __forceinline__ void act1d_run_interior(const float* __restrict__ xb, float* __restrict__ yb, int64_t st,
                                                   int j0, float ea, float ib, const Taps12& f) {
  float win[A1D_W];
#pragma unroll
  for (int i = 0; i < A1D_W; ++i) win[i] = xb[(int64_t)(j0 - 6 + i) * st];
  float sv[A1D_S];
#pragma unroll
  for (int q = 0; q < A1D_S; ++q) {
    // m = 2*j0 - 5 + q; taps k == q (mod 2) read x[(m + 5 - k)/2] = win[(q - k)/2 + 6]
    float u = 0.f;
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      const int k = 2 * kk + (q & 1);
      u = fmaf(f.up[k], win[(q - k) / 2 + 6], u);
    }
    sv[q] = snake(2.0f * u, ea, ib);
  }
#pragma unroll
  for (int r = 0; r < A1D_R; ++r) {
    float o = 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) o = fmaf(f.dn[k], sv[2 * r + k], o);
    yb[(int64_t)(j0 + r) * st] = o;
  }
}

// edge runs (sequence start/end, or T < R+12): direct evaluation with clamped indices, no arrays
__device__ void act1d_run_edge(const float* __restrict__ xb, float* __restrict__ yb, int T, int64_t st, int j0,
                               float ea, float ib, const Taps12& f) {
  for (int j = j0; j < j0 + A1D_R && j < T; ++j) {
    float o = 0.f;
    for (int k = 0; k < 12; ++k) {
      int m = 2 * j + k - 5;
      m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
      float u = 0.f;
      for (int kk = 0; kk < 6; ++kk) {
        const int ku = 2 * kk + ((m & 1) ? 0 : 1);
        int xi = (m + 5 - ku) / 2;
        xi = xi < 0 ? 0 : (xi > T - 1 ? T - 1 : xi);
        u = fmaf(f.up[ku], xb[(int64_t)xi * st], u);
      }
      o = fmaf(f.dn[k], snake(2.0f * u, ea, ib), o);
    }
    yb[(int64_t)j * st] = o;
  }
}

__global__ __launch_bounds__(256) void act1d_kernel(const float* __restrict__ x, float* __restrict__ y, int T, int C,
                                                    int64_t sb, int64_t st, const float* __restrict__ aexp,
                                                    const float* __restrict__ ibeta, const Taps12 f, int runs,
                                                    uint32_t total, FastDiv cdiv, FastDiv rdiv) {
  for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < total; w += gridDim.x * 256u) {
    uint32_t rb, c, b, run;
    cdiv.divmod(w, rb, c);
    rdiv.divmod(rb, b, run);
    const int j0 = (int)run * A1D_R;
    const float* xb = x + (int64_t)b * sb + c;
    float* yb = y + (int64_t)b * sb + c;
    const float ea = aexp[c], ib = ibeta[c];
    if (j0 >= 6 && j0 + A1D_R + 6 <= T) act1d_run_interior(xb, yb, st, j0, ea, ib, f);
    else act1d_run_edge(xb, yb, T, st, j0, ea, ib, f);
  }
}

int activation1d(const float* x, float* y, int B, int T, int C, int64_t sb, int64_t st, const float* alpha_exp,
                 const float* inv_beta, const float* up_filter, const float* down_filter, hipStream_t s) {
  if (!x || !y || !alpha_exp || !inv_beta || !up_filter || !down_filter || B <= 0 || T <= 0 || C <= 0)
    return set_error(ALCM_E_INVALID, "activation1d: bad arguments");
  if (x == y) return set_error(ALCM_E_INVALID, "activation1d: in-place not supported");
  const int runs = (T + A1D_R - 1) / A1D_R;
  const int64_t total = (int64_t)B * runs * C;
  if (total >= (1ll << 31)) return set_error(ALCM_E_INVALID, "activation1d: problem too large");
  Taps12 f;
  for (int k = 0; k < 12; ++k) {
    f.up[k] = up_filter[k];
    f.dn[k] = down_filter[k];
  }
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 64);
  void* tok = prof_start(s);
  hipLaunchKernelGGL(act1d_kernel, dim3(blocks), dim3(256), 0, s, x, y, T, C, sb, st, alpha_exp, inv_beta, f, runs,
                     (uint32_t)total, FastDiv((uint32_t)C), FastDiv((uint32_t)runs));
  // per output sample: 12 up-FIR + 12 down-FIR MACs on 2 upsampled samples, 2 sin; 4 B in + 4 B out
  prof_stop(tok, s, "alcm::act1d_kernel(float const*, float*, int, int, long, long, float const*, float const*, "
            "alcm::Taps12, int, unsigned int, alcm::FastDiv, alcm::FastDiv)", 2.0 * 36.0 * B * (double)T * C,
            8.0 * B * (double)T * C);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- LCM step
// LCMSampler.step, epsilon prediction (scheduling_lcm.py:465-486), same fp32 op order.
struct StepCoeffs {
  float sqrt_a, sqrt_b, c_out, c_skip, sqrt_a_prev, sqrt_b_prev;
};
__global__ void lcm_step_kernel(const float* __restrict__ x, const float* __restrict__ eps,
                                const float* __restrict__ eps_u, float cfg, const float* __restrict__ noise,
                                StepCoeffs k, float* prev, float* den, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xi = x[i];
    float e = eps[i];
    if (eps_u) {  // classifier-free guidance combine, plms.py:184-186: e_u + s * (e_c - e_u)
      const float eu = eps_u[i];
      e = eu + cfg * (e - eu);
    }
    const float x0 = (xi - k.sqrt_b * e) / k.sqrt_a;
    const float d = k.c_out * x0 + k.c_skip * xi;
    if (den) den[i] = d;
    if (prev) prev[i] = noise ? k.sqrt_a_prev * d + k.sqrt_b_prev * noise[i] : d;
  }
}

int lcm_step(const float* x, const float* eps, const float* eps_u, float cfg, const float* noise, const float* c,
             float* prev, float* den, int64_t n, hipStream_t s) {
  if (!x || !eps || !c || n < 0 || (!prev && !den)) return set_error(ALCM_E_INVALID, "lcm_step: bad arguments");
  if (n == 0) return 0;
  StepCoeffs k{c[0], c[1], c[2], c[3], c[4], c[5]};
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(lcm_step_kernel, dim3(blocks), dim3(256), 0, s, x, eps, eps_u, cfg, noise, k, prev, den, n);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- sinusoidal embeddings
// freqs[] is the reference's own fp32 frequency table (computed on the host exactly as
// scheduling_lcm.py:103-105 / concatDiT.py:60-62 do), so the only device math is t*f and sin/cos.
__global__ void sincos_embed_kernel(const float* __restrict__ v, float vscale, const float* __restrict__ freqs, int B,
                                    int half, int cos_first, float* out) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float a = (v[b] * vscale) * freqs[i];
    // arguments reach ~4e3 rad: reduce modulo 2*pi in fp64 (exact enough for |a| < 1e6), then fp32
    // sin/cos on |r| <= pi, matching the reference CPU libm to ~1 ulp (fp32 OCML on the raw argument
    // differed by up to 3e-5 here)
    const double ad = (double)a;
    const double kq = rint(ad * 0.15915494309189535);
    const float r = (float)(ad - kq * 6.283185307179586);
    const float sn = sinf(r), cs = cosf(r);
    out[(int64_t)b * 2 * half + i] = cos_first ? cs : sn;
    out[(int64_t)b * 2 * half + half + i] = cos_first ? sn : cs;
  }
}
__global__ void i64_to_f32_kernel(const int64_t* t, float* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = (float)t[i];
}

int sincos_embedding(const float* v, float vscale, const float* freqs, int B, int half, int cos_first, float* out,
                     hipStream_t s) {
  if (!v || !freqs || !out || B <= 0 || half <= 0) return set_error(ALCM_E_INVALID, "embedding: bad arguments");
  hipLaunchKernelGGL(sincos_embed_kernel, dim3(B), dim3(128), 0, s, v, vscale, freqs, B, half, cos_first, out);
  ALCM_HIP(hipGetLastError());
  return 0;
}

int i64_to_f32(const int64_t* t, float* o, int n, hipStream_t s) {
  hipLaunchKernelGGL(i64_to_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, s, t, o, n);
  ALCM_HIP(hipGetLastError());
  return 0;
}

__global__ void fill_kernel(float* p, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}
int fill_f32(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return 0;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(fill_kernel, dim3(blocks), dim3(256), 0, s, p, n, v);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// NCT (B, C, T) -> channels-last (B, T, Cp), channels C .. Cp - 1 zero: the reference-layout inputs of the DiT proj_in
// and BigVGAN conv_pre (concatDiT.py proj_in on the NCT latent, models.py:183 on the NCT mel) as the vectorised
// channel-contiguous operand of the implicit-GEMM conv instead of a stride-T gather per element.  32 x 32 tiles
// through LDS (reads coalesced along t, writes along c).
__global__ __launch_bounds__(256) void nct_to_cl_kernel(const float* __restrict__ x, int C, int T, int Cp,
                                                        float* __restrict__ y) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + ty + 8 * j, t = t0 + tx;
    tile[ty + 8 * j][tx] = (c < C && t < T) ? x[((int64_t)b * C + c) * T + t] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = t0 + ty + 8 * j, c = c0 + tx;
    if (t < T && c < Cp) y[((int64_t)b * T + t) * Cp + c] = tile[tx][ty + 8 * j];
  }
}
int nct_to_cl(const float* x, int B, int C, int T, int Cp, float* y, hipStream_t s) {
  if (!x || !y || B <= 0 || C <= 0 || T <= 0 || Cp < C) return set_error(ALCM_E_INVALID, "nct_to_cl: bad arguments");
  hipLaunchKernelGGL(nct_to_cl_kernel, dim3((T + 31) / 32, (Cp + 31) / 32, B), dim3(256), 0, s, x, C, T, Cp, y);
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm

// ---------------------------------------------------------------- C-ABI
extern "C" int alcm_group_norm_affine(const float* x, int B, int T, int C, int64_t sb, int64_t st, int groups,
                                      float eps, const float* gamma, const float* beta, float* scale_out,
                                      float* shift_out, alcm_stream_t stream) {
  return alcm::group_norm_affine(x, B, T, C, sb, st, groups, eps, gamma, beta, scale_out, shift_out,
                                 (hipStream_t)stream);
}
extern "C" int alcm_row_stats(const float* x, int rows, int C, int64_t ld, float eps, float* mean, float* rstd,
                              alcm_stream_t stream) {
  return alcm::row_stats(x, rows, C, ld, eps, mean, rstd, (hipStream_t)stream);
}
extern "C" int alcm_layer_norm(const float* x, int rows, int C, int64_t ld_in, float eps, const float* gamma,
                               const float* beta, const float* add, int64_t ld_add, float* y, int64_t ld_out,
                               alcm_stream_t stream) {
  return alcm::layer_norm(x, rows, C, ld_in, eps, gamma, beta, add, ld_add, y, ld_out, (hipStream_t)stream);
}
extern "C" int alcm_softmax_rows(float* x, int rows, int n, int64_t ld, alcm_stream_t stream) {
  return alcm::softmax_rows(x, rows, n, ld, (hipStream_t)stream);
}
extern "C" int alcm_activation1d(const float* x, float* y, int B, int T, int C, int64_t sb, int64_t st,
                                 const float* alpha_exp, const float* inv_beta, const float* up_filter,
                                 const float* down_filter, alcm_stream_t stream) {
  return alcm::activation1d(x, y, B, T, C, sb, st, alpha_exp, inv_beta, up_filter, down_filter, (hipStream_t)stream);
}
extern "C" int alcm_lcm_step(const float* x, const float* eps, const float* noise, const float* coeffs,
                             float* prev_out, float* denoised_out, int64_t n, alcm_stream_t stream) {
  return alcm::lcm_step(x, eps, nullptr, 1.0f, noise, coeffs, prev_out, denoised_out, n, (hipStream_t)stream);
}
extern "C" int alcm_lcm_step_cfg(const float* x, const float* eps_cond, const float* eps_uncond, float cfg_scale,
                                 const float* noise, const float* coeffs, float* prev_out, float* denoised_out,
                                 int64_t n, alcm_stream_t stream) {
  if (!eps_uncond) return alcm::set_error(ALCM_E_INVALID, "lcm_step_cfg: null eps_uncond");
  return alcm::lcm_step(x, eps_cond, eps_uncond, cfg_scale, noise, coeffs, prev_out, denoised_out, n,
                        (hipStream_t)stream);
}
extern "C" int alcm_sincos_embedding(const float* v, float vscale, const float* freqs, int B, int half,
                                     int cos_first, float* out, alcm_stream_t stream) {
  return alcm::sincos_embedding(v, vscale, freqs, B, half, cos_first, out, (hipStream_t)stream);
}

extern "C" int alcm_layer_norm_plane(const float* x, int rows, int C, int64_t ld, float eps, const float* gamma,
                                     const float* beta, void* plane, int prec, alcm_stream_t stream) {
  return alcm::layer_norm_plane(x, rows, C, ld, eps, gamma, beta, plane, prec, (hipStream_t)stream);
}
