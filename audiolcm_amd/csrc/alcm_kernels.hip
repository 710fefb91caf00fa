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
  double s = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    uint32_t t, c;
    cgdiv.divmod((uint32_t)e, t, c);
    s += (double)base[(int64_t)t * st + c];
  }
  const double mean = block_sum(s, sh) / (double)n;
  double v = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    uint32_t t, c;
    cgdiv.divmod((uint32_t)e, t, c);
    const double d = (double)base[(int64_t)t * st + c] - mean;
    v += d * d;
  }
  const double var = block_sum(v, sh) / (double)n;
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
  hipLaunchKernelGGL(gn_affine_kernel, dim3(groups, B), dim3(256), 0, s, x, T, C, sb, st, groups, eps, gamma, beta,
                     scale, shift, FastDiv((uint32_t)(C / groups)));
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- LayerNorm (per-row statistics)
// nn.LayerNorm(576), eps 1e-5 (concatDiT.py:114-116, 97-99).  One wave per row, two-pass.
template <bool APPLY>
__global__ __launch_bounds__(256) void ln_kernel(const float* __restrict__ x, int rows, int C, int64_t ld, float eps,
                                                 float* mean_out, float* rstd_out, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, const float* __restrict__ add,
                                                 int64_t ld_add, float* y, int64_t ld_out) {
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
  float* yr = y + (int64_t)row * ld_out;
  const float* ar = add ? add + (int64_t)row * ld_add : nullptr;
  for (int c = lane; c < C; c += 64) {
    float o = (xr[c] - mean) * rstd * gamma[c] + beta[c];
    if (ar) o += ar[c];
    yr[c] = o;
  }
}

int row_stats(const float* x, int rows, int C, int64_t ld, float eps, float* mean, float* rstd, hipStream_t s) {
  if (!x || !mean || !rstd || rows <= 0 || C <= 0) return set_error(ALCM_E_INVALID, "row_stats: bad arguments");
  hipLaunchKernelGGL(ln_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld, eps, mean, rstd,
                     nullptr, nullptr, nullptr, (int64_t)0, nullptr, (int64_t)0);
  ALCM_HIP(hipGetLastError());
  return 0;
}

int layer_norm(const float* x, int rows, int C, int64_t ld_in, float eps, const float* gamma, const float* beta,
               const float* add, int64_t ld_add, float* y, int64_t ld_out, hipStream_t s) {
  if (!x || !y || !gamma || !beta || rows <= 0 || C <= 0) return set_error(ALCM_E_INVALID, "layer_norm: bad arguments");
  hipLaunchKernelGGL(ln_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, s, x, rows, C, ld_in, eps, nullptr, nullptr,
                     gamma, beta, add, ld_add, y, ld_out);
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
// and the 2R+10 snake samples stay in registers.  Lanes run along channels (coalesced).
constexpr int A1D_R = 16;
constexpr int A1D_W = A1D_R + 12;
constexpr int A1D_S = 2 * A1D_R + 10;

template <bool EDGE>
__device__ __forceinline__ void act1d_run(const float* __restrict__ xb, float* __restrict__ yb, int T, int64_t st,
                                          int j0, float ea, float ib, const float* f_up, const float* f_dn) {
  float win[A1D_W];
#pragma unroll
  for (int i = 0; i < A1D_W; ++i) {
    int ti = j0 - 6 + i;
    if (EDGE) ti = ti < 0 ? 0 : (ti > T - 1 ? T - 1 : ti);
    win[i] = xb[(int64_t)ti * st];
  }
  float sv[A1D_S];
#pragma unroll
  for (int q = 0; q < A1D_S; ++q) {
    float u = 0.f;
    if (!EDGE) {
      // m = 2*j0 - 5 + q; taps k with k == q (mod 2) read x[j0 + (q-k)/2 - 6 + 6] = win[(q-k)/2 + 6]
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        const int k = 2 * kk + (q & 1);
        u += f_up[k] * win[(q - k) / 2 + 6];
      }
    } else {
      int m = 2 * j0 - 5 + q;
      m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
      const int par = (m & 1) ? 0 : 1;  // m even -> odd taps
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        const int k = 2 * kk + par;
        u += f_up[k] * win[(m + 5 - k) / 2 - (j0 - 6)];
      }
    }
    u *= 2.0f;
    const float sn = sinf(u * ea);
    sv[q] = u + ib * (sn * sn);
  }
#pragma unroll
  for (int r = 0; r < A1D_R; ++r) {
    const int j = j0 + r;
    if (EDGE && j >= T) break;
    float o = 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      int q = 2 * r + k;
      if (EDGE) {
        int m = 2 * j + k - 5;
        m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
        q = m - (2 * j0 - 5);
      }
      o += f_dn[k] * sv[q];
    }
    yb[(int64_t)j * st] = o;
  }
}

__global__ __launch_bounds__(256) void act1d_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int T,
                                                    int C, int64_t sb, int64_t st, const float* __restrict__ aexp,
                                                    const float* __restrict__ ibeta, const float* __restrict__ fup,
                                                    const float* __restrict__ fdn, int runs, int64_t total) {
  __shared__ float f_up[12], f_dn[12];
  if (threadIdx.x < 12) {
    f_up[threadIdx.x] = fup[threadIdx.x];
    f_dn[threadIdx.x] = fdn[threadIdx.x];
  }
  __syncthreads();
  for (int64_t w = blockIdx.x * (int64_t)256 + threadIdx.x; w < total; w += (int64_t)gridDim.x * 256) {
    const int c = (int)(w % C);
    const int64_t rb = w / C;
    const int run = (int)(rb % runs);
    const int b = (int)(rb / runs);
    const int j0 = run * A1D_R;
    const float* xb = x + (int64_t)b * sb + c;
    float* yb = y + (int64_t)b * sb + c;
    const bool interior = (j0 >= 6) && (j0 + A1D_R + 6 <= T);
    if (interior) act1d_run<false>(xb, yb, T, st, j0, aexp[c], ibeta[c], f_up, f_dn);
    else act1d_run<true>(xb, yb, T, st, j0, aexp[c], ibeta[c], f_up, f_dn);
  }
}

int activation1d(const float* x, float* y, int B, int T, int C, int64_t sb, int64_t st, const float* alpha_exp,
                 const float* inv_beta, const float* up_filter, const float* down_filter, hipStream_t s) {
  if (!x || !y || !alpha_exp || !inv_beta || !up_filter || !down_filter || B <= 0 || T <= 0 || C <= 0)
    return set_error(ALCM_E_INVALID, "activation1d: bad arguments");
  if (x == y) return set_error(ALCM_E_INVALID, "activation1d: in-place not supported");
  const int runs = (T + A1D_R - 1) / A1D_R;
  const int64_t total = (int64_t)B * runs * C;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 32);
  void* tok = prof_start(s);
  hipLaunchKernelGGL(act1d_kernel, dim3(blocks), dim3(256), 0, s, x, y, B, T, C, sb, st, alpha_exp, inv_beta,
                     up_filter, down_filter, runs, total);
  // per output sample: 12 up-FIR + 12 down-FIR MACs on 2 upsampled samples, 2 sin; 4 B in + 4 B out
  prof_stop(tok, s, "alcm::act1d_kernel(float const*, float*, int, int, int, long, long, float const*, float const*, "
            "float const*, float const*, int, long)", 2.0 * 36.0 * B * (double)T * C, 8.0 * B * (double)T * C);
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
    // arguments reach ~4e3 rad: evaluate sin/cos of the fp32 argument in fp64 so the result is the
    // correctly rounded value the reference's CPU libm returns (fp32 OCML differs by up to 3e-5 here)
    const float sn = (float)sin((double)a), cs = (float)cos((double)a);
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
