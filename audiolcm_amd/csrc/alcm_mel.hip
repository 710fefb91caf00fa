// Audio front-end and encoder helpers: the log-mel spectrogram of
// ldm/data/preprocess/NAT_mel.py:42-85 (MelNet.forward) and the stride-2 Downsample1D of the 1-D VAE
// encoder (ldm/models/autoencoder1d.py:296-317).  The STFT itself and the mel projection are MFMA GEMMs
// (alcm_models.cpp); these kernels are the elementwise glue around them.
#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

// y[b][i] = clamp(x[b][reflect(i - p)], -1, 1) for i in [0, L + 2p): torch's reflect padding (no edge repeat)
__global__ void reflect_pad_clamp_kernel(const float* __restrict__ x, int L, int p, float* __restrict__ y,
                                         int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int Lp = L + 2 * p;
  const int64_t b = i / Lp;
  int j = (int)(i - b * Lp) - p;
  if (j < 0) j = -j;
  if (j >= L) j = 2 * (L - 1) - j;
  y[i] = fminf(fmaxf(x[b * L + j], -1.f), 1.f);
}

int reflect_pad_clamp(const float* x, int B, int L, int p, float* y, hipStream_t s) {
  if (!x || !y || B <= 0 || L <= p || p < 0) return set_error(ALCM_E_INVALID, "reflect_pad: bad arguments");
  const int64_t total = (int64_t)B * (L + 2 * p);
  hipLaunchKernelGGL(reflect_pad_clamp_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, L, p, y,
                     total);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// mag[r][k] = sqrt(re^2 + im^2 + 1e-9) from the STFT GEMM rows [re_0..re_{F-1} | im_0..im_{F-1}]
// (NAT_mel.py:79: torch.sqrt(spec.pow(2).sum(-1) + 1e-9))
__global__ void stft_magnitude_kernel(const float* __restrict__ spec, int F, int64_t rows, float* __restrict__ mag) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * F) return;
  const int64_t r = i / F;
  const int k = (int)(i - r * F);
  const float re = spec[r * 2 * F + k], im = spec[r * 2 * F + F + k];
  mag[i] = sqrtf(re * re + im * im + 1e-9f);
}

int stft_magnitude(const float* spec, int F, int64_t rows, float* mag, hipStream_t s) {
  if (!spec || !mag || F <= 0 || rows <= 0) return set_error(ALCM_E_INVALID, "stft_magnitude: bad arguments");
  const int64_t total = rows * F;
  hipLaunchKernelGGL(stft_magnitude_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, spec, F, rows,
                     mag);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// out[b][c][t] = log10(max(x[b][t][c], 1e-5))  (spectral_normalize_torch, NAT_mel.py:26-27,80), NCT output
__global__ void log10_nct_kernel(const float* __restrict__ x, int T, int C, float* __restrict__ out, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t b = i / ((int64_t)T * C);
  const int64_t rem = i - b * T * C;
  const int c = (int)(rem / T), t = (int)(rem - (int64_t)c * T);
  out[i] = log10f(fmaxf(x[(b * T + t) * C + c], 1e-5f));
}

int log10_nct(const float* x, int B, int T, int C, float* out, hipStream_t s) {
  if (!x || !out || B <= 0 || T <= 0 || C <= 0) return set_error(ALCM_E_INVALID, "log10_nct: bad arguments");
  const int64_t total = (int64_t)B * T * C;
  hipLaunchKernelGGL(log10_nct_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, T, C, out, total);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// out[b][t][:] = in[b][2t][:], t < To: the stride-2 subsampling of a stride-1 conv (Downsample1D)
__global__ void rows_stride2_kernel(const float4* __restrict__ in, int T, int To, int C4, float4* __restrict__ out,
                                    int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t row = i / C4;
  const int c = (int)(i - row * C4);
  const int64_t b = row / To;
  const int t = (int)(row - b * To);
  out[i] = in[(b * T + 2 * t) * C4 + c];
}

int rows_stride2(const float* in, int B, int T, int To, int C, float* out, hipStream_t s) {
  if (!in || !out || B <= 0 || T <= 0 || To <= 0 || 2 * (To - 1) >= T || C % 4)
    return set_error(ALCM_E_INVALID, "rows_stride2: bad arguments");
  const int64_t total = (int64_t)B * To * (C / 4);
  hipLaunchKernelGGL(rows_stride2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(in), T, To, C / 4, reinterpret_cast<float4*>(out), total);
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm
