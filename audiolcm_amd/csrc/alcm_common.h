// Shared device/host helpers for the AudioLCM MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ALCM_WAVE 64

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

// Magic-number unsigned division for n, d < 2^31 (row -> (batch, time) decode).
struct FastDiv {
  uint32_t d, m, s;
  __host__ __device__ FastDiv() : d(1), m(1), s(0) {}
  __host__ FastDiv(uint32_t dv) : d(dv ? dv : 1) {
    s = 0;
    while ((1u << s) < d) ++s;
    m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    uint32_t t = __umulhi(n, m);
    return (t + n) >> s;
  }
  __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const {
    q = div(n);
    r = n - q * d;
  }
};

// MFMA operand precision (alcm_gemm_args.prec / alcm_opconv_args.prec):
//   PREC_BF16  one bf16 MFMA (operands rounded to bf16)
//   PREC_SPLIT bf16x3: hi*hi + hi*lo + lo*hi, ~fp32 accuracy
//   PREC_F16   one fp16 MFMA (operands rounded to fp16, 8x finer than bf16)
//   PREC_F16W2 fp16 activation x fp16 hi+lo weight, 2 MFMAs (only the activation is rounded; BigVGAN
//              narrow-stage operand-plane convs)
enum AlcmPrec : int { PREC_BF16 = 0, PREC_SPLIT = 1, PREC_F16 = 2, PREC_F16W2 = 3 };

// 16x16x32 MFMA step on 16-byte operand fragments held as bf16x8 (fp16 bits for PREC_F16).
template <int PREC>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (PREC == PREC_F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Activation codes shared by GEMM prologue/epilogue and elementwise kernels.
enum AlcmAct : int {
  ACT_NONE = 0,
  ACT_SILU = 1,       // x * sigmoid(x)  (nn.SiLU / VAE swish)
  ACT_GELU_ERF = 2,   // F.gelu default
  ACT_GELU_TANH = 3,  // F.gelu(approximate='tanh')
  ACT_TANH = 4,
};

__device__ __forceinline__ float alcm_act(float x, int act) {
  switch (act) {
    case ACT_SILU: return x / (1.0f + expf(-x));
    case ACT_GELU_ERF: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
    case ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
      float u = k0 * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.0f + tanhf(u));
    }
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Host-side round-to-nearest-even fp32 -> bf16 bits (weights only; no NaN handling needed).
static inline u16 host_bf16_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}
static inline float host_bf16_to_f32(u16 b) {
  uint32_t u = ((uint32_t)b) << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
