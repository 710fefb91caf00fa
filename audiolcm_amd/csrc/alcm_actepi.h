// Activation1d (alias_free_torch/act.py:23-27: UpSample1d x2 -> SnakeBeta -> DownSample1d) on values that
// are already on chip, written as MFMA operand planes.  Shared by the standalone act_op_kernel and the
// fused conv epilogues (alcm_opconv.hip, alcm_wconv.hip), which apply it to an LDS-staged fp32 conv tile
// so the conv output never makes an fp32 round trip through HBM before the next conv reads it.
#pragma once
#include "alcm_common.h"

namespace alcm {

// 12-tap FIR pair of Activation1d; `up` holds 2 x the UpSample1d taps (its ratio-2 gain folded in,
// resample.py:30: x = ratio * conv_transpose1d(...)), `dn` the LowPassFilter1d taps
struct Taps12O {
  float up[12], dn[12];
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// x + h - h*cos(2*pi*x*ea_rev): SnakeBeta (activations.py:62-119) with h = inv_beta/2, ea_rev = exp(alpha)/pi,
// since sin^2(z) = 1/2 - cos(2z)/2 and v_cos_f32 takes revolutions.  No explicit argument reduction: v_cos_f32
// reduces the argument itself — measured on gfx950 (scripts/probes/cos_probe.hip) its result equals
// cos(2 pi fract(z)) within 6e-8 and a float64 cos within 1.2e-7 for |z| up to 4096 revolutions, so the
// v_fract_f32 the previous form spent per sample (10 % of Activation1d's VALU cycles) bought nothing
__device__ __forceinline__ f32x2 snake2(f32x2 u, f32x2 ear, f32x2 h) {
  const f32x2 z = u * ear;
  f32x2 c;
  c.x = __builtin_amdgcn_cosf(z.x);
  c.y = __builtin_amdgcn_cosf(z.y);
  return fma2(-h, c, u + h);
}

// two adjacent channels -> operand plane(s): fp16 (F16/F16W2), bf16 (BF16), bf16 hi at hi + bf16 lo at
// hi + lo_off (SPLIT)
template <int PREC>
__device__ __forceinline__ void op_store2(u16* hi, int64_t lo_off, f32x2 v) {
  uint32_t wh, wl = 0;
  if constexpr (PREC == PREC_F16 || PREC == PREC_F16W2) {
    wh = (uint32_t)__builtin_bit_cast(u16, (_Float16)v.x) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)v.y) << 16);
  } else {
    const __bf16 hx = (__bf16)v.x, hy = (__bf16)v.y;
    wh = (uint32_t)__builtin_bit_cast(u16, hx) | ((uint32_t)__builtin_bit_cast(u16, hy) << 16);
    if (PREC == PREC_SPLIT)
      wl = (uint32_t)__builtin_bit_cast(u16, (__bf16)(v.x - (float)hx)) |
           ((uint32_t)__builtin_bit_cast(u16, (__bf16)(v.y - (float)hy)) << 16);
  }
  *reinterpret_cast<uint32_t*>(hi) = wh;
  if (PREC == PREC_SPLIT) *reinterpret_cast<uint32_t*>(hi + lo_off) = wl;
}

// Activation1d of R consecutive outputs j0 .. j0+R-1 of a channel pair whose input rows j0-6 .. j0+R+5 are
// all inside the sequence: win[i] = x[j0 - 6 + i].  Upsampled sample q (m = 2*j0 - 5 + q) feeds outputs r
// with 0 <= q - 2r <= 11 (down tap k = q - 2r, accumulated in ascending k as DownSample1d's conv does).
template <int R, int QB = 4>
__device__ __forceinline__ void act_run_interior(const f32x2 (&win)[R + 12], const Taps12O& f, f32x2 ear, f32x2 h,
                                                 f32x2 (&o)[R]) {
  constexpr int NQ = 2 * R + 10;
#pragma unroll
  for (int r = 0; r < R; ++r) o[r] = f32x2{0.f, 0.f};
  // QB upsampled samples at a time, tap-outer: QB independent up-filter chains back to back (a q-outer order
  // compiles to 6-deep dependent chains with a wait state between links); the order of every sum is unchanged
#pragma unroll
  for (int q0 = 0; q0 < NQ; q0 += QB) {
    f32x2 u[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i) u[i] = f32x2{0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 6; ++kk)
#pragma unroll
      for (int i = 0; i < QB; ++i) {
        const int q = q0 + i;
        if (q < NQ) {
          const int k = 2 * kk + (q & 1);
          u[i] = fma2(f32x2{f.up[k], f.up[k]}, win[(q - k) / 2 + 6], u[i]);
        }
      }
    f32x2 sv[QB];
#pragma unroll
    for (int i = 0; i < QB; ++i)
      if (q0 + i < NQ) sv[i] = snake2(u[i], ear, h);
#pragma unroll
    for (int i = 0; i < QB; ++i) {
      const int q = q0 + i;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = q - 2 * r;
        if (q < NQ && k >= 0 && k < 12) o[r] = fma2(f32x2{f.dn[k], f.dn[k]}, sv[i], o[r]);
      }
    }
  }
}

// Activation1d of R consecutive outputs j0 .. j0+R-1 near a sequence end, from a register window of CLAMPED input
// rows win[i] = x[clamp(j0 - 6 + i, 0, T - 1)] (UpSample1d's replicate padding of x): every upsampled sample m of the
// run is computed once (index math compile-time, as act_run_interior), then DownSample1d's replicate padding of the
// upsampled signal (m outside [0, 2T) takes the value at 0 / 2T - 1, both inside the run when needed) by selects, then
// the down filter.  The same sums in the same order as act_one_clamped: bit-identical to it, with the window loads
// issued together instead of one dependent load per tap (outputs j outside [0, T) are the caller's to mask)
template <int R>
__device__ __forceinline__ void act_run_edge(const f32x2 (&win)[R + 12], int j0, int T, const Taps12O& f, f32x2 ear,
                                             f32x2 h, f32x2 (&o)[R]) {
  constexpr int NQ = 2 * R + 10;
  f32x2 sv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    f32x2 u = f32x2{0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      const int k = 2 * kk + (q & 1);
      u = fma2(f32x2{f.up[k], f.up[k]}, win[(q - k) / 2 + 6], u);
    }
    sv[q] = snake2(u, ear, h);
  }
  const int m0 = 2 * j0 - 5;
  f32x2 slo = sv[0], shi = sv[NQ - 1];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (m0 + q == 0) slo = sv[q];
    if (m0 + q == 2 * T - 1) shi = sv[q];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (m0 + q < 0) sv[q] = slo;
    if (m0 + q >= 2 * T) sv[q] = shi;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    o[r] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 12; ++k) o[r] = fma2(f32x2{f.dn[k], f.dn[k]}, sv[2 * r + k], o[r]);
  }
}

// One output j anywhere in [0, T): replicate padding of the up filter's input (pad 5) and of the down
// filter's input (pad 5 / 6) as index clamps.  ld(i) returns input row i (0 <= i < T) of the pair.
template <typename LD>
__device__ __forceinline__ f32x2 act_one_clamped(int j, int T, const Taps12O& f, f32x2 ear, f32x2 h, LD ld) {
  f32x2 o = f32x2{0.f, 0.f};
  for (int k = 0; k < 12; ++k) {
    int m = 2 * j + k - 5;
    m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
    f32x2 u = f32x2{0.f, 0.f};
    for (int kk = 0; kk < 6; ++kk) {
      const int ku = 2 * kk + ((m & 1) ? 0 : 1);
      int xi = (m + 5 - ku) / 2;
      xi = xi < 0 ? 0 : (xi > T - 1 ? T - 1 : xi);
      u = fma2(f32x2{f.up[ku], f.up[ku]}, ld(xi), u);
    }
    o = fma2(f32x2{f.dn[k], f.dn[k]}, snake2(u, ear, h), o);
  }
  return o;
}

// Fused-epilogue parameters: Activation1d of the conv output into operand planes [B][T][Cp]
struct ActEpiDev {
  u16* plane;
  int64_t plane_lo;  // SPLIT: elements from the hi plane to the lo plane
  int Cp;            // plane channel stride (channels C .. Cp-1 are written as zeros)
  const float* aexp;
  const float* ibeta;
  Taps12O f;
};

constexpr int ACT_EPI_HALO = 8;  // conv tile rows computed beyond each side of the emitted rows

// Activation1d of an LDS-staged fp32 tile, R output rows per work item (the caller picks R so that
// (emitted rows / R) x channel pairs fills its threads: fewer, longer runs also cut the halo recompute,
// (2R + 10) / (2R) upsampled samples per output).  tile[(t - trow0) * ots + col] holds v(b, t, c0 + col) for
// t in [trow0, trow0 + rows) (clamped to [0, T)); emits rows [e_lo, e_hi) for columns [0, ncol) (ncol even)
// of batch b into the planes; channels c >= C are written as zeros (operand padding).  The tile must cover
// [max(e_lo - 6, 0), min(e_hi + 6, T)).
template <int PREC, int R>
__device__ __forceinline__ void act_epilogue_tile(const float* tile, int ots, int trow0, int e_lo, int e_hi, int T,
                                                  int ncol, int c0, int C, int b, const ActEpiDev& A, int tid,
                                                  int nthr) {
  constexpr float INV_PI = 0.318309886183790671538f;
  const int npairs = ncol >> 1;
  const int nreal = max(0, min(npairs, (C - c0) >> 1));  // pairs with channels < C (C even)
  const int nrun = (e_hi - e_lo + R - 1) / R;
  // operand padding (channels >= C): zeros, one (row, pair) per item
  const int npad = npairs - nreal;
  for (int w = tid; w < npad * (e_hi - e_lo); w += nthr) {
    const int row = w / npad, p = nreal + (w - row * npad);
    op_store2<PREC>(A.plane + ((int64_t)b * T + e_lo + row) * A.Cp + c0 + 2 * p, A.plane_lo, f32x2{0.f, 0.f});
  }
  // real pairs: every lane of a wave computes (no padding lanes inside the Activation1d work)
  for (int w = tid; w < nreal * nrun; w += nthr) {
    const int run = w / nreal, p = w - run * nreal;
    const int c = c0 + 2 * p;
    const int j0 = e_lo + run * R;
    const int jn = min(R, e_hi - j0);
    u16* yb = A.plane + ((int64_t)b * T) * A.Cp + c;
    const float* col = tile + 2 * p;
    const f32x2 ear = f32x2{A.aexp[c], A.aexp[c + 1]} * INV_PI;
    const f32x2 h = f32x2{A.ibeta[c], A.ibeta[c + 1]} * 0.5f;
    if (jn == R && j0 >= 6 && j0 + R + 6 <= T) {
      f32x2 win[R + 12];
#pragma unroll
      for (int i = 0; i < R + 12; ++i) win[i] = *reinterpret_cast<const f32x2*>(col + (j0 - 6 + i - trow0) * ots);
      f32x2 o[R];
      act_run_interior<R>(win, A.f, ear, h, o);
#pragma unroll
      for (int r = 0; r < R; ++r) op_store2<PREC>(yb + (int64_t)(j0 + r) * A.Cp, A.plane_lo, o[r]);
    } else {
      for (int r = 0; r < jn; ++r) {
        const f32x2 o = act_one_clamped(j0 + r, T, A.f, ear, h, [&](int i) {
          return *reinterpret_cast<const f32x2*>(col + (i - trow0) * ots);
        });
        op_store2<PREC>(yb + (int64_t)(j0 + r) * A.Cp, A.plane_lo, o);
      }
    }
  }
}

// act_epilogue_tile with the channel pairs NP of the tile known at compile time and no operand-padding work (the
// caller's planes keep their padding channels, which no consumer reads): work item w = (run, pair) by a constant
// division, the caller picks R so that NP * runs ~ its thread count (one pass)
template <int PREC, int R, int NP, bool NOSTORE = false>
__device__ __forceinline__ void act_epilogue_ct(const float* tile, int ots, int trow0, int e_lo, int e_hi, int T,
                                                int c0, int b, const ActEpiDev& A, int tid, int nthr) {
  // NOSTORE (timing ablation only, results wrong): the plane stores replaced by a never-taken dependent store
  f32x2 sink = f32x2{0.f, 0.f};
  constexpr float INV_PI = 0.318309886183790671538f;
  const int nrun = (e_hi - e_lo + R - 1) / R;
  // the batch's plane base is uniform; per-item byte offsets stay 32-bit (a batch's plane is < 4 GB), so the stores
  // need no 64-bit per-lane address arithmetic
  char* const pb = reinterpret_cast<char*>(A.plane + ((int64_t)b * T) * A.Cp);
  for (int w = tid; w < NP * nrun; w += nthr) {
    const int run = w / NP, p = w - run * NP;
    const int c = c0 + 2 * p;
    const int j0 = e_lo + run * R;
    const int jn = min(R, e_hi - j0);
    const uint32_t yo = (uint32_t)(j0 * A.Cp + c) * 2u, ys = (uint32_t)A.Cp * 2u;
    const float* col = tile + 2 * p;
    const f32x2 ear = f32x2{A.aexp[c], A.aexp[c + 1]} * INV_PI;
    const f32x2 h = f32x2{A.ibeta[c], A.ibeta[c + 1]} * 0.5f;
    if (jn == R && j0 >= 6 && j0 + R + 6 <= T) {
      f32x2 win[R + 12];
#pragma unroll
      for (int i = 0; i < R + 12; ++i) win[i] = *reinterpret_cast<const f32x2*>(col + (j0 - 6 + i - trow0) * ots);
      f32x2 o[R];
      act_run_interior<R>(win, A.f, ear, h, o);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (NOSTORE) sink += o[r];
        else op_store2<PREC>(reinterpret_cast<u16*>(pb + (yo + r * ys)), A.plane_lo, o[r]);
      }
    } else {
      for (int r = 0; r < jn; ++r) {
        const f32x2 o = act_one_clamped(j0 + r, T, A.f, ear, h, [&](int i) {
          return *reinterpret_cast<const f32x2*>(col + (i - trow0) * ots);
        });
        if constexpr (NOSTORE) sink += o;
        else op_store2<PREC>(reinterpret_cast<u16*>(pb + (yo + r * ys)), A.plane_lo, o);
      }
    }
  }
  if constexpr (NOSTORE)
    if (sink.x == 123.f && sink.y == 321.f) op_store2<PREC>(reinterpret_cast<u16*>(pb), A.plane_lo, sink);
}

}  // namespace alcm
