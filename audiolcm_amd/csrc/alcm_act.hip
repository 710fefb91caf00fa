// Activation1d -> MFMA operand planes, LDS-cooperative form (alias_free_torch/act.py:23-27:
// UpSample1d x2 -> SnakeBeta -> DownSample1d; resample.py:10-48, activations.py:62-119).
//
// The Activation1d arithmetic is VALU-bound (two 12-tap FIRs and a cos per upsampled sample).  The
// per-thread form (act_op_kernel) recomputes the 10 upsampled samples that overlap neighbouring runs
// (26 upsampled samples per 8 outputs).  Here a workgroup owns a tile of AC_TT output rows x 32 channels of
// one batch:
//   phase 1: every upsampled + SnakeBeta sample of the tile (2 per output + 10 halo) is computed exactly
//            once, by threads (channel pair, segment of consecutive samples), into LDS;
//   phase 2: threads (channel pair, run of 8 outputs) apply the 12-tap down filter from LDS and write the
//            operand planes.
// Replicate padding (UpSample1d pad 5 on x, DownSample1d pad 5/6 on the upsampled signal) is applied by
// computing the sample at the clamped index, so phase 2 needs no edge cases.  ~19 VALU issue slots per
// element instead of ~30.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

// Tiles: NP channel pairs x (2048 / NP) output rows.  NP = 32 (64 channels: whole 128-B lines of the fp16
// output rows and 256-B input row segments) where Cp allows, else NP = 16.
constexpr int AC_SEG = 18;                 // upsampled samples per phase-1 thread (even: static FIR indexing)

// 8-byte load at a 32-bit byte offset from a workgroup-uniform base: the saddr + voffset address form, no 64-bit
// per-lane address arithmetic
__device__ __forceinline__ f32x2 ld_f32x2(const float* base, uint32_t byte_off) {
  return *reinterpret_cast<const f32x2*>(reinterpret_cast<const char*>(base) + byte_off);
}

// NSET parameter sets over the same input (the three resblocks' first Activation1d of a BigVGAN stage: the x window
// is loaded once, then per set phase 1 -> barrier -> phase 2 into that set's planes)
struct ActSets {
  u16* y[3];
  const float* aexp[3];
  const float* ibeta[3];
};

template <int PREC, int AC_NP, int NSET>
__global__ __launch_bounds__(256) void act_coop_kernel(const float* __restrict__ x, const ActSets S, int64_t y_lo,
                                                       int T, int C, int Cp, const Taps12O f, int tiles_t,
                                                       int tiles_c) {
  constexpr float INV_PI = 0.318309886183790671538f;
  constexpr int AC_TT = 2048 / AC_NP;             // output rows per tile (8 per phase-2 thread)
  constexpr int NSEG = 256 / AC_NP;                // phase-1 segments
  constexpr int AC_NU = NSEG * AC_SEG;             // upsampled samples staged per channel (>= 2 * AC_TT + 11)
  constexpr int AC_RS = AC_NP + 1;                 // LDS sample-row stride (f32x2): conflict-free phase-2 reads
  static_assert(AC_NU >= 2 * AC_TT + 11 && AC_TT == 8 * NSEG, "act_coop tile");
  __shared__ __attribute__((aligned(16))) f32x2 sv[AC_NU * AC_RS];  // [m - m0][pair]
  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int ct = bid % tiles_c;
  bid /= tiles_c;
  const int tt = bid % tiles_t;
  const int b = bid / tiles_t;
  const int t0 = tt * AC_TT, c0 = ct * 2 * AC_NP;
  const int p = tid % AC_NP;
  const int c = c0 + 2 * p;
  const bool live = c < C;  // pairs at or beyond C: operand padding (zeros)
  // per-batch bases are workgroup-uniform (SGPRs); per-lane offsets stay 32-bit (a batch is < 2^31 elements), so
  // each load / store is a saddr + 32-bit voffset access instead of a 64-bit multiply-add per address
  const float* xb = x + ((int64_t)b * T) * C;
  const int xc = live ? c : 0;
  const int m0 = 2 * t0 - 6;  // sample index 0 of the tile (even); output j reads m = 2j - 5 .. 2j + 6
  const int seg = tid / AC_NP;
  const int mb = m0 + seg * AC_SEG;
  const int xlo = mb / 2 - 3;  // sample mb + q reads x rows xlo + (q + 5 - ku) / 2 + 3 - 3
  const bool interior = mb >= 0 && mb + AC_SEG - 1 <= 2 * T - 1 && xlo >= 0 && xlo + 14 <= T - 1;
  f32x2 win[15];
  if (live && interior) {
    const uint32_t o0 = (uint32_t)(xlo * C + xc);
#pragma unroll
    for (int i = 0; i < 15; ++i) win[i] = ld_f32x2(xb, (o0 + (uint32_t)(i * C)) * 4u);
  }
  const int run = tid / AC_NP;
  const int j0 = t0 + run * 8;
  const int jn = min(8, T - j0);

  // tap-outer order: the 18 accumulation chains are independent instructions back to back (a q-outer order compiles
  // to 6-deep dependent chains with a wait state between links)
  auto up_fir = [&](f32x2 (&u)[AC_SEG]) {
#pragma unroll
    for (int q = 0; q < AC_SEG; ++q) u[q] = f32x2{0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 6; ++kk)
#pragma unroll
      for (int q = 0; q < AC_SEG; ++q) {
        const int ku = 2 * kk + ((q & 1) ? 0 : 1);
        u[q] = fma2(f32x2{f.up[ku], f.up[ku]}, win[(q + 5 - ku) / 2 + 3], u[q]);
      }
  };
  // NSET = 3 (the three resblocks' first Activation1d of a tail stage): UpSample1d does not depend on the SnakeBeta
  // parameters, so the samples are computed once for the three sets (x3 launches 1.49 -> 1.37 ms/step, bit-identical,
  // profiles/r6j); with one set the FIR stays inside the set's phase 1, where it fills the SnakeBeta / LDS latency
  // (hoisted there: +5.6 %, profiles/r6f)
  f32x2 u3[NSET > 1 ? AC_SEG : 1];
  if constexpr (NSET > 1)
    if (live && interior) up_fir(u3);

#pragma unroll
  for (int st = 0; st < NSET; ++st) {
    const f32x2 ear = live ? f32x2{S.aexp[st][c], S.aexp[st][c + 1]} * INV_PI : f32x2{0.f, 0.f};
    const f32x2 h = live ? f32x2{S.ibeta[st][c], S.ibeta[st][c + 1]} * 0.5f : f32x2{0.f, 0.f};
    // ---- phase 1: upsampled samples mb .. mb + 17 of segment seg (mb even, so the polyphase tap parity and the
    //      x-window offsets are compile-time); replicate padding = the sample at the clamped index
    if (live) {
      if (interior) {
        if constexpr (NSET > 1) {
#pragma unroll
          for (int q = 0; q < AC_SEG; ++q) sv[(seg * AC_SEG + q) * AC_RS + p] = snake2(u3[q], ear, h);
        } else {
          f32x2 u[AC_SEG];
          up_fir(u);
#pragma unroll
          for (int q = 0; q < AC_SEG; ++q) sv[(seg * AC_SEG + q) * AC_RS + p] = snake2(u[q], ear, h);
        }
      } else {
        for (int q = 0; q < AC_SEG; ++q) {
          int m = mb + q;
          m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
          f32x2 u = f32x2{0.f, 0.f};
          for (int kk = 0; kk < 6; ++kk) {
            const int ku = 2 * kk + ((m & 1) ? 0 : 1);
            int xi = (m + 5 - ku) / 2;
            xi = xi < 0 ? 0 : (xi > T - 1 ? T - 1 : xi);
            u = fma2(f32x2{f.up[ku], f.up[ku]}, ld_f32x2(xb, (uint32_t)(xi * C + xc) * 4u), u);
          }
          sv[(seg * AC_SEG + q) * AC_RS + p] = snake2(u, ear, h);
        }
      }
    }
    __syncthreads();
    // ---- phase 2: outputs j0 .. j0 + 7 of pair p: o[j] = sum_k dn[k] * sv[2j + k - 5 - m0]
    if (j0 < T) {
      u16* yb = S.y[st] + ((int64_t)b * T) * Cp;
      if (!live) {
        for (int r = 0; r < jn; ++r) op_store2<PREC>(yb + (uint32_t)((j0 + r) * Cp + c), y_lo, f32x2{0.f, 0.f});
      } else {
        const f32x2* sp = sv + (2 * (j0 - t0) + 1) * AC_RS + p;
        f32x2 sr[26];
#pragma unroll
        for (int i = 0; i < 26; ++i) sr[i] = sp[i * AC_RS];
        // tap-outer: 8 independent chains (one per output, each summed in ascending tap order like the fused
        // epilogue's), then the stores (no per-row branch between the chains)
        f32x2 o[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) o[r] = f32x2{0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 12; ++k)
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] = fma2(f32x2{f.dn[k], f.dn[k]}, sr[2 * r + k], o[r]);
        const uint32_t yo = (uint32_t)(j0 * Cp + c) * 2u;  // byte offset from the uniform batch base
        auto yp = [&](int r) {
          return reinterpret_cast<u16*>(reinterpret_cast<char*>(yb) + (yo + (uint32_t)(r * Cp) * 2u));
        };
        if (jn == 8) {
#pragma unroll
          for (int r = 0; r < 8; ++r) op_store2<PREC>(yp(r), y_lo, o[r]);
        } else {
          for (int r = 0; r < jn; ++r) op_store2<PREC>(yp(r), y_lo, o[r]);
        }
      }
    }
    if (st + 1 < NSET) __syncthreads();  // phase-2 reads of sv retired before the next set's phase 1
  }
}

// nset parameter sets (1 or 3) of one input: y[i], alpha_exp[i], inv_beta[i]
int act_coop(const float* x, void* const* y, int nset, int B, int T, int C, int Cp, const float* const* alpha_exp,
             const float* const* inv_beta, const Taps12O& f, int prec, hipStream_t s) {
  if (nset != 1 && nset != 3) return set_error(ALCM_E_INVALID, "activation1d: 1 or 3 parameter sets");
  // 64-channel tiles (whole 128-B output lines) measured faster at C = 768 (-15 %) and for the two-plane split
  // output (-10 %), slower at C = 384 (+10..15 %), even at C = 192 fp16 (scripts/microbench.py actnp)
  const bool wide = Cp % 64 == 0 && (C >= 768 || prec == PREC_SPLIT);
  const int np = wide ? 32 : 16, tt = 2048 / np;
  const int tiles_t = (T + tt - 1) / tt, tiles_c = Cp / (2 * np);
  const int64_t nwg = (int64_t)B * tiles_t * tiles_c;
  if (nwg >= (1ll << 31)) return set_error(ALCM_E_INVALID, "activation1d_op: problem too large");
  const int64_t y_lo = (int64_t)B * T * Cp;
  ActSets S{};
  for (int i = 0; i < nset; ++i) {
    S.y[i] = (u16*)y[i];
    S.aexp[i] = alpha_exp[i];
    S.ibeta[i] = inv_beta[i];
  }
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), 0, s, x, S, y_lo, T, C, Cp, f, tiles_t, tiles_c);
  };
  auto pick = [&](auto npc) {
    constexpr int NP = decltype(npc)::value;
    if (nset == 3) {
      if (prec == PREC_SPLIT) launch(act_coop_kernel<PREC_SPLIT, NP, 3>);
      else if (prec == PREC_BF16) launch(act_coop_kernel<PREC_BF16, NP, 3>);
      else launch(act_coop_kernel<PREC_F16, NP, 3>);
    } else {
      if (prec == PREC_SPLIT) launch(act_coop_kernel<PREC_SPLIT, NP, 1>);
      else if (prec == PREC_BF16) launch(act_coop_kernel<PREC_BF16, NP, 1>);
      else launch(act_coop_kernel<PREC_F16, NP, 1>);
    }
  };
  if (wide) pick(std::integral_constant<int, 32>{});
  else pick(std::integral_constant<int, 16>{});
  return 0;
}

// ------------------------------------------------------------------------------------------------------------------
// Activation1d on MFMA (alias_free_torch/act.py:23-27), fp16 operand planes out, for the wide BigVGAN stages (C = 768 /
// 384 / 192 under the mixed policy).  Both 12-tap FIRs are banded Toeplitz products per 16-channel group:
//   up   U[16 samples][16 ch]   = A_up[16][K = 13 x rows x (hi, lo tap)] . X[K][16 ch]   one 16x16x32 MFMA per block
//   down Y^T[16 ch][16 outputs] = S^T[16 ch][K = 42 samples x (hi, lo tap)] . D[K][16]   three MFMAs per block
// with every operand pair (v, v) against the taps' fp16 (hi, lo) split, so the TAPS are exact to 22 bits and only the
// FIR inputs (x and the SnakeBeta samples) are rounded to fp16 — emulated on the recipe weights at +2e-5 waveform rel-L2
// for stages 0-2 (scripts/precision_emulate.py fir: mixed policy 6.02e-4 -> 6.25e-4; fp16 taps would cost 4e-3, and
// fp16 inputs on the narrow stages 1.15e-3, so those keep the fp32 VALU FIRs).  The tap fragments depend only on the
// lane (the sample / output offsets of a block are fixed), so they are built once per wave; SnakeBeta stays on the VALU
// in fp32 between the two products.  One wave owns 16 channels x 64 outputs: x rows t0 - 5 .. t0 + 74 (clamped:
// UpSample1d's replicate padding) as (v, v) fp16 pairs in LDS [ch][row], 9 up blocks -> 144 samples m = 2 t0 - 5 + i
// as pairs in LDS [ch][i] (samples outside [0, 2T): DownSample1d's replicate padding, patched in LDS), 4 down blocks
// -> 4 channels x one output per lane, 8-B plane stores.  No cross-wave sharing: no workgroup barrier.
constexpr int AM_XS = 84;            // x row stride in pairs: = 20 mod 64 (conflict-free 4-B transposing writes)

__device__ __forceinline__ float am_sel12(const float (&t)[12], int i) {
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 12; ++k) v = (i == k) ? t[k] : v;
  return v;
}
__device__ __forceinline__ uint32_t am_pair(float v) {  // (v, v) as two fp16
  const uint32_t h = __builtin_bit_cast(u16, (_Float16)v);
  return h | (h << 16);
}

constexpr int AM_STRIP = 8;          // wave tiles per workgroup strip (the tap fragments are built once per strip)

// TT outputs per wave tile: 64 (two 59 KB workgroups per CU).  A 48-output tile (7 up / 3 down blocks, 51 KB: three
// workgroups per CU) measured the same (8.92 vs 8.94 ms/step over the 270 launches, profiles/r4z): occupancy is not
// what bounds this kernel
template <int TT>
struct AmGeo {
  static constexpr int XR = TT + 16;                   // staged x rows
  static constexpr int UPB = (2 * TT + 10 + 15) / 16;  // up blocks
  static constexpr int OCC = 4;                        // workgroups per CU (31 KB of LDS, <= 128 VGPRs)
  static_assert(XR <= AM_XS && 8 * (UPB - 1) + 15 < XR && TT % 16 == 0 && 2 * (TT / 16 - 1) + 2 < UPB,
                "act_mfma tile");
};

// IN16: x is an fp16 plane [B][T][C] (a conv1 that wrote its output in the format this kernel rounds its input to:
// the same (v, v) pairs, half the bytes read)
template <int TT, bool DEFER, bool IN16 = false>
__global__ __launch_bounds__(256, (AmGeo<TT>::OCC)) void act_mfma_kernel(const void* __restrict__ xin,
                                                                          u16* __restrict__ y, int T, int C, int Cp,
                                                                          const float* __restrict__ aexp,
                                                                          const float* __restrict__ ibeta,
                                                                          const Taps12O f, int strips_t, int tiles_c) {
  constexpr float INV_PI = 0.318309886183790671538f;
  constexpr int AM_TT = TT, AM_XR = AmGeo<TT>::XR, AM_UPB = AmGeo<TT>::UPB;
  // per wave [16 ch][XS rows] of (v, v) pairs; waves 4 pairs apart (= 4 mod 64 banks: the cooperative writes below
  // are conflict-free)
  constexpr int XWS = 16 * AM_XS + 4;
  __shared__ __attribute__((aligned(16))) uint32_t xs[4 * XWS];
  // the workgroup's output tile [TT rows][64 channels] (row stride 72 halves), written out as whole 128-B row segments
  // (each wave's own 32-B pieces of 16 rows left partial lines for the L2 to merge: 1.7x the plane bytes in PMC)
  constexpr int OS = 72;
  __shared__ __attribute__((aligned(16))) u16 ob[AM_TT * OS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, l16 = lane & 15;
  int bid = blockIdx.x;
  const int ct = bid % tiles_c;
  bid /= tiles_c;
  const int st = bid % strips_t;
  const int b = bid / strips_t;
  const int c0 = ct * 64 + wave * 16;
  const int tile0 = st * AM_STRIP, ntile = min(AM_STRIP, (T + AM_TT - 1) / AM_TT - tile0);
  uint32_t* const xw = xs + wave * XWS;

  // tap fragments, once per strip: up A[q = l16][k = 8 q4 + e] = tap_(e&1)[ku], ku = q - 2 r' + 10, r' = 4 q4 + e / 2
  // (x row of the block); down B[k][n = l16] = tap_(e&1)[i' - 2 n], i' = 16 p + 4 q4 + e / 2 (sample of the block)
  f16x8 aup, bdn[3];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int rr = 4 * q4 + e / 2;
    const int ku = l16 - 2 * rr + 10;
    const float tv = (ku >= 0 && ku < 12) ? am_sel12(f.up, ku) : 0.f;
    const _Float16 hi = (_Float16)tv;
    aup[e] = (e & 1) ? (_Float16)(tv - (float)hi) : hi;
  }
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * p + 4 * q4 + e / 2 - 2 * l16;
      const float tv = (k >= 0 && k < 12) ? am_sel12(f.dn, k) : 0.f;
      const _Float16 hi = (_Float16)tv;
      bdn[p][e] = (e & 1) ? (_Float16)(tv - (float)hi) : hi;
    }
  const int cl = c0 + l16;  // this lane's channel in the up products
  const float ear = aexp[cl] * INV_PI, hh = ibeta[cl] * 0.5f;

  // x rows t0 - 5 + r (clamped) of the workgroup's 64 channels, loaded cooperatively as whole 256-B row segments: wave
  // w's instruction it covers rows 16 it + 4 w .. + 3, lane = (row, 16-B piece); each piece belongs to the wave
  // owning its 16 channels.  The next tile's rows are loaded into registers while this tile computes
  // (each wave loading its own 16 channels as 64-B row pieces measured 8.32 vs 8.18 ms/step, profiles/r4ae)
  // (IN16: the same lanes and rows, 8-B pieces of four fp16 channels: 128-B row segments)
  typedef typename std::conditional<IN16, uint2, float4>::type XPiece;
  const char* const xb = reinterpret_cast<const char*>(xin) +
                         ((int64_t)b * T * C + ct * 64 + (lane & 15) * 4) * (IN16 ? 2 : 4);
  XPiece xv[AM_XR / 16];
  auto xrow = [&](int it) { return it * 16 + wave * 4 + (lane >> 4); };
  auto load_x = [&](int t0) {
#pragma unroll
    for (int it = 0; it < AM_XR / 16; ++it) {
      const int t = min(max(t0 - 5 + xrow(it), 0), T - 1);
      xv[it] = *reinterpret_cast<const XPiece*>(xb + (int64_t)t * C * (IN16 ? 2 : 4));
    }
  };
  load_x(tile0 * AM_TT);
  u16* const yb = y + (int64_t)b * T * Cp + ct * 64;
  // the output tile staged in ob goes out one iteration late, issued BEFORE the next prefetch: the compiler waits for a
  // tile's x rows with vmcnt(0) at the loop head, and stores issued after the prefetch (at the end of the tile) made
  // that wait drain their round trip every tile; issued before it, they are a whole tile old by then
  auto store_tile = [&](int t0) {
#pragma unroll
    for (int k = 0; k < AM_TT * 8 / 256; ++k) {
      const int e = tid + 256 * k, r = e >> 3, sg = e & 7;
      if (t0 + r < T)
        *reinterpret_cast<uint4*>(yb + (int64_t)(t0 + r) * Cp + sg * 8) =
            *reinterpret_cast<const uint4*>(ob + r * OS + sg * 8);
    }
  };
  for (int tl = 0; tl < ntile; ++tl) {
    const int t0 = (tile0 + tl) * AM_TT;
    // (v, v) fp16 pairs at xw'[c * XS + r] of the owning wave w'
    {
      uint32_t* const xo = xs + ((lane & 15) >> 2) * XWS;
      const int c = (lane & 3) * 4;
#pragma unroll
      for (int it = 0; it < AM_XR / 16; ++it) {
        const int r = xrow(it);
        if constexpr (IN16) {
          const uint2 h = xv[it];
          xo[(c + 0) * AM_XS + r] = (h.x & 0xffffu) | (h.x << 16);
          xo[(c + 1) * AM_XS + r] = (h.x >> 16) | (h.x & 0xffff0000u);
          xo[(c + 2) * AM_XS + r] = (h.y & 0xffffu) | (h.y << 16);
          xo[(c + 3) * AM_XS + r] = (h.y >> 16) | (h.y & 0xffff0000u);
        } else {
          xo[(c + 0) * AM_XS + r] = am_pair(xv[it].x);
          xo[(c + 1) * AM_XS + r] = am_pair(xv[it].y);
          xo[(c + 2) * AM_XS + r] = am_pair(xv[it].z);
          xo[(c + 3) * AM_XS + r] = am_pair(xv[it].w);
        }
      }
    }
    if (DEFER && tl > 0) store_tile(t0 - AM_TT);  // (ob is rewritten only after the barrier below)
    if (tl + 1 < ntile) load_x(t0 + AM_TT);
    // every wave's x pairs staged: LDS-only wait (a __syncthreads fence would also wait for the prefetch)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // up blocks: samples i = 16 bk + 4 q4 + r of channel l16 -> SnakeBeta (fp32) -> (s, s) pairs, kept in registers: the
    // MFMA output fragment of up block bk (lane (q4, l16): channel l16, samples 16 bk + 4 q4 .. + 3) is exactly the A
    // fragment of the down block reading samples 16 bk .. + 15 (row = channel l16, k-group q4), so the samples never
    // go through LDS (round 4 staged them: 84 KB of the tile's 156 KB of LDS traffic)
    uint4 sf[AM_UPB];
#pragma unroll
    for (int bk = 0; bk < AM_UPB; ++bk) {
      const f16x8 bx = *reinterpret_cast<const f16x8*>(xw + l16 * AM_XS + 8 * bk + 4 * q4);
      const f32x4 u = __builtin_amdgcn_mfma_f32_16x16x32_f16(aup, bx, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      uint32_t* op = reinterpret_cast<uint32_t*>(&sf[bk]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sv = fmaf(-hh, __builtin_amdgcn_cosf(u[r] * ear), u[r] + hh);
        op[r] = am_pair(sv);
      }
    }
    // DownSample1d replicate padding: samples m = 2 t0 - 5 + i outside [0, 2T) take s(0) / s(2T - 1) (wave-uniform:
    // only the tiles at a clip's ends): the pair at local index i_lo / i_hi of this lane's channel, from the lane
    // holding it (q4 = (i >> 2) & 3, same l16)
    const int i_lo = 5 - 2 * t0, i_hi = 2 * T + 4 - 2 * t0;  // local indices of m = 0 and m = 2T - 1
    if (i_lo > 0 || i_hi < AM_UPB * 16 - 1) {
      auto pick = [&](int i) -> uint32_t {  // this lane's pair r = i & 3 of block i >> 4 (selects: register arrays)
        uint32_t v = 0u;
#pragma unroll
        for (int bk = 0; bk < AM_UPB; ++bk) {
          const uint32_t* sp = reinterpret_cast<const uint32_t*>(&sf[bk]);
#pragma unroll
          for (int r = 0; r < 4; ++r) v = (bk == (i >> 4) && r == (i & 3)) ? sp[r] : v;
        }
        return v;
      };
      const int il = max(i_lo, 0), ih = min(max(i_hi, 0), AM_UPB * 16 - 1);
      const uint32_t vlo = (uint32_t)__shfl((int)pick(il), ((il >> 2) & 3) * 16 + l16);
      const uint32_t vhi = (uint32_t)__shfl((int)pick(ih), ((ih >> 2) & 3) * 16 + l16);
#pragma unroll
      for (int bk = 0; bk < AM_UPB; ++bk) {
        uint32_t* sp = reinterpret_cast<uint32_t*>(&sf[bk]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * bk + 4 * q4 + r;
          if (i_lo > 0 && i < i_lo) sp[r] = vlo;
          if (i_hi >= 0 && i_hi < AM_UPB * 16 - 1 && i > i_hi) sp[r] = vhi;
        }
      }
    }

    // down blocks: outputs j = t0 + 16 d + l16, channels c0 + 4 q4 .. + 3 -> 8-B fp16 plane stores
#pragma unroll
    for (int d = 0; d < AM_TT / 16; ++d) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 3; ++p)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, sf[2 * d + p]), bdn[p], acc, 0, 0, 0);
      uint2 w;
      w.x = (uint32_t)__builtin_bit_cast(u16, (_Float16)acc[0]) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)acc[1]) << 16);
      w.y = (uint32_t)__builtin_bit_cast(u16, (_Float16)acc[2]) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)acc[3]) << 16);
      *reinterpret_cast<uint2*>(ob + (16 * d + l16) * OS + wave * 16 + 4 * q4) = w;
    }
    // every wave's 16 channels of the tile staged, and every wave past its up reads of xs (the next tile's x pairs
    // may be written)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (!DEFER) {  // (ALCM_ACT_DEFER=0: the stores at the end of their own tile)
      store_tile(t0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  if (DEFER && ntile > 0) store_tile((tile0 + ntile - 1) * AM_TT);
}

// act_mfma_kernel for the three resblocks' first Activation1d of a wide stage (one input, three SnakeBeta parameter
// sets, the same FIR taps): x staged and the up products computed ONCE per tile and kept as fp32 fragments (UPB x 4
// registers), then per set SnakeBeta -> (s, s) pairs -> down products -> that set's plane, the staged output tile
// stored right away (no one-tile deferral: three tiles would be in flight).  The same operations per set as
// act_mfma_kernel<TT, .., false>: bit-identical to three calls.
template <int TT>
__global__ __launch_bounds__(256, 2) void act_mfma3_kernel(const float* __restrict__ xin, const ActSets S, int T, int C,
                                                           int Cp, const Taps12O f, int strips_t, int tiles_c) {
  constexpr float INV_PI = 0.318309886183790671538f;
  constexpr int AM_TT = TT, AM_XR = AmGeo<TT>::XR, AM_UPB = AmGeo<TT>::UPB;
  constexpr int XWS = 16 * AM_XS + 4;
  __shared__ __attribute__((aligned(16))) uint32_t xs[4 * XWS];
  constexpr int OS = 72;
  __shared__ __attribute__((aligned(16))) u16 ob[AM_TT * OS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, l16 = lane & 15;
  int bid = blockIdx.x;
  const int ct = bid % tiles_c;
  bid /= tiles_c;
  const int st = bid % strips_t;
  const int b = bid / strips_t;
  const int c0 = ct * 64 + wave * 16;
  const int tile0 = st * AM_STRIP, ntile = min(AM_STRIP, (T + AM_TT - 1) / AM_TT - tile0);
  uint32_t* const xw = xs + wave * XWS;
  f16x8 aup, bdn[3];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int rr = 4 * q4 + e / 2;
    const int ku = l16 - 2 * rr + 10;
    const float tv = (ku >= 0 && ku < 12) ? am_sel12(f.up, ku) : 0.f;
    const _Float16 hi = (_Float16)tv;
    aup[e] = (e & 1) ? (_Float16)(tv - (float)hi) : hi;
  }
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * p + 4 * q4 + e / 2 - 2 * l16;
      const float tv = (k >= 0 && k < 12) ? am_sel12(f.dn, k) : 0.f;
      const _Float16 hi = (_Float16)tv;
      bdn[p][e] = (e & 1) ? (_Float16)(tv - (float)hi) : hi;
    }
  const int cl = c0 + l16;
  float ear[3], hh[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    ear[k] = S.aexp[k][cl] * INV_PI;
    hh[k] = S.ibeta[k][cl] * 0.5f;
  }
  const char* const xb = reinterpret_cast<const char*>(xin) + ((int64_t)b * T * C + ct * 64 + (lane & 15) * 4) * 4;
  float4 xv[AM_XR / 16];
  auto xrow = [&](int it) { return it * 16 + wave * 4 + (lane >> 4); };
  auto load_x = [&](int t0) {
#pragma unroll
    for (int it = 0; it < AM_XR / 16; ++it) {
      const int t = min(max(t0 - 5 + xrow(it), 0), T - 1);
      xv[it] = *reinterpret_cast<const float4*>(xb + (int64_t)t * C * 4);
    }
  };
  load_x(tile0 * AM_TT);
  for (int tl = 0; tl < ntile; ++tl) {
    const int t0 = (tile0 + tl) * AM_TT;
    {
      uint32_t* const xo = xs + ((lane & 15) >> 2) * XWS;
      const int c = (lane & 3) * 4;
#pragma unroll
      for (int it = 0; it < AM_XR / 16; ++it) {
        const int r = xrow(it);
        xo[(c + 0) * AM_XS + r] = am_pair(xv[it].x);
        xo[(c + 1) * AM_XS + r] = am_pair(xv[it].y);
        xo[(c + 2) * AM_XS + r] = am_pair(xv[it].z);
        xo[(c + 3) * AM_XS + r] = am_pair(xv[it].w);
      }
    }
    if (tl + 1 < ntile) load_x(t0 + AM_TT);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // the up products of the tile, once for the three sets
    f32x4 ub[AM_UPB];
#pragma unroll
    for (int bk = 0; bk < AM_UPB; ++bk) {
      const f16x8 bx = *reinterpret_cast<const f16x8*>(xw + l16 * AM_XS + 8 * bk + 4 * q4);
      ub[bk] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aup, bx, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    const int i_lo = 5 - 2 * t0, i_hi = 2 * T + 4 - 2 * t0;
#pragma unroll
    for (int set = 0; set < 3; ++set) {
      uint4 sf[AM_UPB];
#pragma unroll
      for (int bk = 0; bk < AM_UPB; ++bk) {
        uint32_t* op = reinterpret_cast<uint32_t*>(&sf[bk]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sv = fmaf(-hh[set], __builtin_amdgcn_cosf(ub[bk][r] * ear[set]), ub[bk][r] + hh[set]);
          op[r] = am_pair(sv);
        }
      }
      if (i_lo > 0 || i_hi < AM_UPB * 16 - 1) {  // DownSample1d replicate padding (act_mfma_kernel)
        auto pick = [&](int i) -> uint32_t {
          uint32_t v = 0u;
#pragma unroll
          for (int bk = 0; bk < AM_UPB; ++bk) {
            const uint32_t* sp = reinterpret_cast<const uint32_t*>(&sf[bk]);
#pragma unroll
            for (int r = 0; r < 4; ++r) v = (bk == (i >> 4) && r == (i & 3)) ? sp[r] : v;
          }
          return v;
        };
        const int il = max(i_lo, 0), ih = min(max(i_hi, 0), AM_UPB * 16 - 1);
        const uint32_t vlo = (uint32_t)__shfl((int)pick(il), ((il >> 2) & 3) * 16 + l16);
        const uint32_t vhi = (uint32_t)__shfl((int)pick(ih), ((ih >> 2) & 3) * 16 + l16);
#pragma unroll
        for (int bk = 0; bk < AM_UPB; ++bk) {
          uint32_t* sp = reinterpret_cast<uint32_t*>(&sf[bk]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * bk + 4 * q4 + r;
            if (i_lo > 0 && i < i_lo) sp[r] = vlo;
            if (i_hi >= 0 && i_hi < AM_UPB * 16 - 1 && i > i_hi) sp[r] = vhi;
          }
        }
      }
#pragma unroll
      for (int d = 0; d < AM_TT / 16; ++d) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < 3; ++p)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, sf[2 * d + p]), bdn[p], acc, 0, 0, 0);
        uint2 w;
        w.x = (uint32_t)__builtin_bit_cast(u16, (_Float16)acc[0]) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)acc[1]) << 16);
        w.y = (uint32_t)__builtin_bit_cast(u16, (_Float16)acc[2]) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)acc[3]) << 16);
        *reinterpret_cast<uint2*>(ob + (16 * d + l16) * OS + wave * 16 + 4 * q4) = w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the set's tile staged
      u16* const yb = S.y[set] + (int64_t)b * T * Cp + ct * 64;
#pragma unroll
      for (int k = 0; k < AM_TT * 8 / 256; ++k) {
        const int e = tid + 256 * k, r = e >> 3, sg = e & 7;
        if (t0 + r < T)
          *reinterpret_cast<uint4*>(yb + (int64_t)(t0 + r) * Cp + sg * 8) = *reinterpret_cast<const uint4*>(ob + r * OS + sg * 8);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ob reads retired (and, after the last set,
                                                                        // every wave past its up reads of xs)
    }
  }
}

int act_mfma3(const float* x, void* const y[3], int B, int T, int C, int Cp, const float* const alpha_exp[3],
              const float* const inv_beta[3], const Taps12O& f, hipStream_t s) {
  if ((((uintptr_t)x) & 15)) return set_error(ALCM_E_INVALID, "act_mfma3: alignment");
  ActSets S{};
  for (int i = 0; i < 3; ++i) {
    if ((((uintptr_t)y[i]) & 15)) return set_error(ALCM_E_INVALID, "act_mfma3: alignment");
    S.y[i] = (u16*)y[i];
    S.aexp[i] = alpha_exp[i];
    S.ibeta[i] = inv_beta[i];
  }
  constexpr int TT = 64;
  const int tiles_t = (T + TT - 1) / TT, tiles_c = C / 64;
  const int strips_t = (tiles_t + AM_STRIP - 1) / AM_STRIP;
  const int64_t nwg = (int64_t)B * strips_t * tiles_c;
  if (nwg >= (1ll << 31) || (int64_t)T * C >= (1ll << 31)) return set_error(ALCM_E_INVALID, "act_mfma3: too large");
  hipLaunchKernelGGL(act_mfma3_kernel<TT>, dim3((unsigned)nwg), dim3(256), 0, s, x, S, T, C, Cp, f, strips_t, tiles_c);
  ALCM_HIP(hipGetLastError());
  return 0;
}

bool act_mfma_ok(int C, int Cp, int prec) {
  return knobs().act_mfma && prec == PREC_F16 && C >= 192 && C % 64 == 0 && Cp == C;
}

int act_mfma(const void* x, bool x16, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
             const float* inv_beta, const Taps12O& f, hipStream_t s) {
  if ((((uintptr_t)x) & 15) || (((uintptr_t)y) & 15)) return set_error(ALCM_E_INVALID, "act_mfma: alignment");
  constexpr int TT = 64;
  const int tiles_t = (T + TT - 1) / TT, tiles_c = C / 64;
  const int strips_t = (tiles_t + AM_STRIP - 1) / AM_STRIP;
  const int64_t nwg = (int64_t)B * strips_t * tiles_c;
  if (nwg >= (1ll << 31) || (int64_t)T * C >= (1ll << 31)) return set_error(ALCM_E_INVALID, "act_mfma: too large");
  auto kern = x16 ? (knobs().act_defer ? act_mfma_kernel<TT, true, true> : act_mfma_kernel<TT, false, true>)
                  : (knobs().act_defer ? act_mfma_kernel<TT, true> : act_mfma_kernel<TT, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), 0, s, x, (u16*)y, T, C, Cp, alpha_exp, inv_beta, f,
                     strips_t, tiles_c);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// Fused BigVGAN output head (models.py:201-203): activation_post (Activation1d) -> conv_post (k7, C -> 1, zero pad 3)
// -> tanh, all in fp32 on the VALU, one launch.  Replaces an Activation1d into bf16 hi/lo planes (its 8 B per element
// written and read back) and a split-precision N = 1 MFMA conv padded to 16 columns (0.32 + 0.74 ms per step).  Per
// tile of 128 waveform samples of one clip: phase 1 as act_coop_kernel (every upsampled + SnakeBeta sample once,
// replicate padding by clamped indices, the same tap order), phase 2 the 12-tap down filter for the 134 activation
// rows the conv reads (rows outside [0, T) are the conv's zero padding) into LDS, phase 3 two lanes per sample (12
// channels each) for the 7 x C taps, summed in (tap, channel) order per half, bias, tanh.
template <int C>
__global__ __launch_bounds__(256) void post_kernel(const float* __restrict__ x, float* __restrict__ wav, int T,
                                                   const float* __restrict__ aexp, const float* __restrict__ ibeta,
                                                   const Taps12O f, const float* __restrict__ w, float bias,
                                                   int tiles_t) {
  constexpr float INV_PI = 0.318309886183790671538f;
  constexpr int NP = C / 2;           // channel pairs
  constexpr int TT = 128;             // samples per tile
  constexpr int AR = TT + 6;          // activation rows the k7 conv reads
  constexpr int SEG = 18, NSEG = 16;  // phase 1: 16 segments of 18 upsampled samples (>= 2 AR + 12)
  constexpr int RS = NP + 1;          // sample-row stride (f32x2)
  constexpr int RUN = 9;              // phase 2: 16 runs of 9 rows (>= AR)
  constexpr int ARS = C + 1;          // activation row stride (floats, odd)
  static_assert(NP <= 16 && NSEG * SEG >= 2 * AR + 12 && 16 * RUN >= AR, "post tile");
  __shared__ __attribute__((aligned(16))) f32x2 sv[NSEG * SEG * RS];
  __shared__ float av[16 * RUN * ARS];
  __shared__ float wl[7 * C];
  const int tid = threadIdx.x;
  const int tile = blockIdx.x % tiles_t, b = blockIdx.x / tiles_t;
  const int t0 = tile * TT;
  const int j0a = t0 - 3;              // first activation row
  const int m0 = 2 * j0a - 6;          // first upsampled sample (even)
  for (int i = tid; i < 7 * C; i += 256) wl[i] = w[i];
  const float* xb = x + (int64_t)b * T * C;
  const int p = tid & 15;
  const bool live = p < NP;
  const int c = 2 * (live ? p : 0);
  const f32x2 ear = f32x2{aexp[c], aexp[c + 1]} * INV_PI;
  const f32x2 h = f32x2{ibeta[c], ibeta[c + 1]} * 0.5f;
  // ---- phase 1: upsampled + SnakeBeta samples m0 + seg * 18 .. + 17 of pair p
  if (live) {
    const int seg = tid >> 4;
    const int mb = m0 + seg * SEG;
    const int xlo = mb / 2 - 3;
    if (mb >= 0 && mb + SEG - 1 <= 2 * T - 1 && xlo >= 0 && xlo + 14 <= T - 1) {
      f32x2 win[15];
#pragma unroll
      for (int i = 0; i < 15; ++i) win[i] = *reinterpret_cast<const f32x2*>(xb + (xlo + i) * C + c);
      f32x2 u[SEG];
#pragma unroll
      for (int q = 0; q < SEG; ++q) u[q] = f32x2{0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 6; ++kk)
#pragma unroll
        for (int q = 0; q < SEG; ++q) {
          const int ku = 2 * kk + ((q & 1) ? 0 : 1);
          u[q] = fma2(f32x2{f.up[ku], f.up[ku]}, win[(q + 5 - ku) / 2 + 3], u[q]);
        }
#pragma unroll
      for (int q = 0; q < SEG; ++q) sv[(seg * SEG + q) * RS + p] = snake2(u[q], ear, h);
    } else {
      for (int q = 0; q < SEG; ++q) {
        int m = mb + q;
        m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
        f32x2 u = f32x2{0.f, 0.f};
        for (int kk = 0; kk < 6; ++kk) {
          const int ku = 2 * kk + ((m & 1) ? 0 : 1);
          int xi = (m + 5 - ku) / 2;
          xi = xi < 0 ? 0 : (xi > T - 1 ? T - 1 : xi);
          u = fma2(f32x2{f.up[ku], f.up[ku]}, *reinterpret_cast<const f32x2*>(xb + xi * C + c), u);
        }
        sv[(seg * SEG + q) * RS + p] = snake2(u, ear, h);
      }
    }
  }
  __syncthreads();
  // ---- phase 2: activation rows j0a + run * 9 .. + 8 of pair p: o[r] = sum_k dn[k] * sv[2 (row) + 1 + k]
  const int run = tid >> 4;
  const int r0 = run * RUN;
  if (live && r0 < AR) {
    const f32x2* sp = sv + (2 * r0 + 1) * RS + p;
    f32x2 sm[2 * RUN + 10];
#pragma unroll
    for (int i = 0; i < 2 * RUN + 10; ++i) sm[i] = sp[i * RS];
    f32x2 o[RUN];
#pragma unroll
    for (int r = 0; r < RUN; ++r) o[r] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
      for (int r = 0; r < RUN; ++r) o[r] = fma2(f32x2{f.dn[k], f.dn[k]}, sm[2 * r + k], o[r]);
#pragma unroll
    for (int r = 0; r < RUN; ++r) {
      const int j = j0a + r0 + r;
      const bool in = j >= 0 && j < T;
      av[(r0 + r) * ARS + c] = in ? o[r].x : 0.f;
      av[(r0 + r) * ARS + c + 1] = in ? o[r].y : 0.f;
    }
  }
  __syncthreads();
  // ---- phase 3: sample t0 + q from activation rows q .. q + 6 (local), lanes 2q / 2q + 1 take channels [0, C/2) /
  //      [C/2, C)
  const int q = tid >> 1, half = tid & 1;
  float acc = 0.f;
#pragma unroll
  for (int tap = 0; tap < 7; ++tap)
#pragma unroll
    for (int cc = 0; cc < C / 2; ++cc) {
      const int ch = half * (C / 2) + cc;
      acc = fmaf(wl[tap * C + ch], av[(q + tap) * ARS + ch], acc);
    }
  const float y = acc + __shfl_xor(acc, 1) + bias;
  const int t = t0 + q;
  if (half == 0 && t < T) wav[(int64_t)b * T + t] = tanhf(y);
}

int act_conv_post(const float* x, float* wav, int B, int T, int C, const float* alpha_exp, const float* inv_beta,
                  const Taps12O& f, const float* w_tc, float bias, hipStream_t s) {
  if (C != 24) return set_error(ALCM_E_INVALID, "act_conv_post: built for C = 24");
  if (!x || !wav || !alpha_exp || !inv_beta || !w_tc || B <= 0 || T <= 0 || (((uintptr_t)x) & 7))
    return set_error(ALCM_E_INVALID, "act_conv_post: bad arguments");
  if ((int64_t)T * C >= (1ll << 31)) return set_error(ALCM_E_INVALID, "act_conv_post: clip too long");
  const int tiles_t = (T + 127) / 128;
  const int64_t nwg = (int64_t)B * tiles_t;
  if (nwg >= (1ll << 31)) return set_error(ALCM_E_INVALID, "act_conv_post: problem too large");
  hipLaunchKernelGGL(post_kernel<24>, dim3((unsigned)nwg), dim3(256), 0, s, x, wav, T, alpha_exp, inv_beta, f, w_tc,
                     bias, tiles_t);
  ALCM_HIP(hipGetLastError());
  return 0;
}

// fp32 channels-last rows -> MFMA operand planes [rows][Cp] (channels C .. Cp-1 zero), the format `prec` reads:
// the input of a plane conv whose producer writes fp32 (the BigVGAN upsampler reads the stage output x)
template <int PREC>
__global__ void to_planes_kernel(const float* __restrict__ x, u16* __restrict__ y, int64_t rows, int C, int Cp,
                                 int64_t y_lo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int cq = Cp / 4;
  if (i >= rows * cq) return;
  const int64_t r = i / cq;
  const int c = (int)(i - r * cq) * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C) v = *reinterpret_cast<const float4*>(x + r * C + c);
  u16* yp = y + r * Cp + c;
  op_store2<PREC>(yp, y_lo, f32x2{v.x, v.y});
  op_store2<PREC>(yp + 2, y_lo, f32x2{v.z, v.w});
}

int to_planes(const float* x, void* y, int64_t rows, int C, int Cp, int prec, hipStream_t s) {
  if (!x || !y || rows <= 0 || C <= 0 || C % 4 || Cp % 32 || C > Cp || (((uintptr_t)x) & 15) || (((uintptr_t)y) & 7))
    return set_error(ALCM_E_INVALID, "to_planes: bad arguments");
  const int64_t n = rows * (Cp / 4);
  const dim3 grid((unsigned)((n + 255) / 256));
  const int64_t lo = rows * Cp;
  if (prec == PREC_SPLIT) hipLaunchKernelGGL(to_planes_kernel<PREC_SPLIT>, grid, dim3(256), 0, s, x, (u16*)y, rows, C, Cp, lo);
  else if (prec == PREC_BF16) hipLaunchKernelGGL(to_planes_kernel<PREC_BF16>, grid, dim3(256), 0, s, x, (u16*)y, rows, C, Cp, lo);
  else hipLaunchKernelGGL(to_planes_kernel<PREC_F16>, grid, dim3(256), 0, s, x, (u16*)y, rows, C, Cp, lo);
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm
