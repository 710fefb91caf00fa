// Fused AMPBlock1 half-layer pair of the narrow BigVGAN stages (C = 96 / 48 / 24; vocoder/bigvgan/models.py:72-81):
//
//     x_next = x + conv2_{k,1}( Activation1d_2( conv1_{k,d}( Activation1d_1(x) ) ) )
//
// in ONE launch, instead of an Activation1d (or a conv epilogue) writing operand planes to HBM, conv1 reading them and
// writing the next planes, and conv2 reading those, the fp32 residual and writing the fp32 state plus planes (3x the
// bytes of this kernel's x in / x_next out, and three kernels' worth of pipeline fill, latency and tail).
//
// One persistent 512-thread workgroup per CU walks output tiles of E rows (XCD-aware: an XCD owns a contiguous tile
// range, so neighbouring tiles' halo rows are shared in its L2).  Per tile, with conv rows [s1, s1 + CR):
//   1. act1: x rows [s1 - p1 - 6, s1 + CR + p1 + 6) (global, fp32) -> fp16 operand rows a1 [s1 - p1, s1 + CR + p1)
//      in LDS (rows outside [0, T): zeros = conv1's zero padding; replicate padding near the ends as clamped reads);
//   2. conv1 (dense K = tap * C + c; weights by LDS-DMA, resident for the launch (C = 24), one conv resident and
//      swapped under the other phase (C = 48) or streamed per 32-deep slice through a ring (C = 96)) -> acc + bias
//      staged in LDS (fp32, one channel group at a time);
//   3. act2 from the staged rows -> fp16 operand rows a2 [s1 + 6, s1 + CR - 6) over the dead a1 rows;
//   4. conv2 over a2 -> + bias + residual (prefetched during act2) -> x_next rows [e0, e0 + E), e0 = s1 + 6 + (k-1)/2,
//      or for a resblock's last pair the stage mean: out = x_next * out_scale (+ out).
// Every sum keeps the order of the unfused kernels (alcm_tconv.hip: the same dense K slices and MFMA operand lanes,
// lo-plane MFMA before the hi-plane one; alcm_actepi.h: the same Activation1d chains), so the result is bit-identical
// to act_op -> tconv conv1 (+ fused Activation1d) -> tconv conv2 (+ residual), which tests/test_gpu_ops.py checks.
#include <cstdio>
#include <cstring>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

typedef __attribute__((address_space(3))) void ap_lds_t;
typedef __attribute__((address_space(1))) void ap_gbl_t;

__device__ __attribute__((aligned(16))) uint4 g_ampair_zero[8];  // a zero line for padding-row DMA lanes

struct APairDev {
  const float* x;  // [B][T][C] fp32: input state (and the residual)
  float* out;      // [B][T][C]: x_next, or (LAST) the stage accumulator
  int T, dil, p1;  // p1 = (k - 1) * dil / 2
  const u16* w1;   // dense fp16 weights [C][kd] (K = tap * C + c), hi plane; lo plane at + w_lo (F16W2)
  const u16* w2;
  int64_t w_lo;
  const float* b1;
  const float* b2;
  float out_scale;
  int accumulate;
  const float* ae1;  // exp(alpha), 1 / (exp(beta) + 1e-9) of the two SnakeBetas (activations.py:111-119)
  const float* ib1;
  const float* ae2;
  const float* ib2;
  Taps12O f1, f2;
  int tiles_per_batch, ntiles;
  int ablate;  // diagnostics (ALCM_AMPAIR_ABLATE, timing only, results wrong): 1 no act1, 2 no act2, 4 no MFMAs,
               // 8 no output stores
};

template <int C, int NPB, int KS, int CR, int NW_, int V1C_, int WM_, int RD_>
struct APairGeo {
  static constexpr int NW = NW_, NT = NW * 64;
  static constexpr int TM = CR / 16 / NW;                 // 16-row M tiles per wave
  static constexpr int NSP = (C + 15) / 16 * 16, TN = NSP / 16;
  static constexpr int P2 = (KS - 1) / 2;
  static constexpr int E = CR - 12 - 2 * P2;              // emitted rows per tile
  static constexpr int P1MAX = (KS - 1) * 5 / 2;          // dilations <= 5 (BigVGAN: 1, 3, 5)
  static constexpr int A1R = CR + 2 * P1MAX;              // a1 rows (a2 reuses them: CR + 2 P2 <= A1R)
  static constexpr int RSS = (C / 8) % 2 ? C / 8 : C / 8 + 1;  // operand row: odd number of 16-B slots
  static constexpr int RS = RSS * 16;
  static constexpr int A1B = (A1R * RS + 1023) / 1024 * 1024;
  static constexpr int V1C = V1C_, NG = C / V1C;          // conv1 output staged in groups of V1C channels
  static constexpr int V1S = V1C + 2;                     // staged row stride (floats)
  static constexpr int V1B = (CR * V1S * 4 + 1023) / 1024 * 1024;
  static constexpr int KD = (KS * C + 31) / 32 * 32;      // dense K
  static constexpr int NS = KD / 32;                      // slices per conv
  // weight modes: WM 0 streams 32-deep slices of both convs through a ring of RD + 1 slots (RD slices in flight
  // across phases and tiles); WM 1 keeps both convs' weights resident for the whole launch; WM 2 keeps one conv's
  // resident and swaps it under the other phase (W2 loads under act2, the next tile's W1 under the epilogue + act1)
  static constexpr int WM = WM_, RD = RD_, RING = RD + 1;
  static constexpr int SLOT = NSP * 64 * NPB;             // ring: one 32-deep slice of every weight plane
  static constexpr int SPI = SLOT / 1024;                 // DMA instructions per slice
  static constexpr int DPW = (SPI + NW - 1) / NW;         // per wave (uniform: surplus lanes write the scratch line)
  static constexpr int WSL = (KD / 8) % 2 ? KD / 8 : KD / 8 + 1;  // resident: weight row of an odd number of 16-B
  static constexpr int WRS = WSL * 16;                             // slots (conflict-free 16-row fragment reads)
  static constexpr int WCONV = NPB * NSP * WRS;           // one conv's resident planes [plane][row][K]
  static constexpr int WCR = (WCONV + 1023) / 1024 * 1024;
  static constexpr int WB = WM == 0 ? RING * SLOT + 1024 : (WM == 1 ? 2 : 1) * WCR;
  static constexpr int SMEM = A1B + V1B + WB;
  static_assert(C % 16 == 8 || C % 16 == 0, "C % 8");
  static_assert(CR % (16 * NW) == 0 && SLOT % 1024 == 0 && C % V1C == 0 && V1C % 2 == 0, "geometry");
  static_assert(WM == 0 ? (RD >= 2 && (RD - 1) * DPW < 64) : RD == 0, "ring depth");
  static_assert(SMEM <= (NW == 4 ? 81920 : 163840), "LDS (4 waves: two workgroups per CU)");
};

__device__ __forceinline__ void ap_glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((ap_gbl_t*)src, (ap_lds_t*)lds, 16, 0, 0);
}

// fp16 pair -> 4 bytes of an LDS operand row
__device__ __forceinline__ void ap_st2(char* p, f32x2 v) {
  *reinterpret_cast<uint32_t*>(p) =
      (uint32_t)__builtin_bit_cast(u16, (_Float16)v.x) | ((uint32_t)__builtin_bit_cast(u16, (_Float16)v.y) << 16);
}

template <int N>
__device__ __forceinline__ void ap_wait_barrier() {
  static_assert(N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));  // vmcnt(N) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

// Activation1d rows [0, n) of one tile: output row lr is global row t_org + lr, written as fp16 into the operand rows
// dst + lr * RS (rows outside [0, T): zeros); ld(i, p) returns input row i of pair p for ANY 0 <= i < T (the caller's
// loader also clamps to its own storage).  Work item = (run of R rows, channel pair), pairs fastest.  A run whose
// window lies inside [0, T) takes act_run_interior (a partial last run computes R rows and stores jn); runs at the
// sequence ends take act_run_edge on clamped windows, R/2 rows at a time (register budget)
template <int R, int NP, int RS, int NT, class LD>
__device__ __forceinline__ void ap_act(int n, int t_org, int T, const Taps12O& f, const float* ae, const float* ib,
                                       int c0, char* dst, int tid, LD ld) {
  constexpr float INV_PI = 0.318309886183790671538f;
  constexpr int RH = R / 2;
  static_assert(R % 2 == 0, "edge halves");
  const int nrun = (n + R - 1) / R;
  for (int w = tid; w < NP * nrun; w += NT) {
    const int run = w / NP, p = w - run * NP;
    const int c = c0 + 2 * p;
    const int lr0 = run * R, t0 = t_org + lr0;
    const int jn = min(R, n - lr0);
    const f32x2 ear = f32x2{ae[c], ae[c + 1]} * INV_PI;
    const f32x2 h = f32x2{ib[c], ib[c + 1]} * 0.5f;
    char* d = dst + lr0 * RS + c * 2;
    if (t0 >= 6 && t0 + jn + 6 <= T) {
      f32x2 win[R + 12];
#pragma unroll
      for (int i = 0; i < R + 12; ++i) win[i] = ld(min(t0 - 6 + i, T - 1), p);
      f32x2 o[R];
      act_run_interior<R>(win, f, ear, h, o);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < jn) ap_st2(d + r * RS, o[r]);
    } else {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (hh * RH >= jn) break;
        const int j0 = t0 + hh * RH;
        f32x2 win[RH + 12];
#pragma unroll
        for (int i = 0; i < RH + 12; ++i) win[i] = ld(min(max(j0 - 6 + i, 0), T - 1), p);
        f32x2 o[RH];
        act_run_edge<RH>(win, j0, T, f, ear, h, o);
#pragma unroll
        for (int r = 0; r < RH; ++r) {
          const int t = j0 + r;
          if (hh * RH + r < jn) ap_st2(d + (hh * RH + r) * RS, (t >= 0 && t < T) ? o[r] : f32x2{0.f, 0.f});
        }
      }
    }
  }
}

template <int C, int NPB, int KS, int CR, int NW, int V1C_, int WM, int RD, int R, bool LAST>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void ampair_kernel(const APairDev P) {
  using G = APairGeo<C, NPB, KS, CR, NW, V1C_, WM, RD>;
  constexpr int NT = G::NT, TM = G::TM, TN = G::TN, NSP = G::NSP, RS = G::RS, NS = G::NS;
  constexpr int E = G::E, P2 = G::P2, V1C = G::V1C, V1S = G::V1S, SLOT = G::SLOT;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  char* const abuf = smem;                                         // a1, then a2
  float* const v1 = reinterpret_cast<float*>(smem + G::A1B);       // staged conv1 output (one channel group)
  char* const wbuf = smem + G::A1B + G::V1B;                       // weight ring (WM 0) or resident weights
  char* const scratch = wbuf + G::RING * SLOT;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, l16 = lane & 15;
  const int T = P.T;

  // persistent, XCD-aware: XCD x owns tiles [x R8, (x + 1) R8), its workgroups take every nslot-th of them
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int R8 = (P.ntiles + 7) >> 3;
  const int tbeg = xcd * R8 + slot, tend = min(xcd * R8 + R8, P.ntiles);
  const int my_n = tbeg < tend ? (tend - tbeg + nslot - 1) / nslot : 0;
  if (my_n == 0) return;
  const int total = my_n * 2 * NS;  // WM 0: weight slices this workgroup streams
  // the K padding (k >= KS * C) reads up to two rows past the rows act1 writes, against zero weights: start from
  // zeroed operand rows so those reads are finite (uninitialised LDS could hold NaN bit patterns, NaN * 0 = NaN)
  for (int i = tid; i < G::A1B / 16; i += NT) reinterpret_cast<uint4*>(abuf)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();

  // WM 0: weight slice gs (tile gs / (2 NS), conv (gs / NS) & 1, slice gs % NS) -> ring slot gs % RING; instruction
  // i = wave + NW j covers bytes [1024 i, 1024 i + 1024) of the slot: [plane][row n of 64 B][piece], the 16-B piece
  // pq of row n holding K piece pq ^ ((n >> 2) & 3) (conflict-free ds_read_b128 of 16 consecutive rows)
  auto issue = [&](int gs) {
    const int sl = gs % NS;
    const u16* wb = ((gs / NS) & 1) ? P.w2 : P.w1;
    char* dst = wbuf + (gs % G::RING) * SLOT;
#pragma unroll
    for (int j = 0; j < G::DPW; ++j) {
      const int i = wave + G::NW * j;
      const int g = i * 64 + lane;
      const int p = g / (NSP * 4), gg = g - p * (NSP * 4);
      const int n = gg >> 2, pq = gg & 3;
      const int q = pq ^ ((n >> 2) & 3);
      const bool ok = i < G::SPI && n < C;
      const u16* src = ok ? wb + p * P.w_lo + n * G::KD + sl * 32 + q * 8 : reinterpret_cast<const u16*>(g_ampair_zero);
      ap_glds16(src, i < G::SPI ? dst + i * 1024 : scratch);
    }
  };
  // WM 1 / 2: one conv's weights -> resident image [plane][row n (WRS bytes)][K], lane-linear 1 KB DMA instructions
  // (rows >= C, the odd-slot pad and the last instruction's tail: zeros / the region's padding)
  auto load_w = [&](const u16* wsrc, char* dst) {
    constexpr int NI = G::WCR / 1024;
    for (int i = wave; i < NI; i += NW) {
      const int o = i * 1024 + lane * 16;
      const int p = o / (NSP * G::WRS), r = o - p * (NSP * G::WRS);
      const int n = r / G::WRS, qq = (r - n * G::WRS) >> 4;
      const bool ok = o < G::WCONV && n < C && qq < G::KD / 8;
      const u16* src = ok ? wsrc + p * P.w_lo + n * G::KD + qq * 8 : reinterpret_cast<const u16*>(g_ampair_zero);
      ap_glds16(src, dst + i * 1024);
    }
  };
  if constexpr (WM == 0) {
#pragma unroll
    for (int d = 0; d < RD; ++d)
      if (d < total) issue(d);
  } else {
    load_w(P.w1, wbuf);
    if constexpr (WM == 1) load_w(P.w2, wbuf + G::WCR);
  }

  const int bsw = (l16 >> 2) & 3;
  f32x4 acc[TM][TN];
  // one conv's K loop over the operand rows `a` (row of M tile i of this wave for tap t: wave * TM * 16 + i * 16 +
  // l16 + t * dl).  WM 0: slices gs0 .. gs0 + NS - 1 from the ring; slice gs + RD is issued into the slot slice
  // gs - 1 used, one barrier per slice behind a counted wait that leaves the younger slices in flight.  WM 1 / 2:
  // straight from the resident image (no waits, no barriers)
  auto kloop = [&](const char* a, int dl, int conv, int gs0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* arow = a + (wave * TM * 16 + l16) * RS;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int gs = gs0 + s;
      const bool more = WM == 0 && gs + RD < total;
      const int kk = s * 32 + q4 * 8;
      int tap = kk / C;
      const int c = kk - tap * C;
      tap = min(tap, KS - 1);  // K padding: zero weights, any finite operand row
      constexpr int BJ = WM == 0 ? 16 * 64 : 16 * G::WRS, BP = WM == 0 ? NSP * 64 : NSP * G::WRS;
      const char* bs;
      if constexpr (WM == 0) {
        if (more) issue(gs + RD);
        bs = wbuf + (gs % G::RING) * SLOT + l16 * 64 + ((q4 ^ bsw) << 4);
      } else {
        bs = wbuf + (WM == 1 ? conv * G::WCR : 0) + l16 * G::WRS + kk * 2;
      }
      bf16x8 af[TM], bh[TN], bl[NPB == 2 ? TN : 1];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(bs + j * BJ);
        if constexpr (NPB == 2) bl[j] = *reinterpret_cast<const bf16x8*>(bs + BP + j * BJ);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(arow + (i * 16 + tap * dl) * RS + c * 2);
      if (P.ablate & 4) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bh[j]));
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (NPB == 2) acc[i][j] = mfma16<PREC_F16>(af[i], bl[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_F16>(af[i], bh[j], acc[i][j]);
          }
      }
      if constexpr (WM == 0) {
        if (more) ap_wait_barrier<(RD - 1) * G::DPW>();
        else ap_wait_barrier<0>();
      }
    }
  };

  for (int it = 0; it < my_n; ++it) {
    const int tile = tbeg + it * nslot;
    const int b = tile / P.tiles_per_batch;
    const int e0 = (tile - b * P.tiles_per_batch) * E;
    const int s1 = e0 - 6 - P2;
    const float* xb = P.x + (int64_t)b * T * C;
    const int gs0 = it * 2 * NS;

    // ---- 1. act1: x -> a1 rows [s1 - p1, s1 + CR + p1)
    if (!(P.ablate & 1))
    ap_act<R, C / 2, RS, NT>(CR + 2 * P.p1, s1 - P.p1, T, P.f1, P.ae1, P.ib1, 0, abuf, tid,
                              [&](int i, int p) {
                                return *reinterpret_cast<const f32x2*>(
                                    reinterpret_cast<const char*>(xb) + (uint32_t)(i * C + 2 * p) * 4u);
                              });
    // a1 complete; WM 0: slice gs0 resident for every wave (younger slices may stay in flight); WM 1 / 2: W1 resident
    if constexpr (WM == 0) ap_wait_barrier<(RD - 1) * G::DPW>();
    else ap_wait_barrier<0>();

    // ---- 2. conv1
    kloop(abuf, P.dil, 0, gs0);

    float rv[TM][TN][4];
    // ---- 3. act2 per channel group: conv1 + bias -> LDS, then Activation1d -> a2 rows [s1 + 6, s1 + CR - 6)
#pragma unroll
    for (int g = 0; g < G::NG; ++g) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wave * TM * 16 + i * 16 + q4 * 4 + r;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = j * 16 + l16;
            if (n >= g * V1C && n < (g + 1) * V1C && n < C)
              v1[m * V1S + n - g * V1C] = acc[i][j][r] + P.b1[n];
          }
        }
      __syncthreads();
      if constexpr (WM == 2)
        if (g == 0) load_w(P.w2, wbuf);  // every wave is past conv1: W2 over W1, under act2
      if (g == G::NG - 1) {
        // residual rows of this wave's conv2 outputs (row e0 + wave TM 16 + 16 i + 4 q4 + r, column 16 j + l16),
        // loaded under the last group's act2 (the accumulators are dead by then: no register overlap)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int r2 = wave * TM * 16 + i * 16 + q4 * 4 + r;
            const int t = e0 + r2;
            const bool okr = r2 < E && t < T;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int n = j * 16 + l16;
              rv[i][j][r] = (okr && n < C) ? xb[(int64_t)t * C + n] : 0.f;
            }
          }
      }
      if (!(P.ablate & 2))
      ap_act<R, V1C / 2, RS, NT>(CR - 12, s1 + 6, T, P.f2, P.ae2, P.ib2, g * V1C, abuf, tid,
                                  [&](int i, int p) {  // (rows past the staged tile: a partial run's unused tail)
                                    return *reinterpret_cast<const f32x2*>(v1 + min(i - s1, CR - 1) * V1S + 2 * p);
                                  });
      if (WM == 2 && g == G::NG - 1) ap_wait_barrier<0>();  // a2 complete, W2 resident
      else __syncthreads();
    }

    // ---- 4. conv2 + bias + residual -> out
    kloop(abuf, 1, 1, gs0 + NS);
    if constexpr (WM != 0) {
      __syncthreads();  // every wave is past conv2 (a2 / W2 reads) before act1 / the W1 reload overwrite them
      if constexpr (WM == 2)
        if (it + 1 < my_n) load_w(P.w1, wbuf);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int r2 = wave * TM * 16 + i * 16 + q4 * 4 + r;
        const int t = e0 + r2;
        if (r2 >= E || t >= T || (P.ablate & 8)) continue;
        float* orow = P.out + ((int64_t)b * T + t) * C;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = j * 16 + l16;
          if (n >= C) continue;
          float v = acc[i][j][r] + P.b2[n];
          v += rv[i][j][r];
          if constexpr (LAST) {
            v *= P.out_scale;
            if (P.accumulate) v += orow[n];
          }
          orow[n] = v;
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------------------- host
bool ampair_supported(int prec, int C, int ksize, int dil) {
  if (ksize != 3 && ksize != 7 && ksize != 11) return false;
  if (dil < 1 || dil > 5) return false;
  if (C == 96) return prec == PREC_F16;  // (the tail's F16W2-everywhere diagnostic keeps the unfused path)
  return (C == 48 || C == 24) && prec == PREC_F16W2;
}

static int g_ap_ncu = 0;

template <int C, int NPB, int KS, int CR, int NW, int V1C, int WM, int RD>
static int ap_launch(const APairDev& P, bool last, hipStream_t s) {
  using G = APairGeo<C, NPB, KS, CR, NW, V1C, WM, RD>;
  if (!g_ap_ncu) {
    int dev = 0, n = 0;
    g_ap_ncu = (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n >= 8)
                   ? n
                   : 256;
  }
  const int R8 = (P.ntiles + 7) / 8;
  int grid = 8 * std::min(g_ap_ncu * (NW == 4 ? 2 : 1) / 8, R8);
  if (knobs().ampair_grid >= 8) grid = std::min(grid, knobs().ampair_grid / 8 * 8);  // tests: several tiles per WG
  if (last)
    hipLaunchKernelGGL((ampair_kernel<C, NPB, KS, CR, NW, V1C, WM, RD, 16, true>), dim3(grid), dim3(G::NT), 0, s, P);
  else
    hipLaunchKernelGGL((ampair_kernel<C, NPB, KS, CR, NW, V1C, WM, RD, 16, false>), dim3(grid), dim3(G::NT), 0, s, P);
  return 0;
}

template <int C, int NPB, int CR, int NW, int V1C, int WM, int RD>
static int ap_by_k(const APairDev& P, int ksize, bool last, hipStream_t s) {
  switch (ksize) {
    case 3: return ap_launch<C, NPB, 3, CR, NW, V1C, WM, RD>(P, last, s);
    case 7: return ap_launch<C, NPB, 7, CR, NW, V1C, WM, RD>(P, last, s);
    default: return ap_launch<C, NPB, 11, CR, NW, V1C, WM, RD>(P, last, s);
  }
}

// tile geometry by width (ALCM_AMPAIR_NW = 4: the first cut's two 4-wave workgroups per CU, <= 80 KB of LDS each,
// streaming weights through a 3-slot ring).  Default, one 8-wave workgroup per CU: C = 24 keeps both convs' weights
// resident (76 KB at k = 11) over 512 conv rows; C = 48 keeps one conv's (104 KB) and swaps it under the other phase;
// C = 96 (its operand rows alone take 64 KB) streams through a 5-slot ring, four slices in flight
static int ap_waves(int C) { return (C != 96 && knobs().ampair_nw == 4) ? 4 : 8; }
static int ap_rows(int C, int nw) { return (C == 24 && nw == 8) ? 512 : 256; }
static int ap_emitted(int C, int ksize) { return ap_rows(C, ap_waves(C)) - 12 - (ksize - 1); }

// x_next (or, last, the stage mean) of one AMPBlock1 half-layer pair; weights dense fp16 [C][kd] (hi plane at w1 / w2,
// lo plane w_lo elements after it for F16W2), activation parameters as the fused epilogues take them
int ampair(const float* x, float* out, int B, int T, int C, int ksize, int dil, const u16* w1, const u16* w2,
           int64_t w_lo, int kd, const float* b1, const float* b2, float out_scale, int accumulate, bool last,
           const float* ae1, const float* ib1, const Taps12O& f1, const float* ae2, const float* ib2,
           const Taps12O& f2, int prec, hipStream_t s) {
  if (!ampair_supported(prec, C, ksize, dil)) return set_error(ALCM_E_INVALID, "ampair: unsupported shape");
  if (!x || !out || !w1 || !w2 || !b1 || !b2 || !ae1 || !ib1 || !ae2 || !ib2 || B <= 0 || T <= 0 || x == out)
    return set_error(ALCM_E_INVALID, "ampair: bad arguments");
  if (kd != (ksize * C + 31) / 32 * 32) return set_error(ALCM_E_INVALID, "ampair: dense weight layout");
  if ((((uintptr_t)x) & 7) || (((uintptr_t)w1) & 15) || (((uintptr_t)w2) & 15) || (prec == PREC_F16W2 && (w_lo % 8)))
    return set_error(ALCM_E_INVALID, "ampair: alignment");
  if ((int64_t)T * C >= (1ll << 29)) return set_error(ALCM_E_INVALID, "ampair: clip too long");
  APairDev P{};
  P.x = x; P.out = out; P.T = T; P.dil = dil; P.p1 = (ksize - 1) * dil / 2;
  P.w1 = w1; P.w2 = w2; P.w_lo = w_lo;
  P.b1 = b1; P.b2 = b2; P.out_scale = out_scale; P.accumulate = last ? accumulate : 0;
  P.ae1 = ae1; P.ib1 = ib1; P.ae2 = ae2; P.ib2 = ib2; P.f1 = f1; P.f2 = f2;
  P.ablate = knobs().ampair_ablate;
  const int E = ap_emitted(C, ksize);
  P.tiles_per_batch = (T + E - 1) / E;
  const int64_t nt = (int64_t)B * P.tiles_per_batch;
  if (nt >= (1ll << 30)) return set_error(ALCM_E_INVALID, "ampair: problem too large");
  P.ntiles = (int)nt;
  void* tok = prof_start(s);
  int rc;
  const int nw = ap_waves(C);
  if (C == 24)
    rc = nw == 8 ? ap_by_k<24, 2, 512, 8, 24, 1, 0>(P, ksize, last, s) : ap_by_k<24, 2, 256, 4, 24, 0, 2>(P, ksize, last, s);
  else if (C == 48)
    rc = nw == 8 ? ap_by_k<48, 2, 256, 8, 16, 2, 0>(P, ksize, last, s) : ap_by_k<48, 2, 256, 4, 24, 0, 2>(P, ksize, last, s);
  else
    rc = ap_by_k<96, 1, 256, 8, 48, 0, 4>(P, ksize, last, s);
  if (rc) return rc;
  ALCM_HIP(hipGetLastError());
  if (tok) {
    const double M = (double)B * T;
    const int npb = prec == PREC_F16W2 ? 2 : 1;
    const double flops = 2.0 * 2.0 * M * C * (double)ksize * C;
    const double bytes = M * C * 4.0 * (last && accumulate ? 3 : 2) + 2.0 * C * kd * 2.0 * npb;
    char name[96];
    std::snprintf(name, sizeof(name), "alcm::ampair_kernel<C%d, W%d, k%d%s>", C, npb, ksize, last ? ", last" : "");
    prof_stop(tok, s, name, flops, bytes);
  }
  return 0;
}

}  // namespace alcm

static void ap_taps(const float* up, const float* dn, alcm::Taps12O& f) {
  for (int k = 0; k < 12; ++k) {
    f.up[k] = 2.0f * up[k];  // UpSample1d's ratio-2 gain folded in (resample.py:30)
    f.dn[k] = dn[k];
  }
}

extern "C" int alcm_ampblock_pair(const alcm_ampair_args* a, alcm_stream_t stream) {
  using namespace alcm;
  if (!a || !a->w1 || !a->w2 || !a->up_filter1 || !a->down_filter1 || !a->up_filter2 || !a->down_filter2)
    return set_error(ALCM_E_INVALID, "ampblock_pair: bad arguments");
  Taps12O f1, f2;
  ap_taps(a->up_filter1, a->down_filter1, f1);
  ap_taps(a->up_filter2, a->down_filter2, f2);
  // packed by alcm_pack_conv_weight (planes bf16 hi, bf16 lo, fp16 hi, fp16 lo of w_lo_off elements each)
  const u16* w1 = (const u16*)a->w1 + 2 * a->w_lo_off;
  const u16* w2 = (const u16*)a->w2 + 2 * a->w_lo_off;
  return ampair(a->x, a->out, a->B, a->T, a->C, a->ksize, a->dil, w1, w2, a->w_lo_off, a->kpad, a->bias1, a->bias2,
                a->out_scale, a->accumulate, a->last != 0, a->alpha_exp1, a->inv_beta1, f1, a->alpha_exp2,
                a->inv_beta2, f2, a->prec, (hipStream_t)stream);
}
