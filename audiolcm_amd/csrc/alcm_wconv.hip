// Wide implicit-GEMM conv1d on MFMA operand planes (fp16 / bf16) for the MFMA-bound layers: BigVGAN stage 0-2
// AMPBlock convs and upsampler phases (vocoder/bigvgan/models.py:72-81, 160-165), the DiT FFN / attention projections
// (ldm/modules/new_attention.py:48-74), the VAE k3 convs and the text encoders' wide linears.  Two kernels:
//   * wconv2_kernel: 4 waves, two workgroups per CU (128 x 192 or 256 x 96 tiles), window staged per 64-channel
//     chunk, weights double-buffered; strided (ConvTranspose phase) and GEGLU-plane epilogues;
//   * wconv3_kernel: one persistent 8-wave workgroup per CU walking a flat (tile, chunk, tap) step sequence.
// Common: LDS-DMA staging (global_load_lds_dwordx4, no VGPR round trip) into lane-linear images whose 16-B slot s of
// row r sits at s ^ (r & 7) (conflict-free ds_read_b128 fragment reads from any start row); rows outside [0, T) read
// a zero line; XCD-aware workgroup order.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"  // op_store2 / f32x2 (the GEGLU plane stores)

namespace alcm {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __attribute__((aligned(16))) uint4 g_wconv_zero[8];  // 128 zero bytes (zero-initialised)

struct WConvDev {
  const u16* a;  // operand plane [B][T][Cp]
  int T, Cp, ksize, dil, pad;
  const u16* w;  // packed weight plane [N][kpad], K = tap * Cp + ci
  int kpad, N;
  const float* bias;
  const float* res;
  float* out;
  float out_scale;
  int accumulate;
  int tiles_per_batch, tiles_n, nwg;
  int n_major;          // workgroup order: 0 = M-tile major (N tiles of an M tile adjacent), 1 = N-tile major
  int ostride, ooff, orows;  // wconv2 output row of input row t: t * ostride + ooff of orows per batch
  u16* gplane;          // GEGLU epilogue: operand plane [B][T][N/2] instead of the fp32 output
  int out_act;          // wconv2: activation of acc + bias (ALCM_ACT_*, 0 = none)
  u16* oplane;          // wconv2: conv + bias as an operand plane [B][T][N] (PREC) instead of the fp32 output
  int ksplit;           // wconv3: > 1 = the 64-channel chunks split into ksplit contiguous parts, one work item per
                        // (tile, part); each item writes its fp32 partial sums to part + kpart * B T N (no epilogue)
  float* part;
  // wconv3 sum form (nseg > 1): out = (sum over s < nseg of conv_s(sa[s], sw[s]) + sbias[s] + sres[s]) * out_scale
  // (+ out): the AMPBlock chains' last conv2 + residual of a stage in one pass (models.py:190-199), every term with
  // the same T, Cp, N and dilation 1, its own plane, weights, taps, bias and residual
  int nseg;
  const u16* sa[3];
  const u16* sw[3];
  int sk[3], spad[3], skpad[3];
  const float* sbias[3];
  const float* sres[3];
};


__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_base, 16, 0, 0);
}

// ---------------------------------------------------------------------------------------------------------
// Two-workgroups-per-CU kernel: 4 waves, each 64 rows x 96 columns (4 x 6 16x16x32 MFMAs per
// 32-deep K slice, 0.42 fragment reads per MFMA), tile BM x BN = 128 x 192 (waves 2 (M) x 2 (N)) or 256 x 96
// (waves 4 (M) x 1 (N)).  <= 72 KB of LDS (one input window of BM + 64 rows x 64 channels + two weight tiles) so
// two workgroups share a CU: the HBM-bound epilogue (fp32 output + residual + accumulate) of one overlaps the MFMA
// K loop of the other (the round-1 one-workgroup 256-row kernel serialised them: its epilogue was 26-80 % of its
// time on the BigVGAN shapes).  K steps: weights double-buffered (step s+1 staged while step s
// computes, vmcnt(0) + barrier per step); the window is single-buffered and re-staged at each 64-channel chunk
// boundary (the stall is covered by the other workgroup).
//
// Tile choice: every tile re-reads the whole weight slice of its N columns once per M tile, so the L2 -> LDS
// bytes per MFMA flop are ~ 1 / BM for the weights and ~ 1 / (k BN) for the window.  At 128 x 192 the two
// co-resident workgroups of a CU fetch ~32 B/cycle at full MFMA rate on the k = 7 / 11 / 9 shapes, the per-CU
// L2 -> LDS rate measured in MI355X_MICROARCH.md ("Indexed rows"), which is what the DMA ablation shows; 256 x 96
// halves the weight bytes (and doubles the window bytes, amortised over k taps).
constexpr int W2_HALO = 64;  // max (k - 1) * dil

// BM = 160 (waves 2 x 2 of 80 x 96, TM = 5): sequences of T = 312 rows as two tiles (320 rows) instead of three of 128
// (384 rows, 768 tiles on the 512 workgroup slots of the chip: the VAE's k3 convs)
template <int PREC, bool GEGLU, int BM = 128, int BN = 192>
__global__ __launch_bounds__(256, 2) void wconv2_kernel(const WConvDev P) {
  constexpr int WGM = BM == 256 ? 4 : 2, WGN = 4 / WGM;  // wave grid
  constexpr int TM = BM / WGM / 16, TN = 6;
  constexpr int WR_ROWS = TM * 16;                        // rows per wave
  static_assert(WGM * WGN == 4 && WGN * TN * 16 == BN && WGM * WR_ROWS == BM, "4 waves of (16 TM) x 96");
  constexpr int WROWS = BM + W2_HALO;
  constexpr int WBUF = WROWS * 128;      // window image
  constexpr int BBUF = BN * 128;         // weight image
  constexpr int SMEM = WBUF + 2 * BBUF;  // 72 KB (128 x 192) / 64 KB (256 x 96) / 76 KB (160 x 192)
  constexpr int WPW = WROWS / 8 / 4;     // window DMA instructions per wave (6 / 10 / 7)
  static_assert(WROWS % 32 == 0, "whole window DMA instructions per wave");
  constexpr int BPW = BN / 8 / 4;        // weight DMA instructions per wave per step (6 / 3)
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int orig = blockIdx.x;
  // K split (P.ksplit > 1, plain fp32 epilogue only): work item = (K part, tile), part-major; the part writes its raw
  // sums to its fp32 slice of P.part and ksplit_reduce_kernel applies the epilogue
  const int KS = P.ksplit > 1 ? P.ksplit : 1;
  const int items = P.nwg * KS;
  const int xcd = orig & 7, q = items >> 3, r8 = items & 7;
  int wid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int kp = wid / P.nwg;
  wid -= kp * P.nwg;
  int mt, nt;
  if (P.n_major) {
    const int tiles_m = P.nwg / P.tiles_n;
    nt = wid / tiles_m;
    mt = wid - nt * tiles_m;
  } else {
    mt = wid / P.tiles_n;
    nt = wid - mt * P.tiles_n;
  }
  const int b = mt / P.tiles_per_batch;
  const int t0 = (mt - b * P.tiles_per_batch) * BM;
  const int col0 = nt * BN;
  const int K = P.ksize, Cp = P.Cp;
  const int WR = BM + (K - 1) * P.dil;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const int nC = Cp / 64 / KS, cbase = kp * nC;  // this item's 64-channel chunks
    const int steps = nC * K;
    const u16* wsrc[WPW];
    int wstep[WPW];
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int row = 8 * (wave + 4 * j) + (lane >> 3);
      const int ls = (lane & 7) ^ (row & 7);
      const int ts = t0 - P.pad + row;
      const bool ok = row < WR && ts >= 0 && ts < P.T;
      wsrc[j] = ok ? P.a + ((int64_t)b * P.T + ts) * Cp + cbase * 64 + ls * 8 : reinterpret_cast<const u16*>(g_wconv_zero);
      wstep[j] = ok ? 64 : 0;
    }
    const u16* bsrc[BPW];
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int n = 8 * (wave + 4 * j) + (lane >> 3);
      const int ls = (lane & 7) ^ (n & 7);
      bsrc[j] = P.w + (int64_t)min(col0 + n, P.N - 1) * P.kpad + ls * 8;  // (a partial last N tile: rows clamped,
                                                                          // their columns never stored)
    }
    auto stage_w = [&](int c) {
#pragma unroll
      for (int j = 0; j < WPW; ++j) glds16(wsrc[j] + c * wstep[j], smem + (wave + 4 * j) * 1024);
    };
    auto stage_b = [&](int st, int buf) {
      const int c = st / K, tap = st - c * K;
      const int off = tap * Cp + (cbase + c) * 64;
#pragma unroll
      for (int j = 0; j < BPW; ++j) glds16(bsrc[j] + off, smem + WBUF + buf * BBUF + (wave + 4 * j) * 1024);
    };

    const int arow0 = wm * WR_ROWS + (lane & 15);
    const int nrow0 = wn * 96 + (lane & 15);
    const int bsw = lane & 7;

    stage_w(0);
    stage_b(0, 0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    {
      // fragment-pipelined K loop: the second 32-deep slice's fragments are read
      // while the first slice's MFMAs run (B fragments as their last use retires, A fragments after each row),
      // and the next step's A fragments (same chunk: the window is resident) during the second slice, so after
      // each step's barrier only the 6 weight-fragment reads of the new step are exposed, not 10 reads per slice
      auto rdA = [&](int tap, int sub, int i) -> bf16x8 {
        const int arow = arow0 + tap * P.dil;
        return *reinterpret_cast<const bf16x8*>(smem + arow * 128 + (((4 * sub + (lane >> 4)) ^ (arow & 7)) << 4) +
                                                i * 16 * 128);
      };
      auto rdB = [&](const char* Bl, int sub, int j) -> bf16x8 {
        return *reinterpret_cast<const bf16x8*>(Bl + nrow0 * 128 + (((4 * sub + (lane >> 4)) ^ bsw) << 4) +
                                                j * 16 * 128);
      };
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = rdA(0, 0, i);
      int st = 0;
      for (int c = 0; c < nC; ++c) {
        for (int tap = 0; tap < K; ++tap, ++st) {
          if (st + 1 < steps) stage_b(st + 1, (st + 1) & 1);
          const char* Bl = smem + WBUF + (st & 1) * BBUF;
#pragma unroll
          for (int j = 0; j < TN; ++j) bfr[j] = rdB(Bl, 0, j);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[i][j] = mfma16<PREC>(af[i], bfr[j], acc[i][j]);
              if (i == TM - 1) bfr[j] = rdB(Bl, 1, j);
            }
            af[i] = rdA(tap, 1, i);
          }
          // the next step's A fragments: tap + 1 of this chunk (at the chunk's last tap a harmless re-read of this
          // window, replaced after the re-stage below)
          const int ntap = tap + 1 < K ? tap + 1 : tap;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<PREC>(af[i], bfr[j], acc[i][j]);
            af[i] = rdA(ntap, 0, i);
          }
          // pin that interleave (hipcc otherwise sinks the reads behind the slice's MFMAs to save registers):
          // masks MFMA = 0x8, DS_READ = 0x100
#pragma unroll
          for (int i = 0; i < TM - 1; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_s_setprio(0);
          if (tap == K - 1 && c + 1 < nC) {
            // every wave has finished reading window c: re-stage it with chunk c + 1
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            stage_w(c + 1);
          }
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
          if (tap == K - 1) {
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = rdA(0, 0, i);
          }
        }
      }
    }
  }

  // epilogue: one wave row's slice of the tile (64 or 80 rows) at a time through LDS (the K loop's last barrier retired
  // every fragment read and DMA), whole row segments (768 / 384 B) with 16-B loads / stores
  constexpr int OTS = BN + 4;
  static_assert(WR_ROWS * OTS * 4 <= SMEM, "staged slice");
  float* ot = reinterpret_cast<float*>(smem);
  constexpr int cq = BN / 4;
  constexpr int PER = WR_ROWS * cq / 256;  // float4 per thread per slice (12 / 6 / 15)
  static_assert(WR_ROWS * cq % 256 == 0, "whole float4 passes");
  // GEGLU: this thread's bias columns (the same in every slice), loaded once up front: loaded next to each store they
  // made every store-load pair a vmcnt(0) round trip (24 serialised per tile)
  float4 gbv[GEGLU ? PER : 1];
  if constexpr (GEGLU) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = tid + e * 256;
      const int n = (idx - (idx / cq) * cq) * 4;
      gbv[e] = P.bias ? *reinterpret_cast<const float4*>(P.bias + col0 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  for (int h = 0; h < WGM; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            ot[(i * 16 + (lane >> 4) * 4 + r) * OTS + wn * 96 + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    const int r0 = t0 + h * WR_ROWS;
    if constexpr (GEGLU) {
      const int No = P.N / 2;
      for (int e = 0; e < PER; ++e) {
        const int idx = tid + e * 256;
        const int m = idx / cq, n = (idx - m * cq) * 4;
        if (r0 + m >= P.T) continue;
        float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
        v.x += gbv[e].x; v.y += gbv[e].y; v.z += gbv[e].z; v.w += gbv[e].w;
        f32x2 y;
        y.x = v.x * alcm_act(v.y, ACT_GELU_ERF);
        y.y = v.z * alcm_act(v.w, ACT_GELU_ERF);
        op_store2<PREC>(P.gplane + ((int64_t)b * P.T + r0 + m) * No + (col0 + n) / 2, 0, y);
      }
    } else {
      // (K split: this part's raw sums into its slice — no bias / residual / activation / scale / accumulate)
      const bool split = KS > 1;
      float* const outp = split ? P.part + (int64_t)kp * ((int64_t)(P.nwg / P.tiles_n / P.tiles_per_batch) * P.orows * P.N)
                                : P.out;
      const float* const resp = split ? nullptr : P.res;
      const float* const biasp = split ? nullptr : P.bias;
      const int accum = split ? 0 : P.accumulate, oact = split ? 0 : P.out_act;
      const float oscale = split ? 1.f : P.out_scale;
      // passes of PH loads (residual, accumulate, bias): the other halves' accumulators are still live in half 0
      constexpr int PH = PER % 4 == 0 ? (BN == 192 ? PER / 4 : PER / 2) : PER / 5;
      static_assert(PER % PH == 0, "load passes");
#pragma unroll
      for (int e0 = 0; e0 < PER; e0 += PH) {
      float4 rv[PH], pv[PH], bv[PH];  // (bias with them: loaded next to each store it cost a vmcnt(0) per store)
#pragma unroll
      for (int e = 0; e < PH; ++e) {
        const int idx = tid + (e0 + e) * 256;
        const int m = idx / cq, n = (idx - m * cq) * 4;
        const int t = min(r0 + m, P.T - 1);
        const int64_t go = ((int64_t)b * P.orows + (int64_t)t * P.ostride + P.ooff) * P.N + min(col0 + n, P.N - 4);
        rv[e] = resp ? *reinterpret_cast<const float4*>(resp + go) : make_float4(0.f, 0.f, 0.f, 0.f);
        pv[e] = accum ? *reinterpret_cast<const float4*>(outp + go) : make_float4(0.f, 0.f, 0.f, 0.f);
        bv[e] = biasp ? *reinterpret_cast<const float4*>(biasp + min(col0 + n, P.N - 4))
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int e = 0; e < PH; ++e) {
        const int idx = tid + (e0 + e) * 256;
        const int m = idx / cq, n = (idx - m * cq) * 4;
        if (r0 + m >= P.T || col0 + n >= P.N) continue;
        const int64_t go = ((int64_t)b * P.orows + (int64_t)(r0 + m) * P.ostride + P.ooff) * P.N + col0 + n;
        float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
        v.x += bv[e].x; v.y += bv[e].y; v.z += bv[e].z; v.w += bv[e].w;
        if (P.oplane) {  // plane output (no residual / accumulate / act): 4 rounded values, one 8-B store; the
          // residual-free + 0.f turns -0 into +0 exactly as the fp32 route's (v + 0) * 1 + 0 does
          v.x += 0.f; v.y += 0.f; v.z += 0.f; v.w += 0.f;
          op_store2<PREC>(P.oplane + go, 0, f32x2{v.x, v.y});
          op_store2<PREC>(P.oplane + go + 2, 0, f32x2{v.z, v.w});
          continue;
        }
        if (oact) {  // (opconv's order: act(acc + bias), then residual / scale / accumulate)
          v.x = alcm_act(v.x, oact); v.y = alcm_act(v.y, oact);
          v.z = alcm_act(v.z, oact); v.w = alcm_act(v.w, oact);
        }
        v.x = (v.x + rv[e].x) * oscale + pv[e].x;
        v.y = (v.y + rv[e].y) * oscale + pv[e].y;
        v.z = (v.z + rv[e].z) * oscale + pv[e].z;
        v.w = (v.w + rv[e].w) * oscale + pv[e].w;
        *reinterpret_cast<float4*>(outp + go) = v;
      }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------------
// Persistent 8-wave wide conv (ALCM_WCONV3): one 512-thread workgroup per CU walks its tiles of 256 rows x 192
// columns as ONE flat sequence of (tile, 64-channel chunk, tap) steps, so the staging pipeline never drains at a
// tile boundary.  Waves 4 (M) x 2 (N), each 64 x 96 of 16x16x32 MFMAs (24 per 32-deep slice, two slices a step).
//   * LDS (152 KB): input windows (256 + (k-1)d <= 320 rows x 128 B) double-buffered, weight tiles (192 x 128 B) in
//     a 3-slot ring.  Images lane-linear with the 16-B slot swizzle s ^ (r & 7) (conflict-free ds_read_b128).
//   * ONE barrier per step, in its middle (after the first slice's MFMAs are issued), behind a COUNTED vmcnt wait
//     for the next step's weight tile (and, at a chunk's last step, the next chunk's window): every fragment the
//     second slice and the next step's first slice read is then resident, so all fragment reads are issued a whole
//     slice (24 MFMAs) ahead of their use — B fragments double-buffered in registers, A fragments replaced row by
//     row as their last MFMA issues.  Right after that barrier the slot and window this step has finished reading
//     are refilled: weight step g + 3 (2.5 steps of DMA latency hidden), and at a chunk's last step the window two
//     chunks ahead (for a tile's last chunks: the next tile's).
//   * the epilogue of a tile runs straight from the accumulators (no LDS, no barrier) while the next tile's first
//     window and weight steps are already in flight;
//   * per-CU L2 -> LDS bytes per MFMA flop: weights 1/256, window 1/(192 k): at k = 11 / 3, 18 / 24 B per cycle at
//     the full MFMA rate, under the ~29 B/cycle a CU gathers from its L2 (MI355X_MICROARCH.md, "Indexed rows"),
//     where the two-workgroup 256 x 96 / 128 x 192 tiles need 20-41.
// Persistent order: XCD x owns the tile range [x R, (x+1) R) (R = ceil(tiles / 8)), its workgroups take every
// (grid / 8)-th tile of it, N-major (concurrent tiles share a weight slice in the XCD's L2) or M-major.
constexpr int W3_BM = 256, W3_BN = 192, W3_WROWS = 320;
constexpr int W3_WBUF = W3_WROWS * 128;  // 40 KB
constexpr int W3_BBUF = W3_BN * 128;     // 24 KB
constexpr int W3_WPW = W3_WROWS / 8 / 8;  // window DMA instructions per wave (5)
constexpr int W3_BPW = W3_BN / 8 / 8;     // weight DMA instructions per wave per step (3)

// s_waitcnt vmcnt(N) lgkmcnt(0) through the builtin (the compiler's wait insertion sees it and does not re-wait for
// LDS reads it already retired), then the barrier
template <int N>
__device__ __forceinline__ void w3_wait_barrier() {
  static_assert(N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));
  __builtin_amdgcn_s_barrier();
}
template <typename V>
__device__ __forceinline__ V w3_sel(const V (&v)[3], int i) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]);
}
// KSP: the K-split form (P.ksplit parts) is compiled in (its own instantiation, so profiles tell the two apart)
template <int PREC, int SEG, bool KSP>
__global__ __launch_bounds__(512, 1) void wconv3_kernel(const WConvDev P) {
  constexpr int TM = 4, TN = 6;
  __shared__ __attribute__((aligned(1024))) char smem[2 * W3_WBUF + 3 * W3_BBUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  // work items: tiles, or (K split) (part, tile) pairs part-major, so an XCD's contiguous item range walks the
  // tiles of one part as the unsplit kernel walks its tiles
  const int KS = KSP && P.ksplit > 1 ? P.ksplit : 1;
  const int ntiles = P.nwg;
  const int nitems = ntiles * KS;
  const int R = (nitems + 7) >> 3;
  const int tbeg = xcd * R, tend = min(tbeg + R, nitems);
  const int first = tbeg + slot;
  const int my_n = first < tend ? (tend - first + nslot - 1) / nslot : 0;
  if (my_n == 0) return;
  const int Cp = P.Cp, nC = Cp / 64 / KS;  // 64-channel chunks per item and term
  // SEG > 1: a tile's chunks are the terms' chunks in order (term s: chunks s nC .. s nC + nC - 1, P.sk[s] taps each)
  const int NCH = SEG * nC;
  const int total = my_n * nC * (SEG == 1 ? P.ksize : P.sk[0] + P.sk[1] + (SEG > 2 ? P.sk[2] : 0));  // steps
  const int nchunks = my_n * NCH;  // windows
  const int tiles_m = ntiles / P.tiles_n;
  auto tile_of = [&](int ti, int& b, int& t0, int& col0, int& kp) {
    int tile = first + ti * nslot;
    kp = tile / ntiles;  // K part (0 unless split)
    tile -= kp * ntiles;
    int mt, nt;
    if (P.n_major) {
      nt = tile / tiles_m;
      mt = tile - nt * tiles_m;
    } else {
      mt = tile / P.tiles_n;
      nt = tile - mt * P.tiles_n;
    }
    b = mt / P.tiles_per_batch;
    t0 = (mt - b * P.tiles_per_batch) * W3_BM;
    col0 = nt * W3_BN;
  };
  // window of global chunk q (tile q / nC, channel chunk q % nC) -> buffer q & 1, as W3_WPW DMA instructions (each
  // 8 rows x 128 B per wave); win_setup resolves the chunk once, win_piece issues instruction j
  const u16* wsrc_base = P.a;  // batch b, channel chunk c
  int wrow0 = 0;               // first window row's time index (t0 - pad)
  int wbuf = 0;
  int WR = W3_BM + (P.ksize - 1) * P.dil;  // window rows of the chunk being staged
  auto win_setup = [&](int q) {
    const int ti = q / NCH;
    int c = q - ti * NCH;
    int b, t0, col0, kp;
    tile_of(ti, b, t0, col0, kp);
    if constexpr (SEG == 1) {
      wsrc_base = P.a + (int64_t)b * P.T * Cp + (kp * nC + c) * 64;
      wrow0 = t0 - P.pad;
    } else {
      const int sg = c / nC;
      c -= sg * nC;
      wsrc_base = w3_sel(P.sa, sg) + (int64_t)b * P.T * Cp + c * 64;
      wrow0 = t0 - w3_sel(P.spad, sg);
      WR = W3_BM + w3_sel(P.sk, sg) - 1;
    }
    wbuf = q & 1;
  };
  auto win_piece = [&](int j) {
    const int row = 8 * (wave + 8 * j) + (lane >> 3);
    const int ls = (lane & 7) ^ (row & 7);
    const int ts = wrow0 + row;
    const bool ok = row < WR && ts >= 0 && ts < P.T;
    const u16* src = ok ? wsrc_base + (int64_t)ts * Cp + ls * 8 : reinterpret_cast<const u16*>(g_wconv_zero);
    glds16(src, smem + wbuf * W3_WBUF + (wave + 8 * j) * 1024);
  };
  auto stage_win = [&](int q) {
    win_setup(q);
#pragma unroll
    for (int j = 0; j < W3_WPW; ++j) win_piece(j);
  };
  // the next chunk's window is spread over the current chunk's first K - 2 steps (piece j at tap j % (K - 2)), so
  // the whole grid's window stream (40 KB per CU per chunk) does not land as one burst that queues the weight DMA
  // behind it (a burst every 11 steps cost 12 % in scripts/probes/mfma_lds_probe.hip); issued no later than tap
  // K - 3, every piece is covered by the counted wait at the chunk's last mid-step (a burst at the chunk's first
  // step measured equal within 2 %)
  int K = SEG == 1 ? P.ksize : P.sk[0];  // taps of the chunk being computed
  int wspread = K - 2;

  // weight DMA: per-lane 32-bit byte offsets (row n * kpad + 16-B piece) from a workgroup-uniform base, so each
  // instruction is a saddr + voffset access with no per-step 64-bit address arithmetic; instruction j covers rows
  // 8 (wave + 8 j) .. + 7
  uint32_t boff[W3_BPW];
  auto set_boff = [&](int kpad) {
#pragma unroll
    for (int j = 0; j < W3_BPW; ++j) {
      const int n = 8 * (wave + 8 * j) + (lane >> 3);
      boff[j] = (uint32_t)(n * kpad + ((lane & 7) ^ (n & 7)) * 8) * 2u;
    }
  };
  set_boff(SEG == 1 ? P.kpad : P.skpad[0]);
  // issue cursor: weight step ig = (tile iti, chunk ic, tap itap) at element offset iwoff of the weight plane; past
  // the last step it stays on the last tile (the ring slot it refills is never read again)
  int ig = 0, ic = 0, itap = 0, iti = 0;
  int64_t iwoff;
  int icol0;                                           // the issue tile's first column
  int iK = SEG == 1 ? P.ksize : P.sk[0];               // the issue step's term: taps, weight plane
  const u16* iw = SEG == 1 ? P.w : P.sw[0];
  {
    int b_, t0_, kp_;
    tile_of(0, b_, t0_, icol0, kp_);
    iwoff = (int64_t)icol0 * (SEG == 1 ? P.kpad : P.skpad[0]) + kp_ * nC * 64;
  }
  auto issue_wt = [&](int sl) {
    const char* base = reinterpret_cast<const char*>(iw + iwoff);
#pragma unroll
    for (int j = 0; j < W3_BPW; ++j) glds16(base + boff[j], smem + 2 * W3_WBUF + sl * W3_BBUF + (wave + 8 * j) * 1024);
  };
  auto advance_wt = [&]() {
    if (++ig >= total) return;
    iwoff += Cp;
    if (++itap == iK) {
      itap = 0;
      iwoff += 64 - (int64_t)iK * Cp;
      if (++ic == NCH) {
        ic = 0;
        int b_, t0_, kp_;
        tile_of(++iti, b_, t0_, icol0, kp_);
        if constexpr (SEG == 1) {
          iwoff = (int64_t)icol0 * P.kpad + kp_ * nC * 64;
        } else {
          iK = P.sk[0];
          iw = P.sw[0];
          set_boff(P.skpad[0]);
          iwoff = (int64_t)icol0 * P.skpad[0];
        }
      } else if (SEG > 1 && ic % nC == 0) {  // the next term's first chunk
        const int sg = ic / nC;
        iK = w3_sel(P.sk, sg);
        iw = w3_sel(P.sw, sg);
        const int kp = w3_sel(P.skpad, sg);
        set_boff(kp);
        iwoff = (int64_t)icol0 * kp;
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow0 = wm * 64 + (lane & 15);
  const int nrow0 = wn * 96 + (lane & 15);
  const int bsw = lane & 7;
  auto rdA = [&](int buf, int tp, int sub, int i) -> bf16x8 {
    const int arow = arow0 + tp * P.dil;
    return *reinterpret_cast<const bf16x8*>(smem + buf * W3_WBUF + arow * 128 +
                                            (((4 * sub + (lane >> 4)) ^ (arow & 7)) << 4) + i * 16 * 128);
  };
  auto rdB = [&](int sl, int sub, int j) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + 2 * W3_WBUF + sl * W3_BBUF + nrow0 * 128 +
                                            (((4 * sub + (lane >> 4)) ^ bsw) << 4) + j * 16 * 128);
  };

  // tile epilogue, straight from the accumulators: fp32 out = (acc + bias + res) * scale (+ out), or (oplane) the
  // operand plane of acc + bias in the format of PREC (the AMPBlock conv1 whose only consumer, the next Activation1d,
  // rounds its input to that format: the same rounding of the same fp32 value, half the bytes on both sides)
  auto epilogue = [&](int ti) {
    int b, t0, col0, kp;
    tile_of(ti, b, t0, col0, kp);
    // K split: this part's raw sums into its partial slice (bias / residual / scale / accumulate in the reduction)
    const bool split = KS > 1;
    float* const outp = split ? P.part + (int64_t)kp * ((int64_t)(P.nwg / P.tiles_n / P.tiles_per_batch) * P.T * P.N)
                              : P.out;
    const float* const resp = split ? nullptr : P.res;
    const bool accum = !split && P.accumulate;
    const float oscale = split ? 1.f : P.out_scale;
    float bv[TN];
    if constexpr (SEG > 1) {
      // sum form: (acc + (b_0 + b_1 + b_2) + ((r_0 + r_1) + r_2)) * scale (+ out)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + wn * 96 + j * 16 + (lane & 15);
        float v = 0.f;
#pragma unroll
        for (int sg = 0; sg < SEG; ++sg) v += P.sbias[sg] ? P.sbias[sg][col] : 0.f;
        bv[j] = v;
      }
      if (P.oplane) {
        // the stage output as the next stage's operand plane (its only consumer, the upsampler, reads that format):
        // fp16 / bf16 of the fp32 value the fp32 route stores ((acc + b + r) * scale + 0), column pairs by DPP
        const bool odd = lane & 1;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) {
            const int r = 2 * rp + (odd ? 1 : 0);
            const int t = t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
            const int64_t rb = ((int64_t)b * P.T + min(t, P.T - 1)) * P.N + col0 + wn * 96;
            float rv[2][TN];
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // rows 2 rp (h = 0) and 2 rp + 1 of this lane's column
              const int64_t ro = ((int64_t)b * P.T + min(t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + 2 * rp + h,
                                                         P.T - 1)) * P.N + col0 + wn * 96 + (lane & 15);
#pragma unroll
              for (int j = 0; j < TN; ++j) {
                float v = P.sres[0] ? P.sres[0][ro + j * 16] : 0.f;
#pragma unroll
                for (int sg = 1; sg < SEG; ++sg) v += P.sres[sg] ? P.sres[sg][ro + j * 16] : 0.f;
                rv[h][j] = v;
              }
            }
            u16* const rowp = P.oplane + rb + (lane & 14);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const float v0 = (acc[i][j][2 * rp] + bv[j] + rv[0][j]) * oscale + 0.f;
              const float v1 = (acc[i][j][2 * rp + 1] + bv[j] + rv[1][j]) * oscale + 0.f;
              const float send = odd ? v0 : v1;
              const float recv = __builtin_bit_cast(
                  float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, true));
              const float lo = odd ? recv : v0, hi = odd ? v1 : recv;
              if (t < P.T) op_store2<PREC>(rowp + j * 16, 0, f32x2{lo, hi});
            }
          }
        return;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int rh = 0; rh < 4; rh += 2) {  // row pairs: 3 residual reads per output
          float rv[2][TN], pv[2][TN];
          int orow[2];
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int t = t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + rh + r;
            orow[r] = t < P.T ? b * P.T + t : -1;
            const int64_t ro = (int64_t)max(orow[r], 0) * P.N + col0 + wn * 96 + (lane & 15);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              float v = P.sres[0] ? P.sres[0][ro + j * 16] : 0.f;
#pragma unroll
              for (int sg = 1; sg < SEG; ++sg) v += P.sres[sg] ? P.sres[sg][ro + j * 16] : 0.f;
              rv[r][j] = v;
              pv[r][j] = accum ? outp[ro + j * 16] : 0.f;
            }
          }
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            if (orow[r] < 0) continue;
            const int64_t ro = (int64_t)orow[r] * P.N + col0 + wn * 96 + (lane & 15);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              outp[ro + j * 16] = (acc[i][j][rh + r] + bv[j] + rv[r][j]) * oscale + pv[r][j];
          }
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[j] = (P.bias && !split) ? P.bias[col0 + wn * 96 + j * 16 + (lane & 15)] : 0.f;
    if (P.oplane) {
      // column pairs through a lane-pair exchange (DPP quad_perm [1, 0, 3, 2]): per accumulator row pair (r0, r1) the
      // even lane of a pair stores row r0, columns (c, c + 1), the odd lane row r1, columns (c - 1, c): 4-B stores
      const bool odd = lane & 1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          const int r = 2 * rp + (odd ? 1 : 0);
          const int t = t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          u16* const rowp = P.oplane + ((int64_t)b * P.T + min(t, P.T - 1)) * P.N + col0 + wn * 96 + (lane & 14);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            // (+ 0.f: the fp32 epilogue's value, acc + bias + a zero residual, signed zeros included)
            const float v0 = acc[i][j][2 * rp] + bv[j] + 0.f, v1 = acc[i][j][2 * rp + 1] + bv[j] + 0.f;
            const float send = odd ? v0 : v1;
            const float recv = __builtin_bit_cast(
                float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, true));
            const float lo = odd ? recv : v0, hi = odd ? v1 : recv;
            if (t < P.T) op_store2<PREC>(rowp + j * 16, 0, f32x2{lo, hi});
          }
        }
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float rv[4][TN], pv[4][TN];
      int orow[4];  // output row (b T + t) of each accumulator row, -1 where nothing is stored
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        orow[r] = t < P.T ? b * P.T + t : -1;
        const int64_t ro = (int64_t)max(orow[r], 0) * P.N + col0 + wn * 96 + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          rv[r][j] = resp ? resp[ro + j * 16] : 0.f;
          pv[r][j] = accum ? outp[ro + j * 16] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (orow[r] < 0) continue;
        const int64_t ro = (int64_t)orow[r] * P.N + col0 + wn * 96 + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          outp[ro + j * 16] = (acc[i][j][r] + bv[j] + rv[r][j]) * oscale + pv[r][j];
      }
    }
  };

  // prologue: window 0, weights 0, 1, 2 (window 1 is issued in pieces during chunk 0)
  stage_win(0);
  issue_wt(0);
  advance_wt();
  issue_wt(1);
  advance_wt();
  issue_wt(2);
  advance_wt();
  w3_wait_barrier<2 * W3_BPW>();
  int pieces_last = 0;  // window pieces issued at the previous mid-step (they may stay in flight)

  bf16x8 aA[TM], aB[TM], bA[TN], bB[TN];  // slice-0 / slice-1 fragments
#pragma unroll
  for (int i = 0; i < TM; ++i) aA[i] = rdA(0, 0, 0, i);
#pragma unroll
  for (int j = 0; j < TN; ++j) bA[j] = rdB(0, 0, j);

  int ti = 0, c = 0, tap = 0, sl = 0, q = 0;  // q: global chunk (window buffer q & 1)
  // ---- mid-step: weight step g + 1 (and at a chunk's last step the next chunk's window) resident in every wave's
  //      share; every wave done reading this slot and, at a chunk's last step, this chunk's window.  Loads issued after
  //      weight step g + 1 (weight step g + 2, and the window issued at the previous mid-step) stay in flight
  auto mid_step = [&]() {
    switch (pieces_last) {
      case 0: w3_wait_barrier<W3_BPW>(); break;
      case 1: w3_wait_barrier<W3_BPW + 1>(); break;
      case 2: w3_wait_barrier<W3_BPW + 2>(); break;
      default: w3_wait_barrier<W3_BPW + W3_WPW>(); break;
    }
    pieces_last = 0;
    if (tap < wspread && tap < W3_WPW && q + 1 < nchunks) {
      if (tap == 0) win_setup(q + 1);
      for (int j = tap; j < W3_WPW; j += wspread) {
        win_piece(j);
        ++pieces_last;
      }
    }
  };
  for (int g = 0; g < total; ++g) {
    const bool chunk_end = tap == K - 1;
    const int sl1 = sl == 2 ? 0 : sl + 1;
    const int nbuf = chunk_end ? (q + 1) & 1 : q & 1;
    const int ntap = chunk_end ? 0 : tap + 1;
    // ---- slice 0: MFMAs on (aA, bA); slice 1's fragments (this slot, this window) read under them
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<PREC>(aA[i], bA[j], acc[i][j]);
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bB[j] = rdB(sl, 1, j);
#pragma unroll
        for (int ii = 0; ii < TM; ++ii) aB[ii] = rdA(q & 1, tap, 1, ii);
      }
    }
    // pin the interleave: all ten reads of the next slice's fragments after the first row's MFMAs, so the newest
    // is 18 MFMAs old when the next slice starts (the compiler's wait there is lgkmcnt(0)); issued before the first
    // row they would leave 16 LDS reads outstanding, past lgkmcnt's 4-bit range
    __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TN + TM, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, (TM - 1) * TN, 0);
    __builtin_amdgcn_s_setprio(0);

    mid_step();
    // ---- slice 1: MFMAs on (aB, bB); the next step's slice-0 fragments read under them
    // (after the last step these re-read resident LDS: harmless)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<PREC>(aB[i], bB[j], acc[i][j]);
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bA[j] = rdB(sl1, 0, j);
#pragma unroll
        for (int ii = 0; ii < TM; ++ii) aA[ii] = rdA(nbuf, ntap, 0, ii);
        // weight step g + 3 into the slot this step has finished reading (every wave passed the mid-step barrier)
        issue_wt(sl);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TN + TM, 0);
    __builtin_amdgcn_sched_group_barrier(0x10, W3_BPW, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, (TM - 1) * TN, 0);
    __builtin_amdgcn_s_setprio(0);
    advance_wt();

    sl = sl1;
    if (!chunk_end) {
      ++tap;
      continue;
    }
    tap = 0;
    ++q;
    if (++c == NCH) {
      epilogue(ti);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c = 0;
      ++ti;
    }
    if constexpr (SEG > 1) {  // the next chunk's term
      K = w3_sel(P.sk, c / nC);
      wspread = K - 2;
    }
  }
}

static int g_ncu = 0;

// K-split reduction of wconv3's partial slices: out = (sum over parts, in part order, + bias + res) * scale (+ out) —
// the unsplit epilogue's expression with its accumulator replaced by the ordered part sum, so a launch is
// deterministic (bit-stable run to run); float4 per lane over the B T N / 4 outputs (N % 4 == 0)
__global__ __launch_bounds__(256) void ksplit_reduce_kernel(const float4* __restrict__ part, int ks, int64_t n4, int N4,
                                                            const float4* __restrict__ bias, const float4* res,
                                                            float4* out, float scale, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = part[i];
    for (int p = 1; p < ks; ++p) {
      const float4 v = part[(int64_t)p * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    const float4 bv = bias ? bias[i % N4] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 rv = res ? res[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 pv = accumulate ? out[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 o;
    o.x = (a.x + bv.x + rv.x) * scale + pv.x;
    o.y = (a.y + bv.y + rv.y) * scale + pv.y;
    o.z = (a.z + bv.z + rv.z) * scale + pv.z;
    o.w = (a.w + bv.w + rv.w) * scale + pv.w;
    out[i] = o;
  }
}

// the reduction launch of a K-split conv (same stream, right after the parts)
static void ksplit_reduce(const alcm_opconv_args& a, int ks, hipStream_t s) {
  const int64_t n4 = (int64_t)a.B * a.T * a.N / 4;
  const unsigned rg = (unsigned)std::min<int64_t>((n4 + 255) / 256, (int64_t)g_ncu * 8);
  hipLaunchKernelGGL(ksplit_reduce_kernel, dim3(rg), dim3(256), 0, s, reinterpret_cast<const float4*>(a.ksplit_ws), ks,
                     n4, a.N / 4, reinterpret_cast<const float4*>(a.bias), reinterpret_cast<const float4*>(a.res),
                     reinterpret_cast<float4*>(a.out), a.out_scale, a.accumulate);
}

// K parts for wconv3 on a grid that does not fill the chip (items = tiles x parts): the smallest part count that
// minimises rounds-of-items per part (e.g. the DiT FFN down-projection: 192 tiles of 256 x 192 on 256 CUs, 0.75 busy;
// 4 parts = 768 items = 3 per CU, 0.75 of the time plus the reduction), within the caller's partial workspace; 1 =
// no split
static int wconv3_parts(const alcm_opconv_args& a, int64_t tiles, int ncu) {
  if (!a.ksplit_ws || knobs().ksplit == 0 || a.out_plane || a.Cp % 64) return 1;
  const int nc = a.Cp / 64;
  int ks = 1;
  double best = (double)((tiles + ncu - 1) / ncu);
  for (int k = 2; k <= 8; ++k) {
    if (nc % k || nc / k < 4 || (double)k * a.B * a.T * a.N > (double)a.ksplit_ws_floats) continue;
    const double t = (double)((tiles * k + ncu - 1) / ncu) / k;
    if (t < best * 0.95) {
      best = t;
      ks = k;
    }
  }
  return ks;
}

// Eligible: fp16 / bf16 operands, Cp % 64 == 0, 3 <= k, (k-1) d <= 64, N % 192 == 0, plain fp32 epilogue (bias,
// residual, scale, accumulate; no GEGLU / strided output).  Returns 1 when it launched.
static int wconv3_try(const alcm_opconv_args& a, const u16* wplane, double flops, double bytes, hipStream_t s,
                      int ks = 1) {
  if (a.prec != PREC_F16 && a.prec != PREC_BF16) return 0;
  if (a.out_act || a.out_stride > 0 || a.geglu_plane || a.Cp % 64 || a.ksize < 3 || (a.ksize - 1) * a.dil > 64 ||
      a.N % W3_BN)
    return 0;
  if (a.out_plane ? (a.out || a.res || a.accumulate || (((uintptr_t)a.out_plane) & 3)) : !a.out) return 0;
  if (!g_ncu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                hipSuccess && n >= 8)
      g_ncu = n;
    else
      g_ncu = 256;
  }
  WConvDev P{};
  P.a = (const u16*)a.a;
  P.T = a.T; P.Cp = a.Cp; P.ksize = a.ksize; P.dil = a.dil; P.pad = a.pad;
  P.w = wplane; P.kpad = a.kpad; P.N = a.N;
  P.bias = a.bias; P.res = a.res; P.out = a.out; P.out_scale = a.out_scale; P.accumulate = a.accumulate;
  P.oplane = (u16*)a.out_plane;
  P.tiles_per_batch = (P.T + W3_BM - 1) / W3_BM;
  P.tiles_n = a.N / W3_BN;
  const int64_t nt = (int64_t)a.B * P.tiles_per_batch * P.tiles_n;
  if (nt >= (1ll << 30) || (int64_t)a.B * a.T * a.Cp >= (1ll << 40) || (int64_t)a.B * a.T * a.N >= (1ll << 40)) return 0;
  if ((int64_t)W3_BN * a.kpad * 2 >= (1ll << 31)) return 0;  // per-lane 32-bit weight-row byte offsets
  P.nwg = (int)nt;
  P.n_major = 1;
  if (ks > 1) {
    if (a.out_plane || (a.Cp / 64) % ks || (int64_t)a.N % 4 || (((uintptr_t)a.ksplit_ws) & 15) ||
        (a.bias && (((uintptr_t)a.bias) & 15)) || (a.res && (((uintptr_t)a.res) & 15)) || (((uintptr_t)a.out) & 15))
      return 0;
    P.ksplit = ks;
    P.part = a.ksplit_ws;
  }
  const int R = (int)((nt * ks + 7) / 8);
  int grid = 8 * std::min(g_ncu / 8, R);
  if (knobs().wconv3_grid >= 8) grid = std::min(grid, knobs().wconv3_grid / 8 * 8);  // tests: several tiles per workgroup
  void* tok = prof_start(s);
  if (a.prec == PREC_F16) {
    if (ks > 1) hipLaunchKernelGGL((wconv3_kernel<PREC_F16, 1, true>), dim3(grid), dim3(512), 0, s, P);
    else hipLaunchKernelGGL((wconv3_kernel<PREC_F16, 1, false>), dim3(grid), dim3(512), 0, s, P);
  } else {
    if (ks > 1) hipLaunchKernelGGL((wconv3_kernel<PREC_BF16, 1, true>), dim3(grid), dim3(512), 0, s, P);
    else hipLaunchKernelGGL((wconv3_kernel<PREC_BF16, 1, false>), dim3(grid), dim3(512), 0, s, P);
  }
  if (ks > 1) ksplit_reduce(a, ks, s);
  if (tok) {
    char name[96];
    // (the rocprofv3 names of the instantiations, so bench.py finds their PMC traffic in profiles/*/kernels.json)
    std::snprintf(name, sizeof(name),
                  ks > 1 ? "alcm::wconv3_kernel<%d, 1, true> + ksplit_reduce" : "alcm::wconv3_kernel<%d, 1, false>",
                  a.prec);
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " T%d C%d N%d k%d", a.T, a.Cp, a.N,
                    a.ksize);
    prof_stop(tok, s, name, flops, bytes);
  }
  return 1;
}

// Sum form (alcm_opconv_sum): three same-length terms with their own planes, weights, taps, biases and residuals
// into one output, one pass of the persistent kernel and one epilogue (out = (sum of the terms' conv + bias +
// residual) * scale (+ out)).  Eligible: the terms' shared B, T, Cp, N and precision (F16 / BF16), dilation 1,
// 3 <= k <= 65, Cp % 64 == 0, N % 192 == 0, full 256-row tiles filling the chip (as wconv3 by shape).  Returns 1
// when it launched.
bool wconv3_sum_ok(const alcm_opconv_args* a, int n) {
  if (n != 3 || knobs().wconv_sum == 0 || knobs().wconv <= 0 || knobs().wconv3 == 0) return false;
  const alcm_opconv_args& a0 = a[0];
  if ((a0.prec != PREC_F16 && a0.prec != PREC_BF16) || a0.Cp % 64 || a0.N % W3_BN) return false;
  // output: fp32 out, or (no accumulate) the operand plane of the value the fp32 route would store
  if (a0.out_plane ? (a0.out || a0.accumulate || (((uintptr_t)a0.out_plane) & 3)) : !a0.out) return false;
  for (int i = 0; i < n; ++i) {
    const alcm_opconv_args& t = a[i];
    if (t.B != a0.B || t.T != a0.T || t.Cp != a0.Cp || t.N != a0.N || t.prec != a0.prec || t.dil != 1 ||
        t.ksize < 3 || t.ksize - 1 > 64 || 2 * t.pad != t.ksize - 1 || t.out_act || t.out_stride > 0 ||
        t.geglu_plane || (i > 0 && t.out_plane) || t.act_plane || (int64_t)W3_BN * t.kpad * 2 >= (1ll << 31))
      return false;
  }
  if (!g_ncu) {
    int dev = 0, nc = 0;
    g_ncu = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&nc, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && nc >= 8)
                ? nc
                : 256;
  }
  const int mt256 = (a0.T + W3_BM - 1) / W3_BM;
  const int64_t nt = (int64_t)a0.B * mt256 * (a0.N / W3_BN);
  const bool full = a0.T * 100 >= mt256 * W3_BM * 85;
  if (!(knobs().wconv3 > 0 || (full && nt >= g_ncu))) return false;
  return nt < (1ll << 30) && (int64_t)a0.B * a0.T * a0.Cp < (1ll << 40) && (int64_t)a0.B * a0.T * a0.N < (1ll << 40);
}

int wconv3_sum_try(const alcm_opconv_args* a, int n, hipStream_t s) {
  if (!wconv3_sum_ok(a, n)) return 0;  // (sets g_ncu)
  const alcm_opconv_args& a0 = a[0];
  const int mt256 = (a0.T + W3_BM - 1) / W3_BM;
  const int64_t nt = (int64_t)a0.B * mt256 * (a0.N / W3_BN);
  WConvDev P{};
  P.a = (const u16*)a0.a;
  P.T = a0.T; P.Cp = a0.Cp; P.ksize = a0.ksize; P.dil = 1; P.pad = a0.pad;
  P.N = a0.N;
  P.out = a0.out; P.out_scale = a0.out_scale; P.accumulate = a0.accumulate;
  P.oplane = (u16*)a0.out_plane;
  P.tiles_per_batch = mt256;
  P.tiles_n = a0.N / W3_BN;
  P.nwg = (int)nt;
  P.n_major = 1;
  P.nseg = n;
  double flops = 0, bytes = (double)a0.B * a0.T * a0.N * (a0.out_plane ? 2.0 : 4.0 * (a0.accumulate ? 2 : 1));
  for (int i = 0; i < n; ++i) {
    const bool f16 = a[i].prec == PREC_F16;
    P.sa[i] = (const u16*)a[i].a;
    P.sw[i] = (const u16*)a[i].w + (f16 ? 2 * a[i].w_lo_off : 0);
    P.sk[i] = a[i].ksize;
    P.spad[i] = a[i].pad;
    P.skpad[i] = a[i].kpad;
    P.sbias[i] = a[i].bias;
    P.sres[i] = a[i].res;
    flops += 2.0 * a0.B * a0.T * a0.N * (double)a[i].ksize * a[i].C;
    bytes += (double)a0.B * a0.T * a0.Cp * 2.0 + (double)a0.N * a[i].kpad * 2.0 +
             (a[i].res ? (double)a0.B * a0.T * a0.N * 4.0 : 0.0);
  }
  P.w = P.sw[0]; P.kpad = P.skpad[0];
  const int R = (int)((nt + 7) / 8);
  int grid = 8 * std::min(g_ncu / 8, R);
  if (knobs().wconv3_grid >= 8) grid = std::min(grid, knobs().wconv3_grid / 8 * 8);  // tests: several tiles per workgroup
  void* tok = prof_start(s);
  if (a0.prec == PREC_F16) hipLaunchKernelGGL((wconv3_kernel<PREC_F16, 3, false>), dim3(grid), dim3(512), 0, s, P);
  else hipLaunchKernelGGL((wconv3_kernel<PREC_BF16, 3, false>), dim3(grid), dim3(512), 0, s, P);
  if (tok) {
    char name[96];
    std::snprintf(name, sizeof(name), "alcm::wconv3_kernel<%d, 3, false>", a0.prec);
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " T%d C%d N%d k%d+%d+%d", a0.T, a0.Cp,
                    a0.N, a[0].ksize, a[1].ksize, a[2].ksize);
    prof_stop(tok, s, name, flops, bytes);
  }
  return 1;
}

// wconv2 tile by shape: 256 x 96 where the weight stream dominates the per-CU fetch (k >= 7:
// the window is amortised over >= 7 taps) and there is at least one 256-row tile per CU; 128 x 192 elsewhere.
// Measured per launch (B = 32, one box): s0 C768 k11 0.946 -> 0.860 ms, s1 C384 k11
// 0.973 -> 0.934, s2 C192 k11 0.583 -> 0.559, DiT FFN-down 0.377 -> 0.358; k3 shapes equal or slower (VAE k3 +17 %)
static bool wconv2_tile256(const alcm_opconv_args& a) {
  const int64_t mt = (int64_t)a.B * ((a.T + 255) / 256);
  return a.out_stride <= 0 && a.ksize >= 7 && mt * (a.N / 96) >= 256;
}

// Eligible: single-plane precisions, N a multiple of 192 (128 x 192 tiles) or 96 (256 x 96 tiles), Cp a multiple of
// 64, (k-1)d <= 64, no output activation.  Returns 1 when it launched, 0 when the caller should use opconv_kernel
// (ALCM_WCONV=0: always 0 for plain same-length convs, the A/B reference; the strided and GEGLU epilogues exist
// only here).
int wconv_try(const alcm_opconv_args& a, const u16* wplane, double flops, double bytes, hipStream_t s) {
  const bool off = knobs().wconv <= 0;
  const bool strided = a.out_stride > 0;
  // persistent 8-wave kernel (ALCM_WCONV3: -1 by shape, 0 off, 1 wherever eligible): by shape where the 256-row
  // M tiles are >= 85 % full (BigVGAN T = 2496 / 9984 / 19968, DiT L = 467; not the VAE's T = 312, measured +15 %,
  // nor with the clips laid end to end as padded-flat rows: 2.85 vs 2.61 ms/step on wconv2)
  // A persistent grid with fewer tiles than CUs leaves CUs idle where the two-workgroup kernel's half-size tiles share
  // them: the DiT FFN down-projection (192 tiles of 256 x 192) measured 2.98 vs 2.82 ms/step (profiles/r4s)
  const int w3 = knobs().wconv3;
  const int mt256 = (a.T + W3_BM - 1) / W3_BM;
  const bool full = a.T * 100 >= mt256 * W3_BM * 85;
  if (!g_ncu) {
    int dev = 0, n = 0;
    g_ncu = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n >= 8)
                ? n
                : 256;
  }
  const int64_t tiles3 = (int64_t)a.B * mt256 * (a.N / W3_BN);
  const bool fills = tiles3 >= g_ncu;
  // a grid that does not fill the chip: K parts where the caller gave a partial workspace (ALCM_KSPLIT=0: never)
  const int ks = (!off && w3 != 0 && full && !fills && !strided && !a.geglu_plane && a.N % W3_BN == 0)
                     ? wconv3_parts(a, tiles3, g_ncu) : 1;
  if (!off && (a.out_plane || (int64_t)a.B * a.T >= 1024) && lin_plane_try(a, wplane, flops, bytes, s)) return 1;
  if (!off && w3 != 0 && !strided && !a.geglu_plane && (w3 > 0 || (full && (fills || ks > 1))) &&
      wconv3_try(a, wplane, flops, bytes, s, ks))
    return 1;
  if (off && !a.geglu_plane && !strided && !a.out_plane) return 0;
  if (a.prec != PREC_F16 && a.prec != PREC_BF16) return 0;
  if ((a.out_act && (a.geglu_plane || strided)) || a.Cp % 64 || a.ksize < 1 || (a.ksize - 1) * a.dil > W2_HALO)
    return 0;
  // N % 96: whole tiles; else (N % 4, not strided / GEGLU) 128 x 192 tiles with a partial last one (the T5 wi, N = 5632)
  const bool ragged = a.N % 96 != 0;
  if (ragged && (a.N % 4 || strided || a.geglu_plane)) return 0;
  // (only where the padded last tile wastes <= 25 % of the N tiles' columns: the text encoders' T5 wi / o, N = 5632 /
  // 1024; small ragged N stay on opconv_kernel's narrower tiles)
  if (ragged && 4 * (round_up(a.N, 192) - a.N) > round_up(a.N, 192)) return 0;
  if (!a.geglu_plane && !strided && !a.out_plane && (int64_t)a.B * a.T < 1024) return 0;  // small problems: opconv_kernel's
                                                                                     // 128-row tiles fill the chip better
  auto al16 = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  if (!(al16(a.bias) && al16(a.res) && al16(a.out))) return 0;
  if (a.geglu_plane && (a.res || a.accumulate || (((uintptr_t)a.geglu_plane) & 3))) return 0;
  // wconv2 tile: 256 x 96 halves the weight bytes every tile fetches (see the kernel comment)
  const bool t256 = !ragged && wconv2_tile256(a);
  // 160-row tiles where rounds x tile rows over the two-workgroup slots of the chip drop: the VAE's T = 312 k3 convs at
  // N = 1536 (768 tiles of 128 rows = 1.5 rounds, 512 of 160 = one; 1.82 -> 1.43 ms/step); N = 768
  // (384 tiles, one round either way) stays at 128
  // (strided: the BigVGAN stage 0 / 1 upsampler phases, T = 624 / 2496 at N = 768 / 384: 1.25 / 2.5 rounds of
  // 128-row tiles -> one / two of 160-row ones; ALCM_UPS_T160=0 keeps them at 128)
  bool t160 = false;
  if (!t256 && !a.geglu_plane && (!strided || knobs().ups_t160) && a.N % 192 == 0) {
    const int64_t slots = 2 * (int64_t)g_ncu, tn = a.N / 192;
    const int64_t r128 = ((int64_t)a.B * ((a.T + 127) / 128) * tn + slots - 1) / slots;
    const int64_t r160 = ((int64_t)a.B * ((a.T + 159) / 160) * tn + slots - 1) / slots;
    t160 = r160 * 160 < r128 * 128;
  }
  const int BM2 = t256 ? 256 : (t160 ? 160 : 128), BN2 = t256 ? 96 : 192;
  // K parts where the grid fills less than one round of the chip's two-workgroup slots (the text towers' out-
  // projections at 2464 rows: 80-120 tiles for 512 slots; the DiT to_out): plain fp32 epilogues only, the reduction
  // applies bias / residual / scale / accumulate in part order
  int ks2 = 1;
  if (!off && a.ksplit_ws && knobs().ksplit != 0 && !a.geglu_plane && !strided && !a.out_plane && !a.out_act &&
      a.N % 4 == 0) {
    const int64_t tiles = (int64_t)a.B * ((a.T + BM2 - 1) / BM2) * ((a.N + BN2 - 1) / BN2);
    const int64_t slots = 2 * (int64_t)g_ncu;
    const int nc = a.Cp / 64;
    double best = (double)((tiles + slots - 1) / slots);
    for (int k = 2; k <= 8; ++k) {
      // (>= 4 chunks of 64 channels per part: a part's window staging and its partial-slice epilogue are fixed costs)
      if (nc % k || nc / k < 4 || (double)k * a.B * a.T * a.N > (double)a.ksplit_ws_floats) continue;
      const double t = (double)((tiles * k + slots - 1) / slots) / k;
      if (t < best * 0.95) {
        best = t;
        ks2 = k;
      }
    }
    if (ks2 > 1 && ((((uintptr_t)a.ksplit_ws) & 15) || !a.out)) ks2 = 1;
  }
  if (a.N % BN2 == 0 || ragged) {
    WConvDev P{};
    P.a = (const u16*)a.a;
    P.T = a.T; P.Cp = a.Cp; P.ksize = a.ksize; P.dil = a.dil; P.pad = a.pad;
    P.w = wplane; P.kpad = a.kpad; P.N = a.N;
    P.bias = a.bias; P.res = a.res; P.out = a.out; P.out_scale = a.out_scale; P.accumulate = a.accumulate;
    P.gplane = (u16*)a.geglu_plane;
    P.out_act = a.out_act;
    P.oplane = (u16*)a.out_plane;
    P.ostride = strided ? a.out_stride : 1;
    P.ooff = strided ? a.out_offset : 0;
    P.orows = strided ? a.out_rows : a.T;
    // N-tile-major order where the weight matrix is long (Cp * k >= 4096) and there are enough M tiles to share
    // an XCD's weight slice: that XCD's N tiles stay in its L2 (C768 k11 -17 %, DiT FFN -3..-10 %); M-major
    // elsewhere (the N tiles of an M tile share its input window in L2)
    const int tiles_m = a.B * ((a.T + BM2 - 1) / BM2);
    // (the GEGLU up-projection, 64 M tiles x 48 N tiles of 1 MB weight slices: N-major -4 %, its M-major order
    // re-reads the weights from the Infinity Cache once per M tile, 3 GB counted per launch)
    P.n_major = (a.Cp * a.ksize >= 4096 && (tiles_m >= 128 || (a.geglu_plane && tiles_m >= 64)));
    P.tiles_per_batch = (a.T + BM2 - 1) / BM2;
    P.tiles_n = (a.N + BN2 - 1) / BN2;
    const int64_t nwg2 = (int64_t)a.B * P.tiles_per_batch * P.tiles_n;
    if (nwg2 * ks2 >= (1ll << 30) || (int64_t)a.B * a.T * a.Cp >= (1ll << 40)) return 0;
    P.nwg = (int)nwg2;
    if (ks2 > 1) {
      P.ksplit = ks2;
      P.part = a.ksplit_ws;
    }
    void* tok = prof_start(s);
    const dim3 grid((unsigned)(nwg2 * ks2)), blk(256);
    const bool gl = a.geglu_plane != nullptr;
    auto go = [&](auto bm_c) {
      constexpr int BM = decltype(bm_c)::value, BN = BM == 256 ? 96 : 192;
      if (a.prec == PREC_F16) {
        if (gl) hipLaunchKernelGGL((wconv2_kernel<PREC_F16, true, BM, BN>), grid, blk, 0, s, P);
        else hipLaunchKernelGGL((wconv2_kernel<PREC_F16, false, BM, BN>), grid, blk, 0, s, P);
      } else {
        if (gl) hipLaunchKernelGGL((wconv2_kernel<PREC_BF16, true, BM, BN>), grid, blk, 0, s, P);
        else hipLaunchKernelGGL((wconv2_kernel<PREC_BF16, false, BM, BN>), grid, blk, 0, s, P);
      }
    };
    if (t256) {
      go(std::integral_constant<int, 256>{});
    } else if (t160) {
      go(std::integral_constant<int, 160>{});
    } else {
      go(std::integral_constant<int, 128>{});
    }
    if (ks2 > 1) ksplit_reduce(a, ks2, s);
    if (tok) {
      char name[112];
      // the demangled rocprofv3 name (template defaults included), so bench.py can join the PMC passes by name
      std::snprintf(name, sizeof(name), ks2 > 1 ? "alcm::wconv2_kernel<%d, %s, %d, %d> + ksplit_reduce"
                                                : "alcm::wconv2_kernel<%d, %s, %d, %d>", a.prec, gl ? "true" : "false",
                    BM2, BN2);
      if (knobs().prof_shapes)
        std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " T%d C%d N%d k%d", a.T, a.Cp,
                      a.N, a.ksize);
      prof_stop(tok, s, name, flops, bytes);
    }
    return 1;
  }
  return 0;  // opconv_kernel
}

}  // namespace alcm
