// Narrow AMPBlock conv (BigVGAN stages 3-5, C = 96 / 48 / 24; vocoder/bigvgan/models.py:72-81) with the whole
// weight matrix resident in LDS: a persistent workgroup loads its weights once and then walks output tiles, so
// the K loop has no weight stream and no barriers.
//
// Why a separate kernel (scripts/microbench.py tailab / pmc_tail.sh on the stage-4 conv2 + residual + fused
// Activation1d, opconv_kernel): 60k cycles per 256-row tile-wave, MFMA 22 % busy; half of it the fused
// Activation1d epilogue (2.1k VALU instructions per wave, issued at the one-wave rate, items split 1.5 per thread
// by runtime divisions, plus zero stores for the 48 -> 64 operand padding), half a K loop whose window and
// weight tiles go through registers every 32-channel step (1.5k VALU instructions per wave, a barrier per step).
//
// Structure (one workgroup per CU, NW = BM / 32 waves, each 32 rows x NS columns):
//   * K is dense: k = tap * C + c (no channel padding: 528 instead of 704 deep at C = 48, k = 11), rounded up to
//     32; a lane's 8-element group never straddles a tap (C % 8 == 0), so its A fragment is one ds_read_b128 at
//     window row (m + tap * d), column c;
//   * weights [NSP][kd] fp16 (hi, and lo for the F16W2 precision) are DMA'd once per workgroup into rows of an
//     odd number of 16-B slots (conflict-free ds_read_b128 of 16 consecutive rows), rows NS .. NSP-1 zero;
//   * per tile: the input window (BM + (k-1)d rows x C channels, rows of an odd number of 16-B slots) by LDS-DMA,
//     the residual rows into registers, then the barrier-free K loop; the epilogue stages v = conv + bias in LDS
//     (over the dead window), adds the residual, writes the fp32 state rows it owns and applies Activation1d to
//     them (act_epilogue_ct: compile-time channel pairs, one pass over the threads) into the next conv's planes;
//   * C = 96 runs as two launches' worth of column halves (NS = 48 output channels per tile): its 96 x 1056
//     weight matrix does not fit one CU's LDS.
#include <cstdio>
#include <cstring>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __attribute__((aligned(16))) uint4 g_tconv_zero[8];  // a zero line for out-of-range DMA lanes

struct TConvDev {
  const u16* a;       // operand plane [B][T][Cp] (fp16); channels >= C are never read
  int T, Cp, ksize, dil, pad;
  const u16* w;       // dense fp16 weights [N][kd] (K = tap * C + c); lo plane at w + w_lo (F16W2)
  int64_t w_lo;
  int kd, N;
  const float* bias;
  const float* res;   // [B][T][N] or null
  float* out;         // [B][T][N] or null
  float out_scale;
  int accumulate;
  ActEpiDev act;      // act.plane == null: no Activation1d
  int tiles_per_batch, ntiles, ncg;  // ncg: column groups (N / NS)
  int wslots;         // 16-B slots per LDS weight row (odd)
  // diagnostics, read only by the DG = true instantiations (chosen when ALCM_TCONV_ABLATE or ALCM_TCONV_TRACE is set;
  // the production instantiations compile neither in):
  int ablate;         // ALCM_TCONV_ABLATE (timing only, results wrong): 1 no epilogue, 2 no MFMA, 4 no window DMA,
                      // 8 no plane stores, 16 no fp32 state stores
  unsigned long long* trace;  // ALCM_TCONV_TRACE: per-phase shader-clock sums over waves and tiles, or null
};

// phase timer of the diagnostics trace: wave-uniform shader-clock stamps, summed per phase over the tiles of a wave
// and added to P.trace by lane 0 at the end (vector atomics).  TcTimer<false> (the production instantiations) is
// empty: no registers, no clock reads, no atomics
template <bool DG>
struct TcTimer {
  bool on;
  unsigned long long last, ph[8];
  __device__ __forceinline__ void init(bool enable) {
    on = enable;
    for (int i = 0; i < 8; ++i) ph[i] = 0;
    last = on ? __builtin_readcyclecounter() : 0;
  }
  __device__ __forceinline__ void mark(int i) {
    if (!on) return;
    const unsigned long long t = __builtin_readcyclecounter();
    ph[i] += t - last;
    last = t;
  }
  __device__ __forceinline__ void tile() {
    if (on) ph[7] += 1;
  }
  __device__ __forceinline__ void flush(unsigned long long* out) {
    if (!on || (threadIdx.x & 63)) return;
    unsigned long long* o = out + (blockIdx.x & 63) * 8;  // 64 slot sets: no single-address contention
    for (int i = 0; i < 8; ++i) atomicAdd(o + i, ph[i]);
  }
};
template <>
struct TcTimer<false> {
  __device__ __forceinline__ void init(bool) {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void tile() {}
  __device__ __forceinline__ void flush(unsigned long long*) {}
};

// diagnostics (DG, trace on): workgroup residency record — s_memrealtime at entry and exit, HW_ID and XCC_ID of its CU
// (wave 0, lane 0; vector stores) at trace[512 + 4 * blockIdx.x ...] for blockIdx.x < TC_WG_REC
constexpr int TC_WG_REC = 2048;
__device__ __forceinline__ void tc_wg_record(unsigned long long* tr, int which) {
  if (!tr || threadIdx.x != 0 || blockIdx.x >= TC_WG_REC) return;
  unsigned long long* r = tr + 512 + 4 * blockIdx.x;
  r[which] = __builtin_amdgcn_s_memrealtime();
  if (which == 0) {
    r[2] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    r[3] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
  }
}

__device__ __forceinline__ void tc_glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds, 16, 0, 0);
}

// conv tile epilogue shared by the resident- and streamed-weight kernels: v = acc + bias staged in LDS (`ot`, row
// stride NS + 4 floats; the caller's barrier retired every K-loop read of that region), + residual (rv: the tile
// rows' residual, prefetched as float4 element e = tid + i * NT), fp32 state / accumulated output of the owned rows,
// Activation1d of the owned rows into the next conv's planes
template <int NS, int BM, int R, int TM, int TN, int NT, int NRES, bool ACT, bool RES, bool OUTW, bool ACC, bool DG,
          bool PRE = true>
__device__ __forceinline__ void tc_epilogue(const f32x4 (&acc)[TM][TN], const float (&bias_r)[TN],
                                          const float4 (&rv)[PRE ? NRES : 1], float* ot, int wr0, int t0, int e0, int E,
                                          int b, int n0, const TConvDev& P, TcTimer<DG>& tm) {
  constexpr int OTS = NS + 4;
  const int tid = threadIdx.x, lane = tid & 63, q4 = lane >> 4, l16 = lane & 15;
  // v = conv + bias -> LDS
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wr0 + i * 16 + q4 * 4 + r;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + l16;
        if (n < NS) ot[m * OTS + n] = acc[i][j][r] + bias_r[j];
      }
    }
  // residual rows not prefetched before the K loop (C = 96: 18 float4 per thread, too many registers beside the
  // accumulators): every load issued here in one burst, once the accumulators are dead, so the loop below waits for
  // one round trip (one load per iteration, next to the state stores that may alias it, waited for 18 round trips:
  // C96 k3 conv2 + residual + Activation1d 0.59 -> 0.46 ms, scripts/microbench.py tphase)
  constexpr bool LATE = RES && !PRE;
  float4 rl[LATE ? NRES : 1];
  if constexpr (LATE) {
#pragma unroll
    for (int i = 0; i < NRES; ++i) {
      const int e = min(tid + i * NT, BM * (NS / 4) - 1);
      const int m = e / (NS / 4), n = (e - m * (NS / 4)) * 4;
      rl[i] = *reinterpret_cast<const float4*>(P.res + ((int64_t)b * P.T + min(max(t0 + m, 0), P.T - 1)) * P.N + n0 + n);
    }
  }
  __syncthreads();
  tm.mark(3);
  const int e_hi = min(e0 + E, P.T);
  if constexpr (RES || OUTW || ACC) {
    // + residual (all tile rows: the activation reads the halo rows too); fp32 state of the owned rows
#pragma unroll
    for (int i = 0; i < NRES; ++i) {
      const int e = tid + i * NT;
      if (e >= BM * (NS / 4)) break;
      const int m = e / (NS / 4), n = (e - m * (NS / 4)) * 4;
      const int t = t0 + m;
      float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
      if constexpr (RES) {
        float4 r4;
        if constexpr (PRE) r4 = rv[PRE ? i : 0];
        else r4 = rl[LATE ? i : 0];
        v.x += r4.x; v.y += r4.y; v.z += r4.z; v.w += r4.w;
        if constexpr (ACT) *reinterpret_cast<float4*>(ot + m * OTS + n) = v;
      }
      if ((OUTW || ACC) && t >= e0 && t < e_hi && !(DG && (P.ablate & 16))) {
        float* op = P.out + ((int64_t)b * P.T + t) * P.N + n0 + n;
        if constexpr (ACC) {
          v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
          if (P.accumulate) {
            const float4 pv = *reinterpret_cast<const float4*>(op);
            v.x += pv.x; v.y += pv.y; v.z += pv.z; v.w += pv.w;
          }
        }
        *reinterpret_cast<float4*>(op) = v;
      }
    }
    if constexpr (ACT) __syncthreads();
  }
  tm.mark(4);
  if constexpr (ACT) {
    if (DG && (P.ablate & 8)) act_epilogue_ct<PREC_F16, R, NS / 2, true>(ot, OTS, t0, e0, e_hi, P.T, n0, b, P.act, tid, NT);
    else act_epilogue_ct<PREC_F16, R, NS / 2>(ot, OTS, t0, e0, e_hi, P.T, n0, b, P.act, tid, NT);
  }
  tm.mark(5);
}

// one wave's LDS-DMA of a tile window through a buffer descriptor over the batch's plane rows (device-only: the
// buffer builtins inside a kernel lambda make the host pass drop the kernel's launch stub): slot i of this lane at
// byte offset off[i] + shift, out-of-range offsets (before row 0, past the batch, or the 0x7fffffff of an unused
// slot) land as zeros without a memory access
template <int I0, int I1, int N>
__device__ __forceinline__ void tc_window_dma(uintptr_t base, uint32_t bytes, __attribute__((address_space(3))) char* dst,
                                              const uint32_t (&off)[N], uint32_t shift) {
  // descriptor from provably wave-uniform scalars (readfirstlane of the base halves and the size)
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uintptr_t)hi << 32) | lo), 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
#pragma unroll
  for (int i = I0; i < I1; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + i * 1024), 16, off[i] + shift, 0, 0, 0);
}

// the loader's window DMA of one tile (rows [t0 - pad, t0 - pad + WR) of its batch), slots [I0, I1)
// (the diagnostics' "no window DMA" bit is tested by the caller: a template flag here fails the host pass)
template <int I0, int I1, int N>
__device__ __forceinline__ void tc_window_tile(const TConvDev& P, int tile, int E, uint32_t batch_bytes,
                                               __attribute__((address_space(3))) char* dst, const uint32_t (&off)[N]) {
  const int mt = tile / P.ncg;
  const int b = mt / P.tiles_per_batch;
  const int t0 = (mt - b * P.tiles_per_batch) * E - ACT_EPI_HALO;
  tc_window_dma<I0, I1, N>((uintptr_t)(P.a + (int64_t)b * P.T * P.Cp), batch_bytes, dst, off,
                   (uint32_t)((t0 - P.pad) * P.Cp * 2));
}

// weight rows held in LDS: the NS real rows, plus ONE zero row that every B-fragment lane of the padding columns
// NS .. NSP-1 reads (a broadcast) when NS is not a multiple of 16
static constexpr int tc_wrows(int NS) { return NS % 16 ? NS + 1 : NS; }
// weights bytes reserved for taps <= kmax: tc_wrows rows x odd slots, rounded up to whole DMA instructions
static constexpr int tc_wbytes(int C, int NS, int NPB, int kmax) {
  const int kd = (kmax * C + 31) / 32 * 32;
  const int slots = (kd / 8) % 2 ? kd / 8 : kd / 8 + 1;
  return NPB * ((tc_wrows(NS) * slots + 63) / 64) * 1024;
}

// C input channels, NS output channels per tile, NPB weight planes (1 = F16, 2 = F16W2), BM rows per tile,
// R Activation1d rows per work item, KMAX the largest tap count the LDS weight region is sized for.
// NW = BM / 32 compute waves plus one loader wave (the last), which issues every window DMA and nothing else: vmcnt
// is one in-order counter per wave, so with the window DMA issued by the compute waves after their epilogue stores
// each window wait also waited for those stores to drain (scripts/microbench.py tphase, C48 k3 conv2: 12k of a
// 25k-cycle tile); the loader's waits cover its own DMA only and the stores drain under the next tile's K loop.
// Where the LDS holds the window apart from the staged tile (SEP: k <= 7 at C = 48), the loader DMAs the next tile's
// window as soon as the K loop is done with the current one, under the epilogue.
// OCC workgroups per CU (the launch bound on registers; the LDS must allow it too).
// DG: the diagnostics instantiation (ablation bits, phase trace); false in production.
template <int C, int NS, int NPB, int BM, int R, int KMAX, int OCC, bool ACT, bool RES, bool OUTW, bool ACC, bool DG>
__global__ __launch_bounds__(BM * 2 + 64, OCC == 1 ? 1 : (OCC * (BM / 32 + 1) + 3) / 4) void tconv_kernel(const TConvDev P) {
  constexpr int NW = BM / 32, NT = NW * 64;             // compute waves / threads
  constexpr int TM = 2, NSP = (NS + 15) / 16 * 16, TN = NSP / 16;
  constexpr int RSS = (C / 8) % 2 ? C / 8 : C / 8 + 1;  // window row: odd number of 16-B slots
  constexpr int RS = RSS * 16;
  constexpr int WRMAX = BM + 64;
  constexpr int WIN_INSTR = (WRMAX * RSS + 63) / 64;    // window DMA instructions per tile (64 slots each)
  constexpr int OTS = NS + 4;                           // staged fp32 row stride (floats)
  constexpr int STAGE = BM * OTS * 4;
  constexpr int WINB = WIN_INSTR * 1024;
  constexpr int WBYTES = tc_wbytes(C, NS, NPB, KMAX);
  constexpr bool SEP = WBYTES + WINB + STAGE <= 163840 / OCC;
  constexpr int REGION = SEP ? WINB + STAGE : (STAGE > WINB ? STAGE : WINB);
  constexpr int SMEM = WBYTES + REGION;
  static_assert(SMEM <= 163840 / OCC, "LDS: OCC workgroups per CU");
  static_assert(WIN_INSTR <= 60, "one wave's window DMA within the vmcnt range");
  static_assert((BM - 2 * ACT_EPI_HALO) % R == 0, "whole Activation1d runs (a partial run takes the clamped path)");
  static_assert(C % 8 == 0 && NS % 4 == 0, "geometry");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  char* const wl = smem;            // weights
  char* const win = smem + WBYTES;  // window (and, unless SEP, the staged tile after the K loop)
  float* const ot = reinterpret_cast<float*>(SEP ? win + WINB : win);
  // the window as an LDS-address-space pointer, cast once outside the loader's branch (a generic -> LDS cast inside it
  // trips the gfx950 backend: "Operand has incorrect register class" on src_shared_base)
  typedef __attribute__((address_space(3))) char lds_char_t;
  lds_char_t* const win3 = (lds_char_t*)win;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (DG) tc_wg_record(P.trace, 0);
  const int K = P.ksize, dil = P.dil;
  const int WS = P.wslots * 16;
  const int nslice = P.kd / 32;
  const int cg = blockIdx.x % P.ncg;  // column group of this workgroup's tiles (ncg divides the grid stride)
  const int n0 = cg * NS;
  const int E = BM - 2 * ACT_EPI_HALO;  // emitted rows per tile

  // ---- weights, once per workgroup (every wave): slot g of plane p -> row n = g / wslots, 16-B piece q = g % wslots
  // (row NS, when present, is the zero row)
  {
    const int total = tc_wrows(NS) * P.wslots;
    const int instr = (total + 63) / 64;
    for (int p = 0; p < NPB; ++p) {
      for (int i = wave; i < instr; i += NW + 1) {
        const int g = i * 64 + lane;
        const int n = g / P.wslots, q = g - n * P.wslots;
        const bool ok = g < total && n < NS && q < P.kd / 8;
        const u16* src = ok ? P.w + p * P.w_lo + (int64_t)(cg * NS + n) * P.kd + q * 8
                            : reinterpret_cast<const u16*>(g_tconv_zero);
        tc_glds16(src, wl + p * (WBYTES / NPB) + i * 1024);
      }
    }
  }

  if (wave == NW) {
    // ---- loader: the window of each tile (rows [t0 - pad, t0 - pad + WR), slot g -> row g / RSS, piece g % RSS,
    // pieces >= C / 8 zero), one barrier for each of the compute waves' per tile
    // per-lane byte offsets of the window slots relative to row t0 - pad of the batch (tile-invariant); slots past
    // the window or in a row's padding piece get an offset past any batch, which the buffer range check turns into
    // zeros without a memory access (as are rows before 0 or past T: negative or too-large offsets)
    const int WR = BM + (K - 1) * dil;
    uint32_t off[WIN_INSTR];
#pragma unroll
    for (int i = 0; i < WIN_INSTR; ++i) {
      const int g = i * 64 + lane;
      const int r = g / RSS, q = g - r * RSS;
      off[i] = (r < WR && q < C / 8) ? (uint32_t)((r * P.Cp + q * 8) * 2) : 0x7fffffffu;
    }
    const uint32_t batch_bytes = (uint32_t)P.T * (uint32_t)P.Cp * 2u;
    const bool dma = !(DG && (P.ablate & 4));
    int tile = blockIdx.x;
    if (dma && tile < P.ntiles) tc_window_tile<0, WIN_INSTR>(P, tile, E, batch_bytes, win3, off);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // weights + the first window
    // SEP: the next window's DMA issue (~100 cycles a piece) spread over the epilogue's barrier intervals, so that no
    // compute-wave barrier waits for the whole issue (in one piece it held the staging barrier ~3.5k cycles)
    constexpr bool RB = (RES || OUTW || ACC) && ACT;
    constexpr int D1 = WIN_INSTR / 5, D2 = RB ? D1 + WIN_INSTR / 4 : D1;
    for (; tile < P.ntiles; tile += gridDim.x) {
      const int next = tile + gridDim.x;
      const bool more = next < P.ntiles;
      __syncthreads();  // A: the window of `tile` has landed
      __syncthreads();  // B: the compute waves are done reading it
      if (dma && SEP && more) tc_window_tile<0, D1>(P, next, E, batch_bytes, win3, off);
      __syncthreads();  // staged tile written
      if constexpr (RB) {
        if (dma && SEP && more) tc_window_tile<D1, D2>(P, next, E, batch_bytes, win3, off);
        __syncthreads();  // residual / state pass done
      }
      if (dma && SEP && more) tc_window_tile<D2, WIN_INSTR>(P, next, E, batch_bytes, win3, off);
      __syncthreads();  // C: staged-tile reads retired
      if (dma && !SEP && more) tc_window_tile<0, WIN_INSTR>(P, next, E, batch_bytes, win3, off);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight DMA (the barrier A below publishes all)

  const int wr0 = wave * 32;  // first tile row of this wave
  const int q4 = lane >> 4, l16 = lane & 15;
  constexpr int NRES = (BM * (NS / 4) + NT - 1) / NT;  // residual float4 per thread
  float bias_r[TN];                                     // this lane's output-column biases, loaded once
#pragma unroll
  for (int j = 0; j < TN; ++j) bias_r[j] = (P.bias && j * 16 + l16 < NS) ? P.bias[n0 + j * 16 + l16] : 0.f;

  TcTimer<DG> tm;
  tm.init(P.trace != nullptr);
  for (int tile = blockIdx.x; tile < P.ntiles; tile += gridDim.x) {
    const int mt = tile / P.ncg;
    const int b = mt / P.tiles_per_batch;
    const int e0 = (mt - b * P.tiles_per_batch) * E;  // first emitted row
    const int t0 = e0 - ACT_EPI_HALO;                 // first computed row

    // residual rows of the tile (clamped to [0, T)) into registers, waited for in the epilogue
    float4 rv[NRES];
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < NRES; ++i) {
        const int e = tid + i * NT;
        const int m = e / (NS / 4), n = (e - m * (NS / 4)) * 4;
        const int t = min(max(t0 + m, 0), P.T - 1);
        rv[i] = *reinterpret_cast<const float4*>(P.res + ((int64_t)b * P.T + t) * P.N + n0 + (e < BM * (NS / 4) ? n : 0));
      }
    }
    __syncthreads();  // A
    tm.mark(0);

    // ---- barrier-free K loop over 32-deep slices of the dense K
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* arow = win + (wr0 + l16) * RS;
    const char* brow = wl + l16 * WS;
    int bro[TN];  // B-fragment row offsets: row j * 16 + l16, or the zero row NS past the real columns
#pragma unroll
    for (int j = 0; j < TN; ++j) bro[j] = (min(j * 16 + l16, NS) - l16) * WS;
    auto slice = [&](int s) {
      const int kk = s * 32 + q4 * 8;
      int tap = kk / C;
      const int c = kk - tap * C;
      tap = min(tap, K - 1);  // K padding: zero weights, any finite window value
      bf16x8 af[TM], bh[TN], bl[NPB == 2 ? TN : 1];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(arow + (i * 16 + tap * dil) * RS + c * 2);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(brow + bro[j] + kk * 2);
        if constexpr (NPB == 2) bl[j] = *reinterpret_cast<const bf16x8*>(brow + WBYTES / 2 + bro[j] + kk * 2);
      }
      if (DG && (P.ablate & 2)) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bh[j]));
        return;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (NPB == 2) acc[i][j] = mfma16<PREC_F16>(af[i], bl[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_F16>(af[i], bh[j], acc[i][j]);
        }
    };
    // two slices per iteration: the second slice's fragment reads can issue under the first slice's MFMAs
    int s = 0;
    for (; s + 1 < nslice; s += 2) {
      slice(s);
      slice(s + 1);
    }
    if (s < nslice) slice(s);
    tm.mark(1);
    __syncthreads();  // B: every window read retired (the loader may refill it; unless SEP it becomes the staged tile)
    tm.mark(2);
    if (DG && (P.ablate & 1)) {
      float sum = 0.f;  // keep every accumulator (and so the whole K loop) live
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (sum == 123.f && P.out) P.out[tid] = sum;
      __syncthreads();  // the epilogue's barriers, kept in step with the loader
      if constexpr ((RES || OUTW || ACC) && ACT) __syncthreads();
      __syncthreads();
      continue;
    }

    tc_epilogue<NS, BM, R, TM, TN, NT, NRES, ACT, RES, OUTW, ACC, DG>(acc, bias_r, rv, ot, wr0, t0, e0, E, b, n0, P, tm);
    __syncthreads();  // C: staged-tile reads retired
    tm.mark(6);
    tm.tile();
  }
  tm.flush(P.trace);
  if constexpr (DG) tc_wg_record(P.trace, 1);
}

// Streamed-weight variant (ALCM_TCONV=2 / by shape): 4 waves of 64 rows x NS columns, the weights of each 32-deep K
// slice DMA'd two slices ahead into a 4-slot LDS ring (one barrier per slice), <= 80 KB of LDS so two workgroups
// share a CU: the Activation1d epilogue (VALU) of one overlaps the K loop (MFMA) of the other, which the
// resident-weight kernel (one workgroup per CU at C >= 48) cannot do.  Ring slot layout: row n of 64 B (32 fp16 of
// K), its 16-B piece q at physical piece q ^ ((n >> 2) & 3) (conflict-free ds_read_b128 of 16 consecutive rows).
// OCC workgroups per CU: 2, or 4 (<= 128 VGPRs: the residual is then loaded in the epilogue, not prefetched).
// STG: s_sleep(127) count before the second half of a persistent grid starts (C = 96); DG as tconv_kernel.
template <int C, int NS, int NPB, int BM, int R, bool ACT, bool RES, bool OUTW, bool ACC, int OCC, int STG, bool DG>
__global__ __launch_bounds__(256, OCC) void tconv2_kernel(const TConvDev P) {
  constexpr int PD = 2;  // weight slices in flight ahead of the one consumed (3: equal, the K loop is LDS-read bound)
  constexpr int NT = 256, RPW = BM / 4, TM = RPW / 16;
  constexpr int NSP = (NS + 15) / 16 * 16, TN = NSP / 16;
  constexpr int RSS = (C / 8) % 2 ? C / 8 : C / 8 + 1;
  constexpr int RS = RSS * 16;
  constexpr int WRMAX = BM + 64;
  constexpr int WIN_INSTR = (WRMAX * RSS + 63) / 64;
  constexpr int WPW = (WIN_INSTR + 3) / 4;              // window DMA instructions per wave (uniform)
  constexpr int SLOT = NSP * 64 * NPB;                  // one K slice of every weight plane
  constexpr int SPI = (NSP * 4 * NPB + 63) / 64;        // DMA instructions per slice
  constexpr int DPW = (SPI + 3) / 4;                    // per wave (uniform: extra lanes write the scratch line)
  constexpr int RING = 4;
  constexpr int WINB = WPW * 4 * 1024;
  constexpr int RINGB = RING * SLOT;
  constexpr int OTS = NS + 4;
  constexpr int STAGE = BM * OTS * 4;
  constexpr int REGION = (STAGE > WINB + RINGB ? STAGE : WINB + RINGB);
  constexpr int SMEM = REGION + 1024 * 4;               // + one scratch KB per wave for padding DMA instructions
  static_assert(SMEM <= 163840 / OCC, "OCC workgroups per CU");
  static_assert((BM - 2 * ACT_EPI_HALO) % R == 0, "whole Activation1d runs (a partial run takes the clamped path)");
  static_assert(C % 8 == 0 && NS % 4 == 0 && RPW % 16 == 0, "geometry");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  char* const win = smem;
  char* const ring = smem + WINB;
  char* const scratch = smem + REGION;
  float* const ot = reinterpret_cast<float*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, l16 = lane & 15;
  const int K = P.ksize, dil = P.dil;
  const int nslice = P.kd / 32;
  const int E = BM - 2 * ACT_EPI_HALO;
  // persistent grid (C = 96): the second half of the workgroups (the second workgroup of each CU)
  // starts STG sleeps late, so the two workgroups of a CU alternate K loop (MFMA) and Activation1d epilogue
  // (VALU) instead of running both phases in lockstep
  if constexpr (STG > 0)
    if ((int)blockIdx.x >= (int)gridDim.x / 2)
      for (int i = 0; i < STG; ++i) __builtin_amdgcn_s_sleep(127);
  TcTimer<DG> tm;
  tm.init(P.trace != nullptr);
  for (int tile = blockIdx.x; tile < P.ntiles; tile += gridDim.x) {
  const int mt = tile / P.ncg, cg = tile - mt * P.ncg;
  const int n0 = cg * NS;
  const int b = mt / P.tiles_per_batch;
  const int e0 = (mt - b * P.tiles_per_batch) * E;
  const int t0 = e0 - ACT_EPI_HALO;
  const int WR = BM + (K - 1) * dil;
  const int wr0 = wave * RPW;

  float bias_r[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bias_r[j] = (P.bias && j * 16 + l16 < NS) ? P.bias[n0 + j * 16 + l16] : 0.f;
  constexpr int NRES = (BM * (NS / 4) + NT - 1) / NT;
  // residual prefetched into registers at the tile start (C = 96: loaded in the epilogue; prefetched, its 72 registers
  // beside the accumulators spill and the window wait covers it: 0.59 -> 0.75 ms)
  constexpr bool PRE = NRES <= 12 && OCC == 2;
  float4 rv[PRE ? NRES : 1];
  if constexpr (RES && PRE) {
#pragma unroll
    for (int i = 0; i < NRES; ++i) {
      const int e = tid + i * NT;
      const int m = e / (NS / 4), n = (e - m * (NS / 4)) * 4;
      const int t = min(max(t0 + m, 0), P.T - 1);
      rv[i] = *reinterpret_cast<const float4*>(P.res + ((int64_t)b * P.T + t) * P.N + n0 + (e < BM * (NS / 4) ? n : 0));
    }
  }
  // window: slot g -> row g / RSS, piece g % RSS
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int i = wave + 4 * j;
    const int g = i * 64 + lane;
    const int r = g / RSS, q = g - r * RSS;
    const int ts = t0 - P.pad + r;
    const bool ok = i < WIN_INSTR && r < WR && q < C / 8 && ts >= 0 && ts < P.T;
    const u16* src = ok ? P.a + ((int64_t)b * P.T + ts) * P.Cp + q * 8 : reinterpret_cast<const u16*>(g_tconv_zero);
    tc_glds16(src, win + i * 1024);
  }
  // weight slice s -> ring slot s % RING: instruction i covers slots 64 i .. 64 i + 63 of [plane][n][piece]
  auto stage_slice = [&](int s) {
    char* dst = ring + (s % RING) * SLOT;
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int i = wave + 4 * j;
      const int g = i * 64 + lane;
      const int p = g / (NSP * 4), gg = g - p * (NSP * 4);
      const int n = gg >> 2, pq = gg & 3;
      const int q = pq ^ ((n >> 2) & 3);
      const bool ok = i < SPI && n < NS;
      const u16* src = ok ? P.w + p * P.w_lo + (int64_t)(n0 + n) * P.kd + s * 32 + q * 8
                          : reinterpret_cast<const u16*>(g_tconv_zero);
      tc_glds16(src, i < SPI ? dst + i * 1024 : scratch + wave * 1024);
    }
  };
  static_assert(DPW <= 2, "vmcnt immediates below");
  // wait until at most `ahead` slices' DMA are outstanding (every older access of this wave has landed)
  auto wait_ahead = [&](int ahead) {
    if (ahead >= 2) {
      if constexpr (DPW == 1) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else if (ahead == 1) {
      if constexpr (DPW == 1) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
  };
  for (int j = 0; j < PD && j < nslice; ++j) stage_slice(j);
  wait_ahead(min(PD, nslice) - 1);
  __builtin_amdgcn_s_barrier();
  tm.mark(0);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* arow = win + (wr0 + l16) * RS;
  const int bsw = (l16 >> 2) & 3;
  for (int s = 0; s < nslice; ++s) {
    if (s + PD < nslice) stage_slice(s + PD);
    const int kk = s * 32 + q4 * 8;
    int tap = kk / C;
    const int c = kk - tap * C;
    tap = min(tap, K - 1);
    const char* bs = ring + (s % RING) * SLOT + l16 * 64 + ((q4 ^ bsw) << 4);
    bf16x8 af[TM], bh[TN], bl[NPB == 2 ? TN : 1];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(bs + j * 16 * 64);
      if constexpr (NPB == 2) bl[j] = *reinterpret_cast<const bf16x8*>(bs + NSP * 64 + j * 16 * 64);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(arow + (i * 16 + tap * dil) * RS + c * 2);
    if (DG && (P.ablate & 2)) {
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bh[j]));
    } else {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (NPB == 2) acc[i][j] = mfma16<PREC_F16>(af[i], bl[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_F16>(af[i], bh[j], acc[i][j]);
        }
      __builtin_amdgcn_s_setprio(0);
    }
    // slice s + 1 has landed; the slices issued beyond it stay in flight across the barrier
    wait_ahead(min(PD - 1, nslice - 2 - s));
    __builtin_amdgcn_s_barrier();
  }
  tm.mark(1);
  tm.mark(2);
  if (DG && (P.ablate & 1)) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 123.f && P.out) P.out[tid] = sum;
    continue;
  }
  tc_epilogue<NS, BM, R, TM, TN, NT, NRES, ACT, RES, OUTW, ACC, DG, PRE>(acc, bias_r, rv, ot, wr0, t0, e0, E, b, n0, P,
                                                                      tm);
  __syncthreads();  // staged-tile reads retired before the next tile's DMA overwrites the region
  tm.mark(6);
  tm.tile();
  }
  tm.flush(P.trace);
}

// -------------------------------------------------------------------------------------------------- host
unsigned long long* g_tc_trace = nullptr;  // diagnostics trace buffer (64 x 8 sums + TC_WG_REC workgroup records),
                                           // allocated by the first
                                           // alcm_debug_tconv_trace call (never inside a launch path)

struct TConvCfg {
  int C, NS, NPB, BM;
};

bool tconv_supported(int prec, int C, int N, int ksize, int dil) {
  if (knobs().tconv == 0) return false;
  if (prec != PREC_F16 && prec != PREC_F16W2) return false;
  if (C != N || ksize > 11 || (ksize - 1) * dil > 64) return false;
  if (C == 96) return prec == PREC_F16;
  return C == 48 || C == 24;
}

template <int C, int NS, int NPB, int BM, int R, int KMAX, int OCC, bool ACT, bool RES, bool OUTW, bool ACC>
static void tc_launch(const TConvDev& P, bool diag, int grid, hipStream_t s) {
  const dim3 g(grid), blk(BM * 2 + 64);
  if (diag) hipLaunchKernelGGL((tconv_kernel<C, NS, NPB, BM, R, KMAX, OCC, ACT, RES, OUTW, ACC, true>), g, blk, 0, s, P);
  else hipLaunchKernelGGL((tconv_kernel<C, NS, NPB, BM, R, KMAX, OCC, ACT, RES, OUTW, ACC, false>), g, blk, 0, s, P);
}

template <int C, int NS, int NPB, int BM, int R, int KMAX = 11, int OCC = 1>
static int tc_mode(const TConvDev& P, bool diag, int grid, bool act, bool res, bool outw, bool acc, hipStream_t s) {
  if (P.kd > (KMAX * C + 31) / 32 * 32) return set_error(ALCM_E_INVALID, "tconv: weights exceed the LDS reservation");
  if (act && !res && !outw && !acc) tc_launch<C, NS, NPB, BM, R, KMAX, OCC, true, false, false, false>(P, diag, grid, s);
  else if (act && res && outw && !acc) tc_launch<C, NS, NPB, BM, R, KMAX, OCC, true, true, true, false>(P, diag, grid, s);
  else if (!act && res && acc) tc_launch<C, NS, NPB, BM, R, KMAX, OCC, false, true, false, true>(P, diag, grid, s);
  else return set_error(ALCM_E_INVALID, "tconv: unsupported epilogue combination");
  return 0;
}

template <int C, int NS, int NPB, int BM, int R, bool ACT, bool RES, bool OUTW, bool ACC, int OCC, int STG>
static void tc2_launch(const TConvDev& P, bool diag, int grid, hipStream_t s) {
  if (diag) hipLaunchKernelGGL((tconv2_kernel<C, NS, NPB, BM, R, ACT, RES, OUTW, ACC, OCC, STG, true>), dim3(grid), dim3(256), 0, s, P);
  else hipLaunchKernelGGL((tconv2_kernel<C, NS, NPB, BM, R, ACT, RES, OUTW, ACC, OCC, STG, false>), dim3(grid), dim3(256), 0, s, P);
}

template <int C, int NS, int NPB, int BM, int R, int OCC = 2, int STG = 0>
static int tc2_mode(const TConvDev& P, bool diag, int grid, bool act, bool res, bool outw, bool acc, hipStream_t s) {
  if (act && !res && !outw && !acc) tc2_launch<C, NS, NPB, BM, R, true, false, false, false, OCC, STG>(P, diag, grid, s);
  else if (act && res && outw && !acc) tc2_launch<C, NS, NPB, BM, R, true, true, true, false, OCC, STG>(P, diag, grid, s);
  else if (!act && res && acc) tc2_launch<C, NS, NPB, BM, R, false, true, false, true, OCC, STG>(P, diag, grid, s);
  else return set_error(ALCM_E_INVALID, "tconv: unsupported epilogue combination");
  return 0;
}

// conv on operand planes with dense fp16 weights `wd` ([N][kd], K = tap * C + c; lo plane wd_lo elements after
// hi for F16W2): out / res fp32 [B][T][N], Activation1d of the result into act->plane (or none)
int tconv(const alcm_opconv_args& a, const u16* wd, int64_t wd_lo, int kd, const ActEpiDev* act, double flops,
          double bytes, hipStream_t s) {
  if (!tconv_supported(a.prec, a.C, a.N, a.ksize, a.dil)) return set_error(ALCM_E_INVALID, "tconv: unsupported shape");
  if (a.C <= 0 || a.Cp < a.C || a.ksize < 1 || a.dil < 1) return set_error(ALCM_E_INVALID, "tconv: bad geometry");
  if (kd != (a.ksize * a.C + 31) / 32 * 32 || !wd) return set_error(ALCM_E_INVALID, "tconv: dense weight layout");
  if (2 * a.pad != (a.ksize - 1) * a.dil || a.out_stride > 0 || a.out_act || a.geglu_plane)
    return set_error(ALCM_E_INVALID, "tconv: same-length convs only");
  if ((((uintptr_t)a.a) & 15) || (((uintptr_t)wd) & 15) || (wd_lo % 8) || (a.Cp % 8) ||
      (a.res && (((uintptr_t)a.res) & 15)) || (a.out && (((uintptr_t)a.out) & 15)))
    return set_error(ALCM_E_INVALID, "tconv: alignment");
  const bool acc_mode = !act && a.res && a.out;
  if (act && (a.accumulate || (a.out && !a.res))) return set_error(ALCM_E_INVALID, "tconv: epilogue combination");
  TConvDev P{};
  P.a = (const u16*)a.a;
  P.T = a.T; P.Cp = a.Cp; P.ksize = a.ksize; P.dil = a.dil; P.pad = a.pad;
  P.w = wd; P.w_lo = wd_lo; P.kd = kd; P.N = a.N;
  P.bias = a.bias; P.res = a.res; P.out = a.out; P.out_scale = a.out_scale; P.accumulate = a.accumulate;
  if (act) P.act = *act;
  // the diagnostics instantiation only when a diagnostic is asked for (the trace needs its buffer, allocated by the
  // first alcm_debug_tconv_trace call)
  P.ablate = knobs().tconv_ablate;
  if (knobs().tconv_trace) P.trace = g_tc_trace;
  const bool diag = P.ablate != 0 || P.trace != nullptr;
  const int slots = kd / 8;
  P.wslots = slots % 2 ? slots : slots + 1;
  const int npb = a.prec == PREC_F16W2 ? 2 : 1;
  const int C = a.C;
  // streamed weights (two workgroups per CU) where the resident weights would take a CU's LDS: C >= 48
  const int tk = knobs().tconv;
  // measured per launch (scripts/microbench.py tconv): streamed wins at C = 96 and C = 24, resident at C = 48
  const bool streamed = tk == 2 || (tk != 3 && tk != 4 && C != 48);
  // ALCM_TCONV=4 (C = 48): column halves (NS = 24, the B fragments of columns 24..31 read one zero row) on 128-row
  // tiles, so the resident weights (k11: 54 KB) and the window leave room for two workgroups per CU
  const bool half48 = !streamed && C == 48 && (tk == 4 || tk == 5);
  const int occ48 = (tk == 5 && a.ksize <= 3) ? 3 : 2;  // ALCM_TCONV=5: k = 3 at three workgroups per CU
  const int BM = C == 96 ? 192 : (half48 ? 128 : 256);
  const int NS = (!streamed && C == 96) ? 48 : (half48 ? 24 : C);
  P.ncg = a.N / NS;
  P.tiles_per_batch = (a.T + (BM - 2 * ACT_EPI_HALO) - 1) / (BM - 2 * ACT_EPI_HALO);
  const int64_t nt = (int64_t)a.B * P.tiles_per_batch * P.ncg;
  if (nt >= (1ll << 30)) return set_error(ALCM_E_INVALID, "tconv: problem too large");
  P.ntiles = (int)nt;
  const bool outw = a.out && !acc_mode;
  void* tok = prof_start(s);
  int rc;
  if (streamed) {
    // C = 96: persistent, two workgroups per CU, the second half delayed by 2 sleeps (scripts/microbench.py tconv, one
    // box: k11 0.547 -> 0.491 ms, k3 0.300 -> 0.301, conv2 + residual 0.732 -> 0.695); C = 24 one workgroup per tile
    // (persistent measured +5..+17 %)
    int grid2 = (int)nt;
    if (C == 96) {
      int dev = 0, ncu = 256;
      if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      grid2 = (int)std::min<int64_t>(nt, (int64_t)ncu * 2);
    }
    if (C == 96) rc = tc2_mode<96, 96, 1, 192, 11, 2, 2>(P, diag, grid2, act, a.res, outw, acc_mode, s);
    else if (C == 48) {
      if (npb == 2) rc = tc2_mode<48, 48, 2, 256, 24>(P, diag, grid2, act, a.res, outw, acc_mode, s);
      else rc = tc2_mode<48, 48, 1, 256, 24>(P, diag, grid2, act, a.res, outw, acc_mode, s);
    } else {
      // four workgroups per CU (6-row Activation1d runs and the residual loaded in the epilogue keep it at 128 VGPRs):
      // conv2 + residual + Activation1d 0.61 -> 0.51 ms (k3), 0.70 -> 0.55 (k11), conv1 k3 0.39 -> 0.37, end to end
      // -0.5 ms/step (gpurun_out/r5aa)
      if (npb == 2) rc = tc2_mode<24, 24, 2, 256, 6, 4>(P, diag, grid2, act, a.res, outw, acc_mode, s);
      else rc = tc2_mode<24, 24, 1, 256, 12>(P, diag, grid2, act, a.res, outw, acc_mode, s);  // (other policies; a W1 twin of
      // the W2 instantiation's template arguments above made the compiler spill 84 B in the W2 kernel, 12 without)
    }
  } else {
    // persistent: a multiple of ncg workgroups so a workgroup's column group (blockIdx % ncg) is the same for every
    // tile it takes (tile % ncg == blockIdx % ncg); C = 24 fits two per CU
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int wgs = half48 ? occ48 : (C == 24 ? 2 : 1);
    int grid = std::min<int64_t>(nt, (int64_t)ncu * wgs);
    grid = std::max(P.ncg, grid / P.ncg * P.ncg);
    if (C == 96) rc = tc_mode<96, 48, 1, 192, 11>(P, diag, grid, act, a.res, outw, acc_mode, s);
    else if (half48) {
      if (npb == 2 && a.ksize <= 3 && occ48 == 3)
        rc = tc_mode<48, 24, 2, 128, 7, 3, 3>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else if (npb == 2 && a.ksize <= 3) rc = tc_mode<48, 24, 2, 128, 7, 3, 2>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else if (npb == 2 && a.ksize <= 7) rc = tc_mode<48, 24, 2, 128, 7, 7, 2>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else if (npb == 2) rc = tc_mode<48, 24, 2, 128, 7, 11, 2>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else rc = tc_mode<48, 24, 1, 128, 7, 11, 2>(P, diag, grid, act, a.res, outw, acc_mode, s);
    } else if (C == 48) {
      // LDS weight region sized by the taps: k <= 7 leaves room for the window apart from the staged tile
      if (npb == 2 && a.ksize <= 3) rc = tc_mode<48, 48, 2, 256, 12, 3>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else if (npb == 2 && a.ksize <= 7) rc = tc_mode<48, 48, 2, 256, 12, 7>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else if (npb == 2) rc = tc_mode<48, 48, 2, 256, 12>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else rc = tc_mode<48, 48, 1, 256, 12>(P, diag, grid, act, a.res, outw, acc_mode, s);
    } else {
      if (npb == 2) rc = tc_mode<24, 24, 2, 256, 6>(P, diag, grid, act, a.res, outw, acc_mode, s);
      else rc = tc_mode<24, 24, 1, 256, 6>(P, diag, grid, act, a.res, outw, acc_mode, s);
    }
  }
  if (rc) return rc;
  if (tok) {
    char name[96];
    std::snprintf(name, sizeof(name), "alcm::tconv%s_kernel<C%d, W%d, BM%d, %s%s%s>", streamed ? "2" : "", C, npb, BM, act ? "act" : "",
                  a.res ? "+res" : "", acc_mode ? "+acc" : "");
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " T%d k%d", a.T, a.ksize);
    prof_stop(tok, s, name, flops, bytes);
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm

extern "C" int alcm_opconv_dense(const alcm_opconv_args* args, alcm_stream_t stream) {
  using namespace alcm;
  if (!args || !args->a || !args->w || args->B <= 0 || args->T <= 0) return set_error(ALCM_E_INVALID, "opconv_dense: bad arguments");
  const alcm_opconv_args& a = *args;
  ActEpiDev E{};
  const bool act = a.act_plane != nullptr;
  if (act) {
    if (!a.act_alpha_exp || !a.act_inv_beta || !a.act_up_filter || !a.act_down_filter || a.N % 2)
      return set_error(ALCM_E_INVALID, "opconv_dense: activation parameters");
    E.plane = (u16*)a.act_plane;
    E.plane_lo = 0;
    E.Cp = round_up(a.N, 32);
    E.aexp = a.act_alpha_exp;
    E.ibeta = a.act_inv_beta;
    for (int k = 0; k < 12; ++k) {
      E.f.up[k] = 2.0f * a.act_up_filter[k];
      E.f.dn[k] = a.act_down_filter[k];
    }
  }
  const double M = (double)a.B * a.T;
  const double flops = 2.0 * M * a.N * (double)a.ksize * a.C;
  const double bytes = M * a.C * 2.0 + (double)a.N * a.kpad * 2.0 * (a.prec == PREC_F16W2 ? 2 : 1) +
                       M * a.N * 4.0 * ((a.out ? 1 : 0) + (a.res ? 1 : 0) + (a.accumulate ? 1 : 0)) +
                       (act ? M * a.N * 2.0 : 0.0);
  return tconv(a, (const u16*)a.w + 2 * a.w_lo_off, a.w_lo_off, a.kpad, act ? &E : nullptr, flops, bytes,
               (hipStream_t)stream);
}

// diagnostics: the tconv phase trace (ALCM_TCONV_TRACE = 1) summed since the last reset; reset zeroes it.  The first
// call allocates the trace buffer (zeroed, returns zeros; launches trace from then on).  Synchronizes the device.
extern "C" int alcm_debug_tconv_trace(unsigned long long* out8, int reset) {
  using namespace alcm;
  if (!out8) return set_error(ALCM_E_INVALID, "debug_tconv_trace: null output");
  if (!alcm::g_tc_trace) {
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const size_t nb = (512 + 4 * TC_WG_REC) * sizeof(unsigned long long);
    ALCM_HIP(hipMalloc(&alcm::g_tc_trace, nb));
    ALCM_HIP(hipMemset(alcm::g_tc_trace, 0, nb));
    ALCM_HIP(hipDeviceSynchronize());
    return 0;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned long long h[512];
  if (hipMemcpy(h, alcm::g_tc_trace, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  for (int i = 0; i < 8; ++i) {
    out8[i] = 0;
    for (int j = 0; j < 64; ++j) out8[i] += h[j * 8 + i];
  }
  // (the reset clears the workgroup residency records too)
  if (reset && hipMemset(alcm::g_tc_trace, 0, (512 + 4 * TC_WG_REC) * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return 0;
}

// diagnostics: the workgroup residency records of the last traced resident-weight tail conv (ALCM_TCONV_TRACE = 1):
// per workgroup [entry s_memrealtime, exit s_memrealtime, HW_ID, XCC_ID] into out (4 x n_wg values); returns the
// number of records copied (0 before the first alcm_debug_tconv_trace call).  Synchronizes the device.
extern "C" int alcm_debug_tconv_wg_times(unsigned long long* out, int n_wg) {
  using namespace alcm;
  if (!out || n_wg < 0) return set_error(ALCM_E_INVALID, "debug_tconv_wg_times: bad arguments");
  if (!alcm::g_tc_trace) return 0;
  const int n = std::min(n_wg, TC_WG_REC);
  ALCM_HIP(hipDeviceSynchronize());
  ALCM_HIP(hipMemcpy(out, alcm::g_tc_trace + 512, (size_t)n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return n;
}
