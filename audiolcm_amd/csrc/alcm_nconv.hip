// Narrow implicit-GEMM conv1d for the HBM-bound BigVGAN tail (C = N in {96, 48, 24};
// vocoder/bigvgan/models.py:72-81) on operand planes, with the fused epilogues of alcm_opconv.hip.
//
// A narrow layer has little MFMA work per K step (one tap x 32 channels), so a register-staged weight
// prefetch one step ahead leaves every step waiting on an L2 round trip.  Here:
//   * the input windows of ALL channel chunks of the tile (rows [t0 - pad, t0 + BM + (k-1)d - pad) x Cp)
//     are staged once, by LDS-DMA, at the start of the tile;
//   * the weight tiles of the K steps (chunk, tap) stream through a ring of NBUF LDS buffers by LDS-DMA,
//     NBUF - 1 steps ahead, with counted `s_waitcnt vmcnt` and raw barriers (nothing drains the queue);
//   * LDS rows are 64 B (32 channels); the 16-B slot of logical slot s in row r is s ^ ((r >> 1) & 2),
//     applied on the DMA source address and on the fragment read, which makes the ds_read_b128 fragment
//     reads conflict-free at any start row (the tap offset tap*d is arbitrary) — found by exhaustive search
//     over the XOR-linear swizzles of the row bits;
//   * rows outside [0, T) and weight rows >= N read a zero line (per-lane DMA source select).
// Four waves split the tile's BM rows; each covers all BN columns.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

typedef __attribute__((address_space(3))) void nc_lds_void_t;
typedef __attribute__((address_space(1))) void nc_gbl_void_t;

__device__ __attribute__((aligned(16))) uint4 g_nconv_zero[8];  // 128 zero bytes

struct NConvDev {
  const u16* a;  // operand plane [B][T][Cp]
  int T, Cp, ksize, dil, pad;
  const u16* w;  // packed weight planes [N][kpad] (hi) and w + w_lo (lo, F16W2)
  int64_t w_lo;
  int kpad, N;
  const float* bias;
  const float* res;
  float* out;
  float out_scale;
  int accumulate;
  int tiles_per_batch, tstride, tshift;
  ActEpiDev act;
  int act_prefetch;  // ACT: residual prefetched into registers before the K loop
};

constexpr int NC_HALO = 64;  // max (k-1)*dil

__device__ __forceinline__ void nc_glds4(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((nc_gbl_void_t*)src, (nc_lds_void_t*)lds_base, 4, 0, 0);
}
__device__ __forceinline__ void nc_glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((nc_gbl_void_t*)src, (nc_lds_void_t*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ int nc_swz(int row) { return (row >> 1) & 2; }

template <int N>
__device__ __forceinline__ void nc_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// BM rows per tile (4 waves x BM/4), BN >= N columns (multiple of 16), NCH = Cp/32 chunks (all resident),
// NBUF weight ring buffers; PREC F16 / F16W2 / BF16 (single-plane activations)
template <int BM, int BN, int NCH, int NBUF, int PREC, bool ACT>
__global__ __launch_bounds__(256) void nconv_kernel(const NConvDev P) {
  constexpr int TM = BM / 64;            // 16-row fragments per wave
  constexpr int TN = BN / 16;
  constexpr int NPB = PREC == PREC_F16W2 ? 2 : 1;
  constexpr int WROWS = BM + NC_HALO;    // staged window rows per chunk
  constexpr int WBYTES = WROWS * 64;     // one chunk's window
  constexpr int WPW = WROWS * 64 / 1024 / 4;  // 16-B DMA instructions per wave per chunk
  static_assert(WROWS * 64 % 4096 == 0, "window = whole DMA instructions for each of the 4 waves");
  constexpr int SBYTES = BN * 64 * NPB;  // one K step's weight tile (all planes)
  constexpr int G = SBYTES / 256 / 4;    // 4-B DMA instructions per wave per step
  static_assert(SBYTES % 1024 == 0, "weight tile = whole 4-B DMA instructions for each of the 4 waves");
  constexpr int D = NBUF - 1;            // prefetch distance (steps)
  static_assert((D - 1) * G < 64, "vmcnt immediate");
  constexpr int KSMEM = NCH * WBYTES + NBUF * SBYTES;
  constexpr int OTS = BN + 4;
  constexpr int TSMEM = BM * OTS * 4;    // LDS-staged output tile (epilogue, aliases the K-loop buffers)
  constexpr int SMEM = KSMEM > TSMEM ? KSMEM : TSMEM;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  char* const wl = smem;                  // windows
  char* const bl = smem + NCH * WBYTES;   // weight ring

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / P.tiles_per_batch;
  const int t0 = (blockIdx.x - b * P.tiles_per_batch) * P.tstride - P.tshift;
  const int K = P.ksize;
  const int nsteps = NCH * K;

  // ---- windows of every chunk: instruction i (of WROWS/16) covers rows 16i .. 16i+15 (64 B each)
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int i = wave * WPW + j;
    const int row = 16 * i + (lane >> 2);
    const int ls = (lane & 3) ^ nc_swz(row);
    const int ts = t0 - P.pad + row;
    const bool ok = row < BM + (K - 1) * P.dil && ts >= 0 && ts < P.T;
    const u16* src = ok ? P.a + ((int64_t)b * P.T + ts) * P.Cp + ls * 8 : reinterpret_cast<const u16*>(g_nconv_zero);
    const int cstep = ok ? 32 : 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) nc_glds16(src + c * cstep, wl + c * WBYTES + i * 1024);
  }
  // ---- weight step s -> ring buffer: DMA instruction g (of G per wave) covers 256 B = 4 rows of 64 B
  //      (plane-major: plane p rows n at p * BN * 64 + n * 64)
  const u16* bsrc[G];
  bool bok[G];
  int boff[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int byte = (wave * G + g) * 256 + lane * 4;  // byte offset inside the step tile
    const int p = byte / (BN * 64);
    const int rb = byte - p * BN * 64;
    const int n = rb >> 6;
    const int dw = (rb & 63) >> 2;                        // dword inside the row
    const int ls = (dw >> 2) ^ nc_swz(n);                 // logical 16-B slot
    bok[g] = n < P.N;
    bsrc[g] = P.w + (p ? P.w_lo : 0) + (int64_t)(bok[g] ? n : 0) * P.kpad + ls * 8 + (dw & 3) * 2;
    boff[g] = (wave * G + g) * 256;
  }
  auto stage_b = [&](int s, int buf) {
    const int c = s / K, tap = s - c * K;
    const int off = tap * P.Cp + c * 32;
#pragma unroll
    for (int g = 0; g < G; ++g)
      nc_glds4(bok[g] ? (const void*)(bsrc[g] + off) : (const void*)g_nconv_zero, bl + buf * SBYTES + boff[g]);
  };
#pragma unroll
  for (int s = 0; s < D; ++s) stage_b(s < nsteps ? s : nsteps - 1, s);
  // windows + weight step 0 landed; steps 1 .. D-1 stay in flight
  nc_vmcnt<(D - 1) * G>();

  // ACT tiles: residual of every tile row loaded into registers now, consumed by the epilogue
  constexpr int RPA = ACT ? (BM * (BN / 4) + 255) / 256 : 1;
  float4 rpa[RPA];
  const bool prea = ACT && P.res && P.act_prefetch;
  if (prea) {
    const int cq = P.N / 4;
#pragma unroll
    for (int i = 0; i < RPA; ++i) {
      const int e = tid + i * 256;
      const int m = e / cq, n = (e - m * cq) * 4;
      const int t = min(max(t0 + m, 0), P.T - 1);
      rpa[i] = *reinterpret_cast<const float4*>(P.res + ((int64_t)b * P.T + t) * P.N + (e < BM * cq ? n : 0));
    }
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow0 = wave * (BM / 4) + (lane & 15);
  const int bslot = (lane >> 4) ^ nc_swz(lane & 15);  // B rows n = 16j + (l & 15): swizzle of (l & 15)
  int c = 0, tap = 0;
  for (int s = 0; s < nsteps; ++s) {
    stage_b(s + D < nsteps ? s + D : nsteps - 1, (s + D) % NBUF);
    const int arow = arow0 + tap * P.dil;
    const char* ap = wl + c * WBYTES + arow * 64 + (((lane >> 4) ^ nc_swz(arow)) << 4);
    const char* bp = bl + (s % NBUF) * SBYTES + (lane & 15) * 64 + (bslot << 4);
    bf16x8 af[TM], bh[TN], blo[NPB == 2 ? TN : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ap + i * 16 * 64);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(bp + j * 16 * 64);
      if constexpr (NPB == 2) blo[j] = *reinterpret_cast<const bf16x8*>(bp + BN * 64 + j * 16 * 64);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (PREC == PREC_F16W2) {
          acc[i][j] = mfma16<PREC_F16>(af[i], blo[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_F16>(af[i], bh[j], acc[i][j]);
        } else {
          acc[i][j] = mfma16<PREC>(af[i], bh[j], acc[i][j]);
        }
      }
    if (++tap == K) {
      tap = 0;
      ++c;
    }
    nc_vmcnt<(D - 1) * G>();  // weight step s+1 landed (s+2 .. s+D in flight); step s's reads retired
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: v = conv + bias -> LDS tile
  float* ot = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wave * (BM / 4) + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + (lane & 15);
        ot[m * OTS + n] = acc[i][j][r] + ((P.bias && n < P.N) ? P.bias[n] : 0.f);
      }
    }
  __syncthreads();
  const int e_lo = t0 + P.tshift, e_hi = min(e_lo + P.tstride, P.T);
  const int cq = P.N / 4;
  if (prea) {
#pragma unroll
    for (int i = 0; i < RPA; ++i) {
      const int e = tid + i * 256;
      const int m = e / cq, n = (e - m * cq) * 4;
      const int t = t0 + m;
      if (e >= BM * cq || t < 0 || t >= P.T) continue;
      const int64_t go = ((int64_t)b * P.T + t) * P.N + n;
      float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
      v.x += rpa[i].x; v.y += rpa[i].y; v.z += rpa[i].z; v.w += rpa[i].w;
      *reinterpret_cast<float4*>(ot + m * OTS + n) = v;
      if (P.out && t >= e_lo && t < e_hi) {
        v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
        if (P.accumulate) {
          const float4 pv = *reinterpret_cast<const float4*>(P.out + go);
          v.x += pv.x; v.y += pv.y; v.z += pv.z; v.w += pv.w;
        }
        *reinterpret_cast<float4*>(P.out + go) = v;
      }
    }
  } else if (P.res || P.out) {
    // (+ res) for every tile row inside [0, T) (the activation reads halo rows); fp32 out for owned rows
    for (int e = tid; e < BM * cq; e += 256) {
      const int m = e / cq, n = (e - m * cq) * 4;
      const int t = t0 + m;
      if (t < 0 || t >= P.T || (!ACT && t >= e_hi)) continue;
      const int64_t go = ((int64_t)b * P.T + t) * P.N + n;
      float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
      if (P.res) {
        const float4 rv = *reinterpret_cast<const float4*>(P.res + go);
        v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        if (ACT) *reinterpret_cast<float4*>(ot + m * OTS + n) = v;
      }
      if (P.out && t >= e_lo && t < e_hi) {
        v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
        if (P.accumulate) {
          const float4 pv = *reinterpret_cast<const float4*>(P.out + go);
          v.x += pv.x; v.y += pv.y; v.z += pv.z; v.w += pv.w;
        }
        *reinterpret_cast<float4*>(P.out + go) = v;
      }
    }
  }
  if constexpr (ACT) {
    __syncthreads();
    // 240 emitted rows: R = 15 -> 16 runs x 12 pairs (C = 24) = one pass of the 256 threads
    act_epilogue_tile<PREC, (BM == 256 ? 15 : 14)>(ot, OTS, t0, e_lo, e_hi, P.T, P.act.Cp, 0, P.N, b, P.act, tid, 256);
  }
}

// Eligible: single-plane activations (F16 / F16W2 / BF16), N <= 96 with N % 4 == 0, Cp in {32, 64, 96},
// (k-1)d <= 64, no output activation.  Returns 1 when it launched.
int nconv_try(const alcm_opconv_args& a, const u16* wplane, const void* actepi, double flops, double bytes,
              hipStream_t s) {
  const int nck = knobs().nconv;  // diagnostics / A-B: ALCM_NCONV=0 uses opconv_kernel
  if (nck == 0) return 0;
  if (a.prec != PREC_F16 && a.prec != PREC_F16W2 && a.prec != PREC_BF16) return 0;
  if (a.out_act || a.N > 96 || a.N % 4 || (a.ksize - 1) * a.dil > NC_HALO) return 0;
  // measured (scripts/microbench.py tail): faster than opconv_kernel at C = 24 only (C = 48 / 96 pad or
  // lose occupancy); ALCM_NCONV=2 forces it for every narrow shape
  if (a.Cp != 32 && nck != 2) return 0;
  if (a.Cp != 32 && a.Cp != 64 && a.Cp != 96) return 0;
  auto al16 = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  if (!(al16(a.bias) && al16(a.res) && al16(a.out))) return 0;
  const bool act = actepi != nullptr;
  NConvDev P{};
  P.a = (const u16*)a.a;
  P.T = a.T; P.Cp = a.Cp; P.ksize = a.ksize; P.dil = a.dil; P.pad = a.pad;
  P.w = wplane; P.w_lo = a.w_lo_off; P.kpad = a.kpad; P.N = a.N;
  P.bias = a.bias; P.res = a.res; P.out = a.out; P.out_scale = a.out_scale; P.accumulate = a.accumulate;
  if (act) P.act = *reinterpret_cast<const ActEpiDev*>(actepi);
  P.act_prefetch = 1;
  // tile configurations (rows per tile, weight ring depth) sized for >= 2 workgroups per CU where the LDS
  // allows: C = 24 -> 256 x 32, 4 buffers (36 KB, 4 workgroups per CU); C = 48 -> 256 x 64, 4 buffers (72 KB);
  // C = 96 -> 128 x 96, 3 buffers (72 KB)
  int BM, BN, NB;
  if (a.N <= 32 && a.Cp == 32) BM = 256, BN = 32, NB = 4;
  else if (a.N <= 64 && a.Cp == 64) BM = 256, BN = 64, NB = 4;
  else if (a.N <= 96 && a.Cp == 96) BM = 128, BN = 96, NB = 3;
  else return 0;
  P.tstride = act ? BM - 2 * ACT_EPI_HALO : BM;
  P.tshift = act ? ACT_EPI_HALO : 0;
  P.tiles_per_batch = (a.T + P.tstride - 1) / P.tstride;
  const int64_t nwg = (int64_t)a.B * P.tiles_per_batch;
  if (nwg >= (1ll << 31)) return 0;
  void* tok = prof_start(s);
  const dim3 grid((unsigned)nwg), blk(256);
  auto go = [&](auto bm_c, auto bn_c, auto nch_c, auto nbuf_c) {
    constexpr int BMv = decltype(bm_c)::value, BNv = decltype(bn_c)::value;
    constexpr int NCH = decltype(nch_c)::value, NBUF = decltype(nbuf_c)::value;
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, grid, blk, 0, s, P); };
    if (act) {
      if (a.prec == PREC_F16W2) launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_F16W2, true>);
      else if (a.prec == PREC_F16) launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_F16, true>);
      else launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_BF16, true>);
    } else {
      if (a.prec == PREC_F16W2) launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_F16W2, false>);
      else if (a.prec == PREC_F16) launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_F16, false>);
      else launch(nconv_kernel<BMv, BNv, NCH, NBUF, PREC_BF16, false>);
    }
  };
  using std::integral_constant;
  if (BN == 32)
    go(integral_constant<int, 256>{}, integral_constant<int, 32>{}, integral_constant<int, 1>{}, integral_constant<int, 4>{});
  else if (BN == 64) go(integral_constant<int, 256>{}, integral_constant<int, 64>{}, integral_constant<int, 2>{}, integral_constant<int, 4>{});
  else go(integral_constant<int, 128>{}, integral_constant<int, 96>{}, integral_constant<int, 3>{}, integral_constant<int, 3>{});
  if (tok) {
    char name[112];  // the demangled rocprofv3 name of the instantiation
    std::snprintf(name, sizeof(name), "alcm::nconv_kernel<%d, %d, %d, %d, %d, %s>", BM, BN, a.Cp / 32, NB, a.prec,
                  act ? "true" : "false");
    prof_stop(tok, s, name, flops, bytes);
  }
  return 1;
}

}  // namespace alcm
