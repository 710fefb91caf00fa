// Split-precision (bf16x3) 1x1 conv / linear on operand planes: out[m][n] = sum_k A[m][k] W[n][k] (+ bias, + res),
// A and W each carried as bf16 hi + lo planes, products hi*hi + hi*lo + lo*hi with fp32 accumulation (~2^-16
// relative: fp32-reference parity).  Used for the DiT TemporalTransformer proj_in / proj_out (concatDiT.py:159-171,
// the GroupNorm affine applied once by split_planes when the planes are written) and the VAE 1x1 layers
// (autoencoder1d.py nin_shortcut / attention q,k,v / proj_out) under the split policy.
//
// Why not alcm_gemm.hip's gemm_kernel: it re-reads and re-normalises the fp32 A tile for every 128-column tile
// (5 at N = 576) with per-row statistics loads inside each 32-deep K step, and stages both operands through
// registers: 147 us per DiT proj launch (M = 14944, N = K = 576) against an MFMA floor of 12 us.
//
// Structure: 128 x 192 output tile, 4 waves as 2 (M) x 2 (N) of 64 x 96 (16x16x32 MFMAs), 32-deep K stages of
// both planes of both operands (16 + 24 KB) by LDS-DMA (global_load_lds) into a stage ring, two workgroups per CU;
// the epilogue stages 64-row halves of the tile through LDS for whole-row float4 residual loads and stores.
#include <cstdio>
#include <cstring>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"  // op_store2 / f32x2 (plane output)

namespace alcm {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

struct SGemmDev {
  const u16* a;  // [M][K] bf16 hi; lo at a + a_lo
  int64_t a_lo;
  const u16* w;  // [N][kpad] bf16 hi; lo at w + w_lo
  int64_t w_lo;
  int M, N, K, kpad;
  const float* bias;
  const float* res;  // [M][ldr] or null
  int64_t ldr;
  float* out;        // [M][ldo]
  int64_t ldo;
  float out_scale;
  int tiles_n, nwg;
  u16* oplane;       // single-plane kernel: acc + bias as a PREC operand plane [M][ldo] instead of out
};

constexpr int SG_BM = 128, SG_BN = 192;

__device__ __forceinline__ void sg_glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds, 16, 0, 0);
}

// KD-deep K stages of both planes of both operands are DMA'd NST - 1 stages ahead into an NST-stage ring; rows of
// KD * 2 bytes, the 16-B chunk kq of row r at slot kq ^ (r & 7) (KD 64) / kq ^ ((r >> 2) & 2) (KD 32): conflict-free
// ds_read_b128.  Built as KD 32, 2 stages, two workgroups per CU (80 KB each): against 3 stages at one per CU and
// against 64-deep stages (whole 128-B row segments) at one per CU, per step 1.69 vs 2.23 / 2.12 ms over the 120
// launches (DiT proj_in / proj_out 0.94 vs 1.26 / 1.21; bit-identical; +0.6 % end to end, profiles/r4m) — the DiT
// shape's 351 tiles then run in one round instead of 1.4, and the co-resident workgroup hides the DMA waits
//
// NPL = 1 (lin_plane_kernel): the same structure on ONE operand plane (PREC f16 / bf16, one MFMA per fragment pair) for
// the 1x1 convs / linears of the single-plane policies (DiT q,k,v and to_out, text-encoder linears): wconv2 stages its
// input window once per 64-channel chunk, which at k = 1 is every step, so each step waited out a full window DMA
// (68 us per DiT q,k,v launch against a 12 us MFMA floor); here 20 KB stages in a 4-deep ring keep three in flight.
// Same 32-deep slice order as wconv2, so the results are bit-identical to it.
template <int KD, int NST, int OCC, int NPL, int PREC>
__device__ __forceinline__ void sg_body(const SGemmDev& P) {
  constexpr int TM = 4, TN = 6;
  constexpr int RB = KD * 2;                  // LDS row bytes
  constexpr int AB = SG_BM * RB;              // one plane of the A stage
  constexpr int BB = SG_BN * RB;              // one plane of the B stage
  constexpr int STAGE = NPL * (AB + BB);      // 40 KB (two planes, KD 32)
  constexpr int RPI = 1024 / RB;              // rows per DMA instruction (16 / 8)
  constexpr int LPR = RB / 16;                // lanes per row (4 / 8)
  constexpr int AIW = SG_BM / RPI / 4;        // A instructions per plane per wave (2 / 4)
  constexpr int BIW = SG_BN / RPI / 4;        // B instructions per plane per wave (3 / 6)
  constexpr int DPW = NPL * (AIW + BIW);      // DMA instructions per wave per stage
  constexpr int SUB = KD / 32;                // 32-deep MFMA slices per stage
  static_assert(NST * STAGE <= 163840 / OCC, "LDS");
  static_assert((NST - 2) * DPW < 64, "vmcnt");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware order: consecutive work ids (the N tiles of one M tile: they share the A rows) on one XCD
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = P.nwg >> 3, r8 = P.nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int mt = wid / P.tiles_n, nt = wid - mt * P.tiles_n;
  const int m0 = mt * SG_BM, n0 = nt * SG_BN;
  auto swz = [](int kq, int r) { return KD == 64 ? kq ^ (r & 7) : kq ^ ((r >> 2) & 2); };

  // DMA sources: instruction i of a plane covers RPI rows x RB bytes; lane -> (row i * RPI + lane / LPR, slot lane % LPR)
  const int lr = lane / LPR, ps = lane % LPR;
  const u16* asrc[AIW];
#pragma unroll
  for (int j = 0; j < AIW; ++j) {
    const int r = (wave + 4 * j) * RPI + lr;
    asrc[j] = P.a + (int64_t)min(m0 + r, P.M - 1) * P.K + swz(ps, r) * 8;
  }
  const u16* bsrc[BIW];
#pragma unroll
  for (int j = 0; j < BIW; ++j) {
    const int r = (wave + 4 * j) * RPI + lr;
    bsrc[j] = P.w + (int64_t)(n0 + r) * P.kpad + swz(ps, r) * 8;
  }
  auto stage = [&](int ks, int buf) {
    char* base = smem + buf * STAGE;
    const int k0 = ks * KD;
#pragma unroll
    for (int j = 0; j < AIW; ++j) {
      sg_glds16(asrc[j] + k0, base + (wave + 4 * j) * 1024);
      if constexpr (NPL == 2) sg_glds16(asrc[j] + P.a_lo + k0, base + AB + (wave + 4 * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < BIW; ++j) {
      sg_glds16(bsrc[j] + k0, base + NPL * AB + (wave + 4 * j) * 1024);
      if constexpr (NPL == 2) sg_glds16(bsrc[j] + P.w_lo + k0, base + 2 * AB + BB + (wave + 4 * j) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = P.K / KD;
  // fragment geometry: lane reads row (lane & 15) of a 16-row block, chunk (4 sub + lane >> 4); 16-row blocks keep the
  // swizzle, so block i is + i * 16 rows
  const int fr = lane & 15, fq = lane >> 4;
  const int ar = wm * 64 + fr, br = wn * 96 + fr;
  // ring of NST stages, NST - 1 ahead
#pragma unroll
  for (int d = 0; d < NST - 1; ++d)
    if (d < nk) stage(d, d);
  if (nk > NST - 2 && NST > 2) __builtin_amdgcn_s_waitcnt(((NST - 2) * DPW & 15) | (7 << 4) | (((NST - 2) * DPW >> 4) << 14));
  else __builtin_amdgcn_s_waitcnt((7 << 4));  // vmcnt(0)
  __builtin_amdgcn_s_barrier();
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + NST - 1 < nk;
    if (more) stage(ks + NST - 1, (ks + NST - 1) % NST);
    const char* base = smem + (ks % NST) * STAGE;
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int aoff = ar * RB + (swz(4 * sb + fq, ar) << 4), boff = br * RB + (swz(4 * sb + fq, br) << 4);
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const bf16x8*>(base + aoff + i * 16 * RB);
        if constexpr (NPL == 2) al[i] = *reinterpret_cast<const bf16x8*>(base + AB + aoff + i * 16 * RB);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(base + NPL * AB + boff + j * 16 * RB);
        if constexpr (NPL == 2) bl[j] = *reinterpret_cast<const bf16x8*>(base + 2 * AB + BB + boff + j * 16 * RB);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (NPL == 2) {
            acc[i][j] = mfma16<PREC_BF16>(al[i], bh[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_BF16>(ah[i], bl[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_BF16>(ah[i], bh[j], acc[i][j]);
          } else {
            acc[i][j] = mfma16<PREC>(ah[i], bh[j], acc[i][j]);
          }
        }
      __builtin_amdgcn_s_setprio(0);
    }
    // stage ks + 1 has landed; younger stages stay in flight across the barrier
    if (more && NST > 2) __builtin_amdgcn_s_waitcnt(((NST - 2) * DPW & 15) | (7 << 4) | (((NST - 2) * DPW >> 4) << 14));
    else __builtin_amdgcn_s_waitcnt((7 << 4));  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: 64-row halves through LDS, whole 768-B row segments with float4 residual loads / stores
  constexpr int OTS = SG_BN + 4;
  float* ot = reinterpret_cast<float*>(smem);
  constexpr int CQ = SG_BN / 4;
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            ot[(i * 16 + fq * 4 + r) * OTS + wn * 96 + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    for (int e = tid; e < 64 * CQ; e += 256) {
      const int m = e / CQ, n = (e - m * CQ) * 4;
      const int gm = m0 + h * 64 + m;
      if (gm >= P.M) continue;
      float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
      if (P.bias) {
        const float4 bv = *reinterpret_cast<const float4*>(P.bias + n0 + n);
        v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
      }
      if constexpr (NPL == 1) {
        if (P.oplane) {  // (no residual / scale with a plane output, as wconv2)
          u16* d = P.oplane + (int64_t)gm * P.ldo + n0 + n;
          op_store2<PREC>(d, 0, f32x2{v.x, v.y});
          op_store2<PREC>(d + 2, 0, f32x2{v.z, v.w});
          continue;
        }
      }
      if (P.res) {
        const float4 rv = *reinterpret_cast<const float4*>(P.res + (int64_t)gm * P.ldr + n0 + n);
        v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
      }
      v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
      *reinterpret_cast<float4*>(P.out + (int64_t)gm * P.ldo + n0 + n) = v;
    }
    __syncthreads();
  }
}

template <int KD, int NST, int OCC>
__global__ __launch_bounds__(256, OCC) void sgemm_planes_kernel(const SGemmDev P) {
  sg_body<KD, NST, OCC, 2, PREC_BF16>(P);
}

template <int KD, int NST, int PREC>
__global__ __launch_bounds__(256, 2) void lin_plane_kernel(const SGemmDev P) {
  sg_body<KD, NST, 2, 1, PREC>(P);
}

// fp32 rows [rows][C] (optionally x * scale[b][c] + shift[b][c], b = row / T: a GroupNorm affine) -> bf16 hi plane
// [rows][C] and lo plane (x - hi) `lo` elements after it
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ x, int64_t n4, int C, int T,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, u16* __restrict__ y,
                                                           int64_t lo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int64_t e = i * 4;
  const int64_t row = e / C;
  const int c = (int)(e - row * C);
  float4 v = *reinterpret_cast<const float4*>(x + e);
  if (scale) {
    const int64_t bc = (row / T) * C + c;
    const float4 a = *reinterpret_cast<const float4*>(scale + bc), h = *reinterpret_cast<const float4*>(shift + bc);
    v.x = v.x * a.x + h.x; v.y = v.y * a.y + h.y; v.z = v.z * a.z + h.z; v.w = v.w * a.w + h.w;
  }
  const float f[4] = {v.x, v.y, v.z, v.w};
  u16 hh[4], ll[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 b = (__bf16)f[j];
    hh[j] = __builtin_bit_cast(u16, b);
    ll[j] = __builtin_bit_cast(u16, (__bf16)(f[j] - (float)b));
  }
  *reinterpret_cast<uint2*>(y + e) = make_uint2(hh[0] | ((uint32_t)hh[1] << 16), hh[2] | ((uint32_t)hh[3] << 16));
  *reinterpret_cast<uint2*>(y + lo + e) = make_uint2(ll[0] | ((uint32_t)ll[1] << 16), ll[2] | ((uint32_t)ll[3] << 16));
}

int split_planes(const float* x, int64_t rows, int C, int T, const float* scale, const float* shift, u16* y,
                 hipStream_t s) {
  if (!x || !y || rows <= 0 || C % 4 || (((uintptr_t)x) & 15) || (((uintptr_t)y) & 7) ||
      (scale && ((((uintptr_t)scale) & 15) || (((uintptr_t)shift) & 15) || T <= 0)))
    return set_error(ALCM_E_INVALID, "split_planes: bad arguments");
  const int64_t n4 = rows * C / 4;
  void* tok = prof_start(s);
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, x, n4, C,
                     T > 0 ? T : 1, scale, shift, y, rows * C);
  if (tok) prof_stop(tok, s, "alcm::split_planes_kernel", 0.0, (double)rows * C * 8.0);
  ALCM_HIP(hipGetLastError());
  return 0;
}

bool sgemm_planes_ok(int K, int N, int kpad) { return K % 32 == 0 && N % SG_BN == 0 && kpad >= K; }

// 1x1 conv / linear on one operand plane (ALCM_LIN1: 1 = 32-deep stages in a 4-deep ring, 2 = 64-deep stages double-
// buffered, 0 = off: wconv2, -1 = by shape: the 64-deep build for plane outputs only).  Measured per step at B = 32
// (gpurun_out/r4ag): DiT q,k,v (N = 1728, plane output) 1.04 ms on wconv2 -> 0.84 (ring) / 0.75 (64-deep); DiT
// to_out (N = 576, fp32 output + residual, one round of 351 tiles, bound by its epilogue) 0.55 -> 0.62 / 0.60.
// Eligible: f16 / bf16, k = 1 without padding, Cp % 32 == 0, N % 192 == 0, no GEGLU / strided / activated /
// accumulated output.  Returns 1 when it launched.
int lin_plane_try(const alcm_opconv_args& a, const u16* wplane, double flops, double bytes, hipStream_t s) {
  int v = knobs().lin1;
  if (v < 0) {
    if (!a.out_plane) return 0;
    v = 2;
  }
  if (v == 0 || (a.prec != PREC_F16 && a.prec != PREC_BF16)) return 0;
  if (a.ksize != 1 || a.pad != 0 || a.out_stride > 0 || a.geglu_plane || a.out_act || a.accumulate || a.Cp % 32 ||
      a.N % SG_BN || a.kpad < a.Cp || a.kpad % 8)
    return 0;
  if (a.out_plane ? (a.out || a.res) : !a.out) return 0;
  auto al16 = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  if (!al16(a.a) || !al16(wplane) || !al16(a.bias) || !al16(a.res) || !al16(a.out) || (((uintptr_t)a.out_plane) & 7))
    return 0;
  const int64_t M = (int64_t)a.B * a.T;
  const int64_t nwg = (M + SG_BM - 1) / SG_BM * (a.N / SG_BN);
  if (M >= (1ll << 31) || nwg >= (1ll << 30) || M * a.N >= (1ll << 40)) return 0;
  SGemmDev P{};
  P.a = (const u16*)a.a; P.w = wplane;
  P.M = (int)M; P.N = a.N; P.K = a.Cp; P.kpad = a.kpad;
  P.bias = a.bias; P.res = a.res; P.ldr = a.N; P.out = a.out; P.ldo = a.N; P.out_scale = a.out_scale;
  P.oplane = (u16*)a.out_plane;
  P.tiles_n = a.N / SG_BN;
  P.nwg = (int)nwg;
  void* tok = prof_start(s);
  const bool f16 = a.prec == PREC_F16;
  const bool deep = v == 2 && a.Cp % 64 == 0;
  if (deep) {
    if (f16) hipLaunchKernelGGL((lin_plane_kernel<64, 2, PREC_F16>), dim3((unsigned)nwg), dim3(256), 0, s, P);
    else hipLaunchKernelGGL((lin_plane_kernel<64, 2, PREC_BF16>), dim3((unsigned)nwg), dim3(256), 0, s, P);
  } else {
    if (f16) hipLaunchKernelGGL((lin_plane_kernel<32, 4, PREC_F16>), dim3((unsigned)nwg), dim3(256), 0, s, P);
    else hipLaunchKernelGGL((lin_plane_kernel<32, 4, PREC_BF16>), dim3((unsigned)nwg), dim3(256), 0, s, P);
  }
  if (tok) {
    char name[96];
    std::snprintf(name, sizeof(name), "alcm::lin_plane_kernel<%d, %d, %d>", deep ? 64 : 32, deep ? 2 : 4, a.prec);
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " M%d N%d K%d", P.M, a.N, a.Cp);
    prof_stop(tok, s, name, flops, bytes);
  }
  ALCM_HIP(hipGetLastError());
  return 1;
}


int sgemm_planes(const u16* a, int64_t a_lo, int M, int K, const u16* w, int64_t w_lo, int kpad, int N,
                 const float* bias, const float* res, int64_t ldr, float* out, int64_t ldo, float out_scale,
                 hipStream_t s) {
  if (!a || !w || !out || M <= 0 || !sgemm_planes_ok(K, N, kpad))
    return set_error(ALCM_E_INVALID, "sgemm_planes: needs K % 32 == 0, N % 192 == 0");
  auto al16 = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  if (!al16(a) || !al16(w) || (a_lo % 8) || (w_lo % 8) || (kpad % 8) || !al16(out) || ldo % 4 ||
      (res && (!al16(res) || ldr % 4)) || (bias && !al16(bias)))
    return set_error(ALCM_E_INVALID, "sgemm_planes: alignment");
  SGemmDev P{};
  P.a = a; P.a_lo = a_lo; P.w = w; P.w_lo = w_lo;
  P.M = M; P.N = N; P.K = K; P.kpad = kpad;
  P.bias = bias; P.res = res; P.ldr = ldr; P.out = out; P.ldo = ldo; P.out_scale = out_scale;
  P.tiles_n = N / SG_BN;
  const int64_t nwg = (int64_t)((M + SG_BM - 1) / SG_BM) * P.tiles_n;
  if (nwg >= (1ll << 30)) return set_error(ALCM_E_INVALID, "sgemm_planes: problem too large");
  P.nwg = (int)nwg;
  void* tok = prof_start(s);
  hipLaunchKernelGGL((sgemm_planes_kernel<32, 2, 2>), dim3((unsigned)nwg), dim3(256), 0, s, P);
  if (tok) {
    char name[96];
    std::snprintf(name, sizeof(name), "alcm::sgemm_planes_kernel<32, 2, 2>");
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " M%d N%d K%d", M, N, K);
    const double flops = 2.0 * M * N * (double)K;
    const double bytes = (double)M * K * 4.0 + (double)N * K * 4.0 + (double)M * N * 4.0 * (res ? 2 : 1);
    prof_stop(tok, s, name, flops, bytes);
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm
