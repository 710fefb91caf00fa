// Fused multi-head self-attention for the DiT (CrossAttention used as self-attention,
// ldm/modules/new_attention.py:89-130): O = softmax(Q K^T * dh^-1/2) V per (batch, head), with the
// scores kept on chip (flash-attention style online softmax) instead of an (L x L) round trip through HBM.
//
// gfx950 layout (16x16x32 MFMAs, 64-lane waves, fp32 accumulation):
//   * a workgroup = 4 waves = 64 queries of one (b, head); each wave owns 16 queries;
//   * scores are computed transposed, S^T = K Q^T (A = K tile from LDS, B = the wave's Q fragments held in
//     registers), so a lane's accumulators all belong to ONE query (column lane & 15): the running max /
//     sum of the online softmax need only a 4-lane reduction (lanes l, l^16, l^32, l^48);
//   * O^T = V^T P^T reuses the S^T accumulators directly as the B operand: the 8 keys a lane holds for a
//     32-key slice are {4g..4g+3, 16+4g..16+4g+3} (g = lane >> 4) instead of 8g..8g+7, and the A operand
//     (V^T from LDS) is read with the same key permutation, so P never moves between lanes;
//   * K and V^T tiles (64 keys) are converted from the fp32 qkv rows to the MFMA operand format while they
//     are staged into LDS (padded row strides: conflict-free fragment reads).
// Operands are rounded to fp16 (PREC_F16) or bf16 (PREC_BF16) exactly as the GEMM path rounds them; the
// probabilities are rounded after the exp (unnormalised, in (0, 1]) and the 1/l normalisation is applied
// to the fp32 output.
#include <cmath>
#include <cstdio>
#include <type_traits>

#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

constexpr int FA_Q = 64;       // queries per workgroup
constexpr int FA_KT = 64;      // keys per tile
constexpr int FA_DK = 96;      // head dim padded for the QK^T contraction (3 x 32)
constexpr int FA_DV = 80;      // head dim padded for the PV output rows (5 x 16)
constexpr int FA_KS = 104;     // K tile row stride (elements): 208 B
constexpr int FA_VS = 68;      // V^T tile row stride (elements): 136 B

template <int PREC>
__device__ __forceinline__ u16 fa_cvt(float v) {
  if constexpr (PREC == PREC_F16) return __builtin_bit_cast(u16, (_Float16)v);
  else return __builtin_bit_cast(u16, (__bf16)v);
}

template <int PREC>
__global__ __launch_bounds__(256) void flash_attn_kernel(const float* __restrict__ qkv, float* __restrict__ O,
                                                         u16* __restrict__ Op, int L, int H, int nh, int dh,
                                                         float scale) {
  __shared__ __attribute__((aligned(16))) u16 Ks[FA_KT * FA_KS];
  __shared__ __attribute__((aligned(16))) u16 Vt[FA_DV * FA_VS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, cq = lane & 15;
  // XCD-aware order (1-D grid of nqt * B * nh workgroups, dispatched round-robin over the 8 XCDs): each XCD takes a
  // contiguous block of work ids, so the query tiles of one (b, head) share that XCD's L2 copy of its K / V
  const int nwg = (int)gridDim.x, nqt = (L + FA_Q - 1) / FA_Q;
  const int orig = blockIdx.x, xcd = orig & 7, qx = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (qx + 1) : r8 * (qx + 1) + (xcd - r8) * qx) + (orig >> 3);
  const int z = wid / nqt, b = z / nh, h = z - b * nh;
  const int q0 = (wid - z * nqt) * FA_Q + wave * 16;
  const int64_t rs = 3 * (int64_t)H;  // qkv row stride
  const float* base = qkv + (int64_t)b * L * rs + h * dh;

  // Q fragments (B operand of S^T): lane holds Q[q0 + cq][32 ks + 8 g .. + 7]
  bf16x8 qf[3];
  {
    const int q = q0 + cq;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      u16 e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 32 * ks + 8 * g + j;
        e[j] = fa_cvt<PREC>((q < L && d < dh) ? base[(int64_t)q * rs + d] : 0.f);
      }
      qf[ks] = __builtin_bit_cast(bf16x8, e);
    }
  }
  f32x4 o[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const int nkt = (L + FA_KT - 1) / FA_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FA_KT;
    __syncthreads();  // previous tile's fragment reads retired
    // stage K [key][dim] and V^T [dim][key] (zero padding beyond L / dh)
    for (int e = tid; e < FA_KT * (FA_DK / 4); e += 256) {
      const int kr = e / (FA_DK / 4), d4 = (e - kr * (FA_DK / 4)) * 4;
      const int key = k0 + kr;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (key < L && d4 < dh) {
        const float* r = base + (int64_t)key * rs + d4;
        kv = *reinterpret_cast<const float4*>(r + H);
        vv = *reinterpret_cast<const float4*>(r + 2 * H);
      }
      uint2 kp;
      kp.x = (uint32_t)fa_cvt<PREC>(kv.x) | ((uint32_t)fa_cvt<PREC>(kv.y) << 16);
      kp.y = (uint32_t)fa_cvt<PREC>(kv.z) | ((uint32_t)fa_cvt<PREC>(kv.w) << 16);
      *reinterpret_cast<uint2*>(&Ks[kr * FA_KS + d4]) = kp;
      if (d4 < FA_DV) {
        Vt[(d4 + 0) * FA_VS + kr] = fa_cvt<PREC>(vv.x);
        Vt[(d4 + 1) * FA_VS + kr] = fa_cvt<PREC>(vv.y);
        Vt[(d4 + 2) * FA_VS + kr] = fa_cvt<PREC>(vv.z);
        Vt[(d4 + 3) * FA_VS + kr] = fa_cvt<PREC>(vv.w);
      }
    }
    __syncthreads();
    // S^T block kb: rows = keys 16 kb + (4g + r), column = query cq
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[(16 * kb + cq) * FA_KS + 32 * ks + 8 * g]);
        s[kb] = mfma16<PREC>(kf, qf[ks], s[kb]);
      }
    }
    // online softmax over this tile's keys (per query = per lane column)
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * kb + 4 * g + r;
        const float v = key < L ? s[kb][r] * scale : -INFINITY;
        s[kb][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);  // 0 on the first tile (m = -inf)
    m = mn;
    float psum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[kb][r] - mn);
        s[kb][r] = p;
        psum += p;
      }
    l = l * alpha + psum;
#pragma unroll
    for (int i = 0; i < 5; ++i) o[i] *= alpha;
    // O^T += V^T P^T over two 32-key slices
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u16 pe[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pe[r] = fa_cvt<PREC>(s[2 * ks][r]);
        pe[4 + r] = fa_cvt<PREC>(s[2 * ks + 1][r]);
      }
      const bf16x8 pf = __builtin_bit_cast(bf16x8, pe);
#pragma unroll
      for (int db = 0; db < 5; ++db) {
        const u16* vr = &Vt[(16 * db + cq) * FA_VS + 32 * ks + 4 * g];
        const uint2 lo = *reinterpret_cast<const uint2*>(vr);
        const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
        const uint4 vv = make_uint4(lo.x, lo.y, hi.x, hi.y);
        o[db] = mfma16<PREC>(__builtin_bit_cast(bf16x8, vv), pf, o[db]);
      }
    }
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  const int q = q0 + cq;
  if (q >= L) return;
  const float inv = 1.0f / l;
  const int64_t ob = ((int64_t)b * L + q) * H + h * dh;
  if (Op) {  // operand plane for the to_out projection (the same rounding its GEMM would apply)
#pragma unroll
    for (int db = 0; db < 5; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * db + 4 * g + r;
        if (d < dh) Op[ob + d] = fa_cvt<PREC>(o[db][r] * inv);
      }
    return;
  }
#pragma unroll
  for (int db = 0; db < 5; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * db + 4 * g + r;
      if (d < dh) O[ob + d] = o[db][r] * inv;
    }
}


// Resident-K/V form (L <= FR_MAXL): one workgroup of 16 waves per (b, head) stages the head's whole K and V^T
// once (fp32 -> operand format, 157 KB of LDS at L = 512) and every wave then walks its 16-query blocks over
// all key tiles with no further barrier.  The tiled kernel above re-reads K/V from HBM once per 64-query
// workgroup (8x at L = 467); here each head's K/V leave HBM once, and B * heads workgroups (256 at B = 32)
// fill the 256 CUs one per CU.  Same arithmetic and rounding as the tiled kernel (identical per-tile sums).
constexpr int FR_MAXL = 512;   // keys padded to a multiple of 64
constexpr int FR_KS = 80;      // K row stride (elements, 160 B): conflict-free ds_read_b128; dims dh..79 zero
constexpr int FR_MAXDH = 72;
constexpr int FR_THREADS = 1024;  // 16 waves: 4 per SIMD hide the per-tile softmax / LDS latency chain
// (round 4: scores in the log2 domain (q pre-scaled), exp2 straight to v_exp_f32, masking only in the last key tile,
// the running-output rescale skipped when no query's max moved)

// qkv element idx as fp32: from fp32 rows, or (QH) from PREC operand rows (the DiT q/k/v projection's plane output)
template <int PREC, bool QH>
__device__ __forceinline__ float fa_ld(const void* qkv, int64_t idx) {
  if constexpr (!QH) {
    return reinterpret_cast<const float*>(qkv)[idx];
  } else {
    const u16 v = reinterpret_cast<const u16*>(qkv)[idx];
    if constexpr (PREC == PREC_F16) return (float)__builtin_bit_cast(_Float16, v);
    else return __builtin_bit_cast(float, (uint32_t)v << 16);
  }
}
template <int PREC, bool QH>
__device__ __forceinline__ float4 fa_ld4(const void* qkv, int64_t idx) {
  if constexpr (!QH) {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(qkv) + idx);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const u16*>(qkv) + idx);
    auto cv = [](uint32_t h) -> float {
      if constexpr (PREC == PREC_F16) return (float)__builtin_bit_cast(_Float16, (u16)h);
      else return __builtin_bit_cast(float, h << 16);
    };
    return make_float4(cv(u.x & 0xffffu), cv(u.x >> 16), cv(u.y & 0xffffu), cv(u.y >> 16));
  }
}

template <int PREC, bool BIAS, bool QH>
__global__ __launch_bounds__(FR_THREADS) void flash_attn_res_kernel(const void* __restrict__ qkv, float* __restrict__ O,
                                                             u16* __restrict__ Op, int L, int Lp, int H, int nh,
                                                             int dh, float scale, const float* __restrict__ bias,
                                                             int bld) {
  __shared__ __attribute__((aligned(16))) u16 Ks[FR_MAXL * FR_KS];
  __shared__ __attribute__((aligned(16))) u16 Vt[FR_MAXDH * (FR_MAXL + 8)];
  const int VS = Lp + 8;  // V^T row stride: (VS * 2 / 4) mod 64 = 4 * odd -> conflict-free ds_read_b64
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, cq = lane & 15;
  const int z = blockIdx.x, b = z / nh, h = z - b * nh;
  const int64_t rs = 3 * (int64_t)H;
  const int64_t base = (int64_t)b * L * rs + h * dh;  // element offset of this (clip, head)

  // stage K [key][dim] (dims >= dh and keys >= L zero) and V^T [dim][key] (keys >= L zero); 8 items per thread
  // per round so 16 float4 loads are in flight per lane (the staging phase is HBM-latency bound otherwise)
  constexpr int FU = 5;
  const int nitem = Lp * (FR_KS / 4);
  for (int e0 = tid; e0 < nitem; e0 += FR_THREADS * FU) {
    float4 kv[FU], vv[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int e = e0 + FR_THREADS * u;
      const int kr = e / (FR_KS / 4), d4 = (e - kr * (FR_KS / 4)) * 4;
      kv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      vv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nitem && kr < L && d4 < dh) {
        const int64_t r = base + (int64_t)kr * rs + d4;
        kv[u] = fa_ld4<PREC, QH>(qkv, r + H);
        vv[u] = fa_ld4<PREC, QH>(qkv, r + 2 * H);
      }
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int e = e0 + FR_THREADS * u;
      if (e >= nitem) break;
      const int kr = e / (FR_KS / 4), d4 = (e - kr * (FR_KS / 4)) * 4;
      uint2 kp;
      kp.x = (uint32_t)fa_cvt<PREC>(kv[u].x) | ((uint32_t)fa_cvt<PREC>(kv[u].y) << 16);
      kp.y = (uint32_t)fa_cvt<PREC>(kv[u].z) | ((uint32_t)fa_cvt<PREC>(kv[u].w) << 16);
      *reinterpret_cast<uint2*>(&Ks[kr * FR_KS + d4]) = kp;
      if (d4 < dh) {
        Vt[(d4 + 0) * VS + kr] = fa_cvt<PREC>(vv[u].x);
        Vt[(d4 + 1) * VS + kr] = fa_cvt<PREC>(vv[u].y);
        Vt[(d4 + 2) * VS + kr] = fa_cvt<PREC>(vv[u].z);
        Vt[(d4 + 3) * VS + kr] = fa_cvt<PREC>(vv[u].w);
      }
    }
  }
  __syncthreads();

  const int nqb = (L + 15) / 16, nkt = Lp / FA_KT;
  // scores scaled by scale * log2(e) in fp32 after the MFMA (the log2 domain: p = exp2(s - m) is one v_exp_f32); q is
  // rounded to the operand format unscaled (from a plane: exactly as stored), so the scale costs no second rounding
  // and no fp16 range (T5's scores are unscaled)
  const float qs = scale * 1.44269504088896341f;
  for (int qb = wave; qb < nqb; qb += FR_THREADS / 64) {
    const int q0 = qb * 16;
    // (branch-free: clamped addresses and selects; exec-masked loads inside this loop serialise it)
    bf16x8 qf[3];
    {
      const int q = q0 + cq;
      const bool qok = q < L;
      const int64_t qr = base + (int64_t)(qok ? q : 0) * rs;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        u16 e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int d = 32 * ks + 8 * g + j;
          const float v = fa_ld<PREC, QH>(qkv, qr + (d < dh ? d : 0));
          e[j] = fa_cvt<PREC>((qok && d < dh) ? v : 0.f);
        }
        qf[ks] = __builtin_bit_cast(bf16x8, e);
      }
    }
    // K fragment offsets: dims 32 ks + 8 g .. + 7; the slices beyond the 80-element row (ks = 2, g >= 2) read
    // the zero dims 72 .. 79 instead
    int koff[3];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) koff[ks] = (32 * ks + 8 * g < FR_KS) ? 32 * ks + 8 * g : FR_MAXDH;
    // V^T rows >= dh read row dh - 1 and are masked to zero
    int vrow[5];
    uint32_t vmask[5];
#pragma unroll
    for (int db = 0; db < 5; ++db) {
      const int r = 16 * db + cq;
      vrow[db] = (r < dh ? r : dh - 1) * VS;
      vmask[db] = r < dh ? 0xffffffffu : 0u;
    }
    f32x4 o[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    for (int kt = 0; kt < nkt; ++kt) {
      const int k0 = kt * FA_KT;
      f32x4 s[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[(k0 + 16 * kb + cq) * FR_KS + koff[ks]]);
          s[kb] = mfma16<PREC>(kf, qf[ks], s[kb]);
        }
        s[kb] *= qs;
      }
      if constexpr (BIAS) {  // additive score bias [head][query][key] (T5's relative positions), into the log2 domain too
        const float* br = bias + ((int64_t)h * bld + min(q0 + cq, L - 1)) * bld;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + 16 * kb + 4 * g + r;
            s[kb][r] += br[min(key, L - 1)] * 1.44269504088896341f;
          }
      }
      if (k0 + FA_KT > L) {  // (wave-uniform) only the last tile has keys >= L
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + 16 * kb + 4 * g + r;
            s[kb][r] = key < L ? s[kb][r] : -INFINITY;
          }
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[kb][r]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mn = fmaxf(m, tmax);
      // rescale only when some query's running max moved (wave-uniform branch; lanes whose max did not move
      // scale by exactly 1)
      if (__any(mn != m)) {
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] *= alpha;
        m = mn;
      }
      float psum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(s[kb][r] - m);
          s[kb][r] = pv;
          psum += pv;
        }
      l += psum;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u16 pe[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pe[r] = fa_cvt<PREC>(s[2 * ks][r]);
          pe[4 + r] = fa_cvt<PREC>(s[2 * ks + 1][r]);
        }
        const bf16x8 pf = __builtin_bit_cast(bf16x8, pe);
#pragma unroll
        for (int db = 0; db < 5; ++db) {
          const u16* vr = &Vt[vrow[db] + k0 + 32 * ks + 4 * g];
          const uint2 lo = *reinterpret_cast<const uint2*>(vr);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
          const uint32_t mk = vmask[db];
          const uint4 vv = make_uint4(lo.x & mk, lo.y & mk, hi.x & mk, hi.y & mk);
          o[db] = mfma16<PREC>(__builtin_bit_cast(bf16x8, vv), pf, o[db]);
        }
      }
    }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const int q = q0 + cq;
    if (q >= L) continue;
    const float inv = 1.0f / l;
    const int64_t ob = ((int64_t)b * L + q) * H + h * dh;
    if (Op) {
#pragma unroll
      for (int db = 0; db < 5; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = 16 * db + 4 * g + r;
          if (d < dh) Op[ob + d] = fa_cvt<PREC>(o[db][r] * inv);
        }
    } else {
#pragma unroll
      for (int db = 0; db < 5; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = 16 * db + 4 * g + r;
          if (d < dh) O[ob + d] = o[db][r] * inv;
        }
    }
  }
}

// qkv: (B, L, 3H) fp32 rows [q | k | v], head h at columns h*dh; O: (B, L, H) fp32
int flash_attention(const float* qkv, float* O, int B, int L, int H, int nh, int prec, hipStream_t s, void* o_plane,
                    const float* bias, int bld, float scale_in, const void* qkv_plane) {
  if (qkv_plane) {  // q / k / v as PREC operand rows: the resident-K/V kernel only
    const int Lp = (L + FA_KT - 1) / FA_KT * FA_KT;
    const int dh = nh > 0 ? H / nh : 0;
    if (qkv || (!O && !o_plane) || B <= 0 || L <= 0 || nh <= 0 || H % nh || dh > FR_MAXDH || dh % 4 || Lp > FR_MAXL ||
        (prec != PREC_F16 && prec != PREC_BF16) || (((uintptr_t)qkv_plane) & 7) ||
        (bias && bld < L))
      return set_error(ALCM_E_INVALID, "flash_attention: bad plane-input arguments");
    const float scale = scale_in > 0.f ? scale_in : 1.0f / std::sqrt((float)dh);
    void* tok = prof_start(s);
    auto kern = prec == PREC_F16
                    ? (bias ? flash_attn_res_kernel<PREC_F16, true, true> : flash_attn_res_kernel<PREC_F16, false, true>)
                    : (bias ? flash_attn_res_kernel<PREC_BF16, true, true> : flash_attn_res_kernel<PREC_BF16, false, true>);
    hipLaunchKernelGGL(kern, dim3((unsigned)(B * nh)), dim3(FR_THREADS), 0, s, qkv_plane, O, (u16*)o_plane, L, Lp, H, nh,
                       dh, scale, bias, bld);
    if (tok) {
      char name[80];
      std::snprintf(name, sizeof(name), "alcm::flash_attn_res_kernel<%d, %s, true>", prec, bias ? "true" : "false");
      const double z = (double)B * nh;
      prof_stop(tok, s, name, z * 4.0 * L * (double)L * dh, (double)B * L * (3.0 * H * 2.0 + H * 2.0));
    }
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  if (!qkv || (!O && !o_plane) || B <= 0 || L <= 0 || nh <= 0 || H % nh) return set_error(ALCM_E_INVALID, "flash_attention: bad args");
  const int dh = H / nh;
  if (dh > 72 || dh % 4 || H % 4) return set_error(ALCM_E_INVALID, "flash_attention: head dim must be <= 72, % 4");
  if (prec != PREC_F16 && prec != PREC_BF16) return set_error(ALCM_E_INVALID, "flash_attention: F16 or BF16 only");
  if (((uintptr_t)qkv) & 15) return set_error(ALCM_E_INVALID, "flash_attention: qkv must be 16-byte aligned");
  const float scale = scale_in > 0.f ? scale_in : 1.0f / std::sqrt((float)dh);
  if (bias && bld < L) return set_error(ALCM_E_INVALID, "flash_attention: bias pitch < L");
  const int Lp = (L + FA_KT - 1) / FA_KT * FA_KT;
  if (Lp <= FR_MAXL && dh <= FR_MAXDH && (int64_t)B * nh < (1ll << 31)) {
    void* tok = prof_start(s);
    const dim3 grid((unsigned)(B * nh));
    auto kern = prec == PREC_F16
                    ? (bias ? flash_attn_res_kernel<PREC_F16, true, false> : flash_attn_res_kernel<PREC_F16, false, false>)
                    : (bias ? flash_attn_res_kernel<PREC_BF16, true, false> : flash_attn_res_kernel<PREC_BF16, false, false>);
    hipLaunchKernelGGL(kern, grid, dim3(FR_THREADS), 0, s, qkv, O, (u16*)o_plane, L, Lp, H, nh, dh, scale, bias, bld);
    if (tok) {
      char name[64];
      std::snprintf(name, sizeof(name), "alcm::flash_attn_res_kernel<%d, %s, false>", prec, bias ? "true" : "false");
      const double z = (double)B * nh;
      prof_stop(tok, s, name, z * 4.0 * L * (double)L * dh, (double)B * L * (3.0 * H + H) * 4.0);
    }
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  if (bias || scale_in > 0.f) return set_error(ALCM_E_INVALID, "flash_attention: score bias / scale only for L <= 512");
  const int64_t nwg = (int64_t)((L + FA_Q - 1) / FA_Q) * B * nh;
  if (nwg >= (1ll << 31)) return set_error(ALCM_E_INVALID, "flash_attention: problem too large");
  const dim3 grid((unsigned)nwg);
  void* tok = prof_start(s);
  if (prec == PREC_F16)
    hipLaunchKernelGGL(flash_attn_kernel<PREC_F16>, grid, dim3(256), 0, s, qkv, O, (u16*)o_plane, L, H, nh, dh, scale);
  else
    hipLaunchKernelGGL(flash_attn_kernel<PREC_BF16>, grid, dim3(256), 0, s, qkv, O, (u16*)o_plane, L, H, nh, dh, scale);
  if (tok) {
    char name[64];
    std::snprintf(name, sizeof(name), "alcm::flash_attn_kernel<%d>", prec);
    const double z = (double)B * nh;
    prof_stop(tok, s, name, z * 4.0 * L * (double)L * dh, (double)B * L * (3.0 * H + H) * 4.0);
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm

extern "C" int alcm_flash_attention(const float* qkv, float* out, int B, int L, int H, int heads, int prec,
                                    alcm_stream_t stream) {
  return alcm::flash_attention(qkv, out, B, L, H, heads, prec, (hipStream_t)stream);
}
