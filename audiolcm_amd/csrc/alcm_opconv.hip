// Operand-format path of the BigVGAN AMPBlock convolutions (gfx950).
//
// An AMPBlock1 half-layer (vocoder/bigvgan/models.py:72-81) is  y = conv_{k,d}(Activation1d(x)) + b.
// Here it runs as two kernels:
//   activation1d_op Activation1d (alias_free_torch/act.py:23-27: up-FIR x2 -> SnakeBeta -> down-FIR)
//                   of the fp32 (B, T, C) tensor, written straight in MFMA operand format: fp16, or
//                   bf16 hi/lo planes for the bf16x3 split, channels padded to Cp = round_up(C, 32)
//                   (act_mfma_kernel / act_coop_kernel in alcm_act.hip);
//   opconv_kernel   implicit-GEMM conv1d on those planes: per 32-channel chunk the input window
//                   rows [t0 - pad, t0 + BM + (k-1)d - pad) are copied once into LDS (double-buffered
//                   across chunks) and reused by all k taps; the packed weight tile of each (chunk, tap)
//                   step is prefetched two steps ahead through registers into a double-buffered LDS
//                   tile, so the L2 latency of the weight stream hides behind two steps of MFMAs.
// Against the fp32 conv path this halves the conv's A-operand bytes and removes its fp32->bf16
// conversions; against the fused narrow-stage kernel (alcm_ampconv.hip) it trades one 2-byte
// round trip of the activation for a K loop free of activation work.
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

int act_coop(const float* x, void* const* y, int nset, int B, int T, int C, int Cp, const float* const* alpha_exp,
             const float* const* inv_beta, const Taps12O& f, int prec, hipStream_t s);

// three Activation1d of one input with their own SnakeBeta parameters and the same FIR taps (a BigVGAN stage's three
// resblocks' first half-layer): one cooperative pass, the input window loaded once (bit-identical to three calls)
int activation1d_x3(const float* x, void* const y[3], int B, int T, int C, int Cp, const float* const alpha_exp[3],
                    const float* const inv_beta[3], const float* up_filter, const float* down_filter, int prec,
                    hipStream_t s) {
  if (!x || !y[0] || !y[1] || !y[2] || !up_filter || !down_filter || B <= 0 || T <= 0 || C <= 0 || C % 2 ||
      Cp < C || Cp % 32 || prec < PREC_BF16 || prec > PREC_F16W2 || (((uintptr_t)x) & 7))
    return set_error(ALCM_E_INVALID, "activation1d_x3: bad arguments");
  for (int i = 0; i < 3; ++i)
    if (!alpha_exp[i] || !inv_beta[i] || (((uintptr_t)y[i]) & 3)) return set_error(ALCM_E_INVALID, "activation1d_x3: bad arguments");
  if ((int64_t)B * T * Cp >= (1ll << 40)) return set_error(ALCM_E_INVALID, "activation1d_x3: problem too large");
  Taps12O f;
  for (int k = 0; k < 12; ++k) {
    f.up[k] = 2.0f * up_filter[k];
    f.dn[k] = down_filter[k];
  }
  void* tok = prof_start(s);
  // the wide stages' MFMA FIR kernel where it applies (its fp16 FIR inputs: the mixed policy's stages 0-2)
  const bool am = knobs().act_x3_mfma && act_mfma_ok(C, Cp, prec) && !(((uintptr_t)x) & 15) &&
                  !(((uintptr_t)y[0]) & 15) && !(((uintptr_t)y[1]) & 15) && !(((uintptr_t)y[2]) & 15);
  if (am) ALCM_TRY(act_mfma3(x, y, B, T, C, Cp, alpha_exp, inv_beta, f, s));
  else ALCM_TRY(act_coop(x, y, 3, B, T, C, Cp, alpha_exp, inv_beta, f, prec, s));
  if (tok) {
    char name[64];
    if (am) std::snprintf(name, sizeof(name), "alcm::act_mfma3_kernel<64>");
    else std::snprintf(name, sizeof(name), "alcm::act_coop_kernel<%d>, x3", prec == PREC_F16W2 ? PREC_F16 : prec);
    const double e = (double)B * T;
    prof_stop(tok, s, name, 3 * 2.0 * 36.0 * e * C, e * (4.0 * C + 3 * 2.0 * Cp * (prec == PREC_SPLIT ? 2 : 1)));
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

// Activation1d of an fp16 plane (the wide-stage AMPBlock conv1 written by alcm_opconv's out_plane epilogue): only
// the MFMA kernel's shapes, whose FIR input is that fp16 value anyway (bit-identical to the fp32-input call on the
// conv's fp32 output)
int activation1d_op_h16(const void* x16, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                        const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                        hipStream_t s) {
  if (!x16 || !y || !alpha_exp || !inv_beta || !up_filter || !down_filter || B <= 0 || T <= 0 || C <= 0)
    return set_error(ALCM_E_INVALID, "activation1d_op_f16in: bad arguments");
  if (!act_mfma_ok(C, Cp, prec) || (((uintptr_t)x16) & 15) || (((uintptr_t)y) & 15))
    return set_error(ALCM_E_INVALID, "activation1d_op_f16in: needs prec F16, C >= 192, C % 64 == 0, Cp == C and "
                                     "16-byte aligned x / y");
  Taps12O f;
  for (int k = 0; k < 12; ++k) {
    f.up[k] = 2.0f * up_filter[k];
    f.dn[k] = down_filter[k];
  }
  void* tok = prof_start(s);
  ALCM_TRY(act_mfma(x16, true, y, B, T, C, Cp, alpha_exp, inv_beta, f, s));
  if (tok) {
    const double e = (double)B * T;
    prof_stop(tok, s, knobs().act_defer ? "alcm::act_mfma_kernel<64, true, true>" : "alcm::act_mfma_kernel<64, false, true>",
                2.0 * 36.0 * e * C, e * (2.0 * C + 2.0 * Cp));
  }
  return 0;
}

int activation1d_op(const float* x, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                    const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                    hipStream_t s) {
  if (!x || !y || !alpha_exp || !inv_beta || !up_filter || !down_filter || B <= 0 || T <= 0 || C <= 0)
    return set_error(ALCM_E_INVALID, "activation1d_op: bad arguments");
  if (Cp < C || Cp % 32) return set_error(ALCM_E_INVALID, "activation1d_op: Cp must be >= C and a multiple of 32");
  if (C % 2) return set_error(ALCM_E_INVALID, "activation1d_op: C must be even");
  if (prec < PREC_BF16 || prec > PREC_F16W2) return set_error(ALCM_E_INVALID, "activation1d_op: bad prec");
  if ((((uintptr_t)x) & 7) || (((uintptr_t)y) & 3)) return set_error(ALCM_E_INVALID, "activation1d_op: alignment");
  if ((int64_t)B * T * Cp >= (1ll << 40)) return set_error(ALCM_E_INVALID, "activation1d_op: problem too large");
  Taps12O f;
  for (int k = 0; k < 12; ++k) {
    f.up[k] = 2.0f * up_filter[k];
    f.dn[k] = down_filter[k];
  }
  if (act_mfma_ok(C, Cp, prec) && !(((uintptr_t)x) & 15) && !(((uintptr_t)y) & 15)) {  // both FIRs on MFMA (alcm_act.hip): the wide stages under the mixed policy
    void* tok = prof_start(s);
    ALCM_TRY(act_mfma(x, false, y, B, T, C, Cp, alpha_exp, inv_beta, f, s));
    if (tok) {
      const double e = (double)B * T;
      prof_stop(tok, s, knobs().act_defer ? "alcm::act_mfma_kernel<64, true, false>" : "alcm::act_mfma_kernel<64, false, false>",
                2.0 * 36.0 * e * C, e * (4.0 * C + 2.0 * Cp));
    }
    return 0;
  }
  // otherwise the LDS-cooperative kernel (alcm_act.hip)
  void* tok = prof_start(s);
  void* ys[1] = {y};
  const float* ae[1] = {alpha_exp};
  const float* ib[1] = {inv_beta};
  ALCM_TRY(act_coop(x, ys, 1, B, T, C, Cp, ae, ib, f, prec, s));
  if (tok) {
    char name[64];
    std::snprintf(name, sizeof(name), "alcm::act_coop_kernel<%d>", prec == PREC_F16W2 ? PREC_F16 : prec);
    const double e = (double)B * T;
    prof_stop(tok, s, name, 2.0 * 36.0 * e * C, e * (4.0 * C + 2.0 * Cp * (prec == PREC_SPLIT ? 2 : 1)));
  }
  ALCM_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ implicit-GEMM conv on operand planes
struct OpConvDev {
  const u16* a;
  int64_t a_lo;
  int T, Cp, ksize, dil, pad;
  const u16* w;
  int64_t w_lo;
  int kpad, N;
  const float* bias;
  const float* res;
  float* out;
  int out_act, accumulate;
  float out_scale;
  int tiles_per_batch;
  int tstride, tshift;  // tile i of a batch computes rows [i * tstride - tshift, + BM)
  ActEpiDev act;        // ACT: fused Activation1d epilogue into operand planes
  int act_prefetch;     // ACT: residual prefetched into registers before the K loop
  int ostride, ooff, orows;  // output row of conv row t: b * orows + t * ostride + ooff (a ConvTranspose phase)
};

constexpr int OC_AW = 48;       // window row stride (elements): conflict-free fragment reads from any start row
constexpr int OC_HALO = 64;     // max (k-1)*dil

__device__ __forceinline__ int oc_boff(int r, int kq) { return r * 32 + ((kq ^ ((r >> 2) & 2)) << 3); }

// TPS taps per K step (one LDS barrier per TPS*32-deep step); the output tile is staged through LDS
// over the dead window/weight buffers, RG row groups (of TM*16 rows) at a time, and written as whole
// BN-column row segments with 16-byte stores (residual read the same way).  VEC = N % 4 == 0.
// PRE: prefetch the residual into registers at kernel start (narrow tiles whose tile fits one round).
// ACT3: fused-activation tiles without a residual (the dilated conv1 of an AMPBlock layer) built for 3 workgroups
// per CU (<= 168 registers); with a residual the 2-workgroup build keeps its register prefetch of the residual rows
template <int BM, int BN, int WGM, int WGN, int PREC, int TPS, bool VEC, bool ACT, bool ACT3 = false>
__global__ __launch_bounds__(256, ACT3 ? 3 : 1) void opconv_kernel(const OpConvDev P) {
  constexpr int TM = BM / (WGM * 16);
  constexpr int TN = BN / (WGN * 16);
  constexpr int NPA = PREC == PREC_SPLIT ? 2 : 1;
  constexpr int NPB = (PREC == PREC_SPLIT || PREC == PREC_F16W2) ? 2 : 1;
  constexpr int WRM = BM + OC_HALO;
  constexpr int WCH = WRM * 4;  // 16-B chunks of one window plane
  constexpr int WPER = (WCH + 255) / 256;
  constexpr int BCH = BN * 4;   // 16-B chunks of one tap's weight tile (one plane)
  constexpr int BPER = (BCH + 255) / 256;
  static_assert(WGM * WGN == 4 && TM >= 1 && TN >= 1, "4 waves");
  static_assert(TPS == 1 || TPS == 2, "1 or 2 taps per step");
  constexpr int AW_BYTES = 2 * NPA * WRM * OC_AW * 2, BS_BYTES = 2 * NPB * TPS * BN * 32 * 2;
  constexpr int OTS = BN + 4;                                   // output tile row stride (floats)
  constexpr int SMEM0 = AW_BYTES + BS_BYTES;
  constexpr int SMEM = (ACT && BM * OTS * 4 > SMEM0) ? BM * OTS * 4 : SMEM0;  // ACT stages the whole tile                                   // output tile row stride (floats)
  constexpr int GROUP_BYTES = TM * 16 * OTS * 4;                // one row group of the tile
  constexpr int RG0 = SMEM / GROUP_BYTES;
  constexpr int RG = RG0 >= WGM ? WGM : (RG0 >= 1 ? RG0 : 1);   // row groups per epilogue round
  static_assert(GROUP_BYTES <= SMEM, "output row group must fit the LDS");
  static_assert(!ACT || (VEC && RG == WGM), "the fused activation needs the whole tile in LDS");
  constexpr bool PRE = !ACT && VEC && RG == WGM && (BM * BN / 4) <= 12 * 256;
  constexpr int RPER = (BM * BN / 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  auto Aw = reinterpret_cast<__bf16(*)[NPA][WRM * OC_AW]>(smem);
  auto Bs = reinterpret_cast<__bf16(*)[NPB][TPS][BN * 32]>(smem + AW_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int b = blockIdx.x / P.tiles_per_batch;
  const int t0 = (blockIdx.x - b * P.tiles_per_batch) * P.tstride - P.tshift;
  const int col0 = blockIdx.y * BN;
  const int K = P.ksize;
  const int WR = BM + (K - 1) * P.dil;
  const int nC = P.Cp / 32;
  const int SPC = (K + TPS - 1) / TPS;  // steps per chunk
  const int nsteps = nC * SPC;
  const int mrows = min(BM, P.T - t0);  // (ACT tiles can start before t = 0; only the ACT epilogue sees them)
  const int64_t rowbase = (int64_t)b * P.T + t0;  // global output row of tile row 0

  // residual prefetch (narrow tiles): tile rows are one contiguous block of mrows * N floats
  float4 rp[RPER];  // dead (and eliminated) unless PRE
  // ACT tiles: the residual of every tile row (halo rows included) is loaded into registers before the K loop,
  // so the epilogue does not stall on one dependent global load per float4
  // (not in the ACT3 build: the 48 registers would spill)
  constexpr bool PREA_OK = ACT && !ACT3;
  constexpr int RPA = PREA_OK ? (BM * (BN / 4) + 255) / 256 : 1;
  float4 rpa[RPA];
  const bool prea = PREA_OK && P.res && P.act_prefetch;
  if (prea) {
    const int cq = P.N / 4;
#pragma unroll
    for (int i = 0; i < RPA; ++i) {
      const int e = tid + i * 256;
      const int m = e / cq, n = (e - m * cq) * 4;
      const int t = min(max(t0 + m, 0), P.T - 1);
      const int64_t go = ((int64_t)b * P.T + t) * P.N + (e < BM * cq ? n : 0);
      rpa[i] = *reinterpret_cast<const float4*>(P.res + go);
    }
  }
  if constexpr (PRE) {
    const int nq = mrows * (P.N / 4);
#pragma unroll
    for (int i = 0; i < RPER; ++i) {
      const int e = tid + i * 256;
      const int ec = e < nq ? e : 0;
      rp[i] = P.res ? *reinterpret_cast<const float4*>(P.res + rowbase * P.N + (int64_t)ec * 4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // Loads are issued unconditionally from clamped (always valid) addresses and out-of-range data is
  // zeroed when it is written to LDS: divergent `if (ok) load` blocks make hipcc drain vmcnt(0) at
  // every block boundary, which serialises the prefetch pipeline.
  const u16* wsrc[WPER];
  bool wok[WPER];
#pragma unroll
  for (int i = 0; i < WPER; ++i) {
    const int c = tid + i * 256;
    const int w = c >> 2;
    const int ts = t0 + w - P.pad;
    wok[i] = c < WCH && w < WR && ts >= 0 && ts < P.T;
    const int tc = ts < 0 ? 0 : (ts >= P.T ? P.T - 1 : ts);
    wsrc[i] = P.a + ((int64_t)b * P.T + tc) * P.Cp + (c & 3) * 8;
  }
  uint4 wv[WPER][NPA];
  auto load_window = [&](int cc) {
#pragma unroll
    for (int i = 0; i < WPER; ++i)
#pragma unroll
      for (int p = 0; p < NPA; ++p) wv[i][p] = *reinterpret_cast<const uint4*>(wsrc[i] + cc * 32 + p * P.a_lo);
  };
  auto store_window = [&](int buf) {
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int c = tid + i * 256;
      if (WCH % 256 != 0 && c >= WCH) continue;
      const uint32_t m = wok[i] ? 0xffffffffu : 0u;  // zero padding rows, branch-free
#pragma unroll
      for (int p = 0; p < NPA; ++p)
        *reinterpret_cast<uint4*>(&Aw[buf][p][(c >> 2) * OC_AW + (c & 3) * 8]) =
            make_uint4(wv[i][p].x & m, wv[i][p].y & m, wv[i][p].z & m, wv[i][p].w & m);
    }
  };

  // weight rows of this thread
  const u16* bsrc[BPER];
  bool bok[BPER];
#pragma unroll
  for (int i = 0; i < BPER; ++i) {
    const int c = tid + i * 256;
    const int n = col0 + (c >> 2);
    bok[i] = c < BCH && n < P.N;
    bsrc[i] = P.w + (int64_t)(bok[i] ? n : 0) * P.kpad + (c & 3) * 8;
  }
  uint4 breg[2][TPS][BPER][NPB];
  // step order: (chunk cc, tap group g) -> taps g*TPS + t (clamped to K-1: a missing tap of the last
  // group is loaded but its MFMAs are skipped); the loader walks the order incrementally
  int ld_g = 0, ld_cc = 0;
  auto load_b = [&](auto set_c) {
    constexpr int set = decltype(set_c)::value;
#pragma unroll
    for (int t = 0; t < TPS; ++t) {
      const int tap = min(ld_g * TPS + t, K - 1);
      const int k0 = tap * P.Cp + ld_cc * 32;
#pragma unroll
      for (int i = 0; i < BPER; ++i)
#pragma unroll
        for (int p = 0; p < NPB; ++p)
          breg[set][t][i][p] = *reinterpret_cast<const uint4*>(bsrc[i] + k0 + p * P.w_lo);
    }
    if (ld_cc * SPC + ld_g + 1 < nsteps) {
      if (++ld_g == SPC) {
        ld_g = 0;
        ++ld_cc;
      }
    }
  };
  auto store_b = [&](auto set_c, int buf) {
    constexpr int set = decltype(set_c)::value;
#pragma unroll
    for (int t = 0; t < TPS; ++t)
#pragma unroll
      for (int i = 0; i < BPER; ++i) {
        const int c = tid + i * 256;
        if (BCH % 256 != 0 && c >= BCH) continue;
        const int off = oc_boff(c >> 2, c & 3);
        const uint32_t m = bok[i] ? 0xffffffffu : 0u;
#pragma unroll
        for (int p = 0; p < NPB; ++p) {
          const uint4 v = breg[set][t][i][p];
          *reinterpret_cast<uint4*>(&Bs[buf][p][t][off]) = make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
        }
      }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: window 0 and weight step 0 in LDS, weight step 1 in registers
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  load_window(0);
  load_b(S0{});
  store_window(0);
  store_b(S0{}, 0);
  load_b(S1{});
  __syncthreads();

  const int a_base = (wm * TM * 16 + (lane & 15)) * OC_AW + (lane >> 4) * 8;
  const int b_off = oc_boff(wn * TN * 16 + (lane & 15), lane >> 4);
  auto mma_tap = [&](int wb, int tap, const __bf16* bh_base, const __bf16* bl_base) {
    const int a_off = a_base + tap * P.dil * OC_AW;
    bf16x8 ah[TM], al[NPA == 2 ? TM : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(&Aw[wb][0][a_off + i * 16 * OC_AW]);
      if (NPA == 2) al[i] = *reinterpret_cast<const bf16x8*>(&Aw[wb][NPA - 1][a_off + i * 16 * OC_AW]);
    }
    bf16x8 bh[TN], bl[NPB == 2 ? TN : 1];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(bh_base + b_off + j * 16 * 32);
      if (NPB == 2) bl[j] = *reinterpret_cast<const bf16x8*>(bl_base + b_off + j * 16 * 32);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (PREC == PREC_SPLIT) {
          acc[i][j] = mfma16<PREC_BF16>(al[i], bh[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_BF16>(ah[i], bl[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_BF16>(ah[i], bh[j], acc[i][j]);
        } else if constexpr (PREC == PREC_F16W2) {
          acc[i][j] = mfma16<PREC_F16>(ah[i], bl[j], acc[i][j]);
          acc[i][j] = mfma16<PREC_F16>(ah[i], bh[j], acc[i][j]);
        } else {
          acc[i][j] = mfma16<PREC>(ah[i], bh[j], acc[i][j]);
        }
      }
  };
  // one K step = tap group g of chunk cc; SET (= step parity) is compile-time so the register ring
  // never lands in scratch
  auto step = [&](int cc, int g, bool last_in_chunk, auto set_c) {
    constexpr int SET = decltype(set_c)::value;
    load_b(set_c);  // step s+2 (clamped) into register set SET, which held step s (already in LDS)
    const int wb = cc & 1;
    mma_tap(wb, g * TPS, &Bs[SET][0][0][0], &Bs[SET][NPB - 1][0][0]);
    if (TPS == 2 && g * TPS + 1 < K) mma_tap(wb, g * TPS + 1, &Bs[SET][0][1][0], &Bs[SET][NPB - 1][1][0]);
    store_b(std::integral_constant<int, SET ^ 1>{}, SET ^ 1);  // step s+1 (loaded during step s-1)
    if (last_in_chunk) store_window(wb ^ 1);
    __syncthreads();
  };
  for (int cc = 0; cc < nC; ++cc) {
    load_window(cc + 1 < nC ? cc + 1 : cc);  // next chunk's window (the last chunk reloads itself, unused)
    const int s0 = cc * SPC;
    const bool more = cc + 1 < nC;
    int g = 0;
    if (s0 & 1) {
      step(cc, 0, more && SPC == 1, S1{});
      g = 1;
    }
    for (; g + 1 < SPC; g += 2) {
      step(cc, g, false, S0{});
      step(cc, g + 1, more && g + 2 == SPC, S1{});
    }
    if (g < SPC) step(cc, g, more, S0{});
  }

  // epilogue
  if constexpr (ACT) {
    // v = conv + bias (+ res) for every tile row inside [0, T) -> LDS; fp32 out (if any) for the rows this
    // tile owns; then Activation1d(v) of the owned rows -> operand planes (halo rows come from the tile)
    float* ot = reinterpret_cast<float*>(smem);  // the K loop's last barrier retired every LDS read
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = wn * TN * 16 + j * 16 + (lane & 15);
          ot[m * OTS + n] = acc[i][j][r] + ((P.bias && n < P.N) ? P.bias[n] : 0.f);
        }
      }
    __syncthreads();
    const int e_lo = t0 + P.tshift, e_hi = min(e_lo + P.tstride, P.T);
    if (prea) {
      const int cq = P.N / 4;
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
      __syncthreads();
    } else if (P.res || P.out) {
      const int cq = P.N / 4;
      for (int e = tid; e < BM * cq; e += 256) {
        const int m = e / cq, n = (e - m * cq) * 4;
        const int t = t0 + m;
        if (t < 0 || t >= P.T) continue;
        const int64_t go = ((int64_t)b * P.T + t) * P.N + n;
        float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
        if (P.res) {
          const float4 rv = *reinterpret_cast<const float4*>(P.res + go);
          v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
          *reinterpret_cast<float4*>(ot + m * OTS + n) = v;
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
      __syncthreads();
    }
    // emitted rows BM - 16: 240 -> R = 15 (16 runs), 112 -> R = 14 (8 runs)
    act_epilogue_tile<PREC, (BM == 256 ? 15 : (BM == 128 ? 14 : 8))>(ot, OTS, t0, e_lo, e_hi, P.T, P.act.Cp, 0, P.N, b,
                                                                    P.act, tid, 256);
    return;
  }
  if constexpr (VEC) {
    float* ot = reinterpret_cast<float*>(smem);  // the K loop's last barrier retired every LDS read
    for (int h0 = 0; h0 < WGM; h0 += RG) {
      if (wm >= h0 && wm < h0 + RG) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = (wm - h0) * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int n = wn * TN * 16 + j * 16 + (lane & 15);
              float v = acc[i][j][r];
              if (P.bias && col0 + n < P.N) v += P.bias[col0 + n];
              if (P.out_act) v = alcm_act(v, P.out_act);
              ot[m * OTS + n] = v;
            }
          }
      }
      __syncthreads();
      const int r0 = h0 * TM * 16;  // first tile row of this round
      const int rows = min(RG * TM * 16, mrows - r0);
      const int cq = min(BN, P.N - col0) / 4;  // float4 columns of this tile (N % 4 == 0)
      const int nq = rows * cq;
      for (int e = tid; e < (rows > 0 ? nq : 0); e += 256) {
        const int m = e / cq, n = (e - m * cq) * 4;
        const int64_t go = ((int64_t)b * P.orows + (int64_t)(t0 + r0 + m) * P.ostride + P.ooff) * P.N + col0 + n;
        float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (PRE && P.N <= BN) {
          // the tile spans all N columns: its rows are one contiguous block and e is the same element
          // index the residual prefetch used
          const int i = (e - tid) / 256;
#pragma unroll
          for (int ii = 0; ii < RPER; ++ii)
            if (ii == i) rv = rp[ii];
        } else if (P.res) {
          rv = *reinterpret_cast<const float4*>(P.res + go);
        }
        v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
        v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
        if (P.accumulate) {
          const float4 pv = *reinterpret_cast<const float4*>(P.out + go);
          v.x += pv.x; v.y += pv.y; v.z += pv.z; v.w += pv.w;
        }
        *reinterpret_cast<float4*>(P.out + go) = v;
      }
      __syncthreads();
    }
    return;
  }
  // direct stores (N % 4 != 0, e.g. conv_post): rows (b, t0 + m), channels-last output, row stride N
#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
    for (int r = 0; r < 4; ++r) {
      const int t = t0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
      if (t >= P.T) continue;
      const int64_t ro = ((int64_t)b * P.T + t) * P.N;
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j) {
        const int n = col0 + wn * TN * 16 + j * 16 + (lane & 15);
        if (n >= P.N) continue;
        float v = acc[i][j][r];
        if (P.bias) v += P.bias[n];
        if (P.out_act) v = alcm_act(v, P.out_act);
        if (P.res) v += P.res[ro + n];
        v *= P.out_scale;
        if (P.accumulate) v += P.out[ro + n];
        P.out[ro + n] = v;
      }
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int TPS, bool VEC, bool ACT>
static void launch_opconv_v(const OpConvDev& Q, dim3 grid, int prec, hipStream_t s) {
  constexpr int TPS_SPLIT = BN >= 192 ? 1 : TPS;  // LDS: the split operands double both buffers
  constexpr bool SPLIT_FITS = 2 * 2 * (BM + OC_HALO) * OC_AW * 2 + 2 * 2 * TPS_SPLIT * BN * 32 * 2 <= 160 * 1024;
  if constexpr (ACT && BM == 128) {
    // conv1 (no residual) of C = 96 at fp16: the 3-workgroup build (-11..-13 % per launch, scripts/microbench.py
    // tail; the same 128-row build for C = 48 measured +10 % at k11 against its 256-row tiles and is not used)
    if (!Q.res && prec == PREC_F16) {
      hipLaunchKernelGGL((opconv_kernel<BM, BN, WGM, WGN, PREC_F16, TPS, VEC, ACT, true>), grid, dim3(256), 0, s, Q);
      return;
    }
  }
  if (prec == PREC_SPLIT) {
    if constexpr (SPLIT_FITS)
      hipLaunchKernelGGL((opconv_kernel<BM, BN, WGM, WGN, PREC_SPLIT, TPS_SPLIT, VEC, ACT>), grid, dim3(256), 0, s, Q);
  } else if (prec == PREC_F16)
    hipLaunchKernelGGL((opconv_kernel<BM, BN, WGM, WGN, PREC_F16, TPS, VEC, ACT>), grid, dim3(256), 0, s, Q);
  else if (prec == PREC_F16W2)
    hipLaunchKernelGGL((opconv_kernel<BM, BN, WGM, WGN, PREC_F16W2, TPS, VEC, ACT>), grid, dim3(256), 0, s, Q);
  else hipLaunchKernelGGL((opconv_kernel<BM, BN, WGM, WGN, PREC_BF16, TPS, VEC, ACT>), grid, dim3(256), 0, s, Q);
}

template <int BM, int BN, int WGM, int WGN, int TPS>
static int launch_opconv(const OpConvDev& P, int B, int prec, bool act, double flops, double bytes, hipStream_t s) {
  OpConvDev Q = P;
  // ACT tiles overlap by 2 * ACT_EPI_HALO rows: each computes BM conv rows and emits BM - 2*HALO
  Q.tstride = act ? BM - 2 * ACT_EPI_HALO : BM;
  Q.tshift = act ? ACT_EPI_HALO : 0;
  Q.tiles_per_batch = (P.T + Q.tstride - 1) / Q.tstride;
  dim3 grid(B * Q.tiles_per_batch, (P.N + BN - 1) / BN);
  // LDS-staged epilogue for narrow layers (one tile spans N); wide layers store straight from the
  // accumulators (measured faster there: the LDS round trip costs more than the coalescing saves)
  const bool vec = P.N % 4 == 0 && P.N <= BN;
  if (act && !vec) return set_error(ALCM_E_INVALID, "opconv: fused activation needs N % 4 == 0 and one column tile");
  void* tok = prof_start(s);
  if (act) {
    if constexpr (BN <= 96) launch_opconv_v<BM, BN, WGM, WGN, TPS, true, true>(Q, grid, prec, s);
  } else if (vec) launch_opconv_v<BM, BN, WGM, WGN, TPS, true, false>(Q, grid, prec, s);
  else launch_opconv_v<BM, BN, WGM, WGN, TPS, false, false>(Q, grid, prec, s);
  if (tok) {
    char name[128];
    // the demangled rocprofv3 name of the instantiation (bench.py joins the two by name)
    const int tps = (prec == PREC_SPLIT && BN >= 192) ? 1 : TPS;
    const bool act3 = act && BM == 128 && prec == PREC_F16 && !P.res;
    std::snprintf(name, sizeof(name), "alcm::opconv_kernel<%d, %d, %d, %d, %d, %d, %s, %s, %s>", BM, BN, WGM, WGN, prec,
                  tps, (vec || act) ? "true" : "false", act ? "true" : "false", act3 ? "true" : "false");
    prof_stop(tok, s, name, flops, bytes);
  }
  return 0;
}

// narrow-layer tile variant (diagnostics / A-B): ALCM_OPCONV_TILE=0 default, 1 = twice the rows per tile,
// 2 = twice the rows and two taps per K step
static int tile_variant(int prec) {
  return prec != PREC_SPLIT ? knobs().opconv_tile : 0;  // the split operands need the default tiles' LDS
}

bool opconv_act_supported(int prec, int N, int Cp_in) {
  if (N % 4 || N <= 0) return false;
  // opconv_kernel ACT tiles (BN <= 96): HBM-bound layers, the fusion saves ~15%.  Wide layers keep conv + standalone
  // Activation1d: a fused epilogue in the two-workgroup wide conv measured -6 % end to end
  return N <= 96;
}

int opconv(const alcm_opconv_args& a, hipStream_t s) {
  const bool act = a.act_plane != nullptr;
  if (!a.a || !a.w || (!a.out && !act && !a.geglu_plane && !a.out_plane) || a.B <= 0 || a.T <= 0 || a.N <= 0 || a.ksize <= 0 || a.dil <= 0)
    return set_error(ALCM_E_INVALID, "opconv: bad arguments");
  if (a.Cp <= 0 || a.Cp % 32) return set_error(ALCM_E_INVALID, "opconv: Cp must be a positive multiple of 32");
  if ((a.ksize - 1) * a.dil > OC_HALO) return set_error(ALCM_E_INVALID, "opconv: receptive field too large");
  const bool strided = a.out_stride > 0;
  if (strided) {
    if (a.pad < 0 || a.pad > (a.ksize - 1) * a.dil || a.out_offset < 0 || a.out_offset >= a.out_stride ||
        (int64_t)(a.T - 1) * a.out_stride + a.out_offset >= a.out_rows || !a.out || a.res || a.accumulate ||
        a.out_act || a.act_plane || a.geglu_plane)
      return set_error(ALCM_E_INVALID, "opconv: bad strided-output arguments");
  } else if (2 * a.pad != (a.ksize - 1) * a.dil) {
    return set_error(ALCM_E_INVALID, "opconv: only same-length convs");
  }
  if (a.kpad < a.ksize * a.Cp || a.kpad % 32) return set_error(ALCM_E_INVALID, "opconv: kpad mismatch");
  if (a.prec < PREC_BF16 || a.prec > PREC_F16W2) return set_error(ALCM_E_INVALID, "opconv: bad prec");
  if ((((uintptr_t)a.a) & 15) || (((uintptr_t)a.w) & 15) || (a.a_lo_off % 8) || (a.w_lo_off % 8))
    return set_error(ALCM_E_INVALID, "opconv: operands must be 16-byte aligned");
  if (a.C <= 0 || a.C > a.Cp) return set_error(ALCM_E_INVALID, "opconv: C must be in (0, Cp]");
  if (act) {
    if (a.out_act || a.N % 2 || !a.act_alpha_exp || !a.act_inv_beta || !a.act_up_filter || !a.act_down_filter)
      return set_error(ALCM_E_INVALID, "opconv: fused activation needs out_act == 0, even N and its parameters");
    if (a.out && a.res && a.out == a.res) return set_error(ALCM_E_INVALID, "opconv: fused activation: out aliases res");
    if ((((uintptr_t)a.act_plane) & 3) || (a.act_plane_lo_off % 2))
      return set_error(ALCM_E_INVALID, "opconv: act_plane alignment");
    if ((a.res && (((uintptr_t)a.res) & 15)) || (a.out && (((uintptr_t)a.out) & 15)) || a.N % 4)
      return set_error(ALCM_E_INVALID, "opconv: fused activation needs 16-byte aligned res/out and N % 4 == 0");
  }
  OpConvDev P{};
  P.a = (const u16*)a.a; P.a_lo = a.a_lo_off;
  if (act) {
    P.act.plane = (u16*)a.act_plane;
    P.act.plane_lo = a.act_plane_lo_off;
    P.act.Cp = round_up(a.N, 32);
    P.act.aexp = a.act_alpha_exp;
    P.act.ibeta = a.act_inv_beta;
    for (int k = 0; k < 12; ++k) {
      P.act.f.up[k] = 2.0f * a.act_up_filter[k];
      P.act.f.dn[k] = a.act_down_filter[k];
    }
  }
  P.T = a.T; P.Cp = a.Cp; P.ksize = a.ksize; P.dil = a.dil; P.pad = a.pad;
  // planes of the packed weight: bf16 hi | bf16 lo | fp16 hi | fp16 lo, w_lo_off apart
  const bool f16 = a.prec == PREC_F16 || a.prec == PREC_F16W2;
  P.w = (const u16*)a.w + (f16 ? 2 * a.w_lo_off : 0);
  P.w_lo = a.w_lo_off; P.kpad = a.kpad; P.N = a.N;
  P.bias = a.bias; P.res = a.res; P.out = a.out; P.out_act = a.out_act; P.accumulate = a.accumulate;
  P.out_scale = a.out_scale;
  P.act_prefetch = 1;
  P.ostride = strided ? a.out_stride : 1;
  P.ooff = strided ? a.out_offset : 0;
  P.orows = strided ? a.out_rows : a.T;
  const double M = (double)a.B * a.T;
  const int npa = a.prec == PREC_SPLIT ? 2 : 1, npb = (a.prec == PREC_SPLIT || a.prec == PREC_F16W2) ? 2 : 1;
  const double flops = 2.0 * M * a.N * (double)a.ksize * a.C;
  const double bytes = M * a.Cp * 2.0 * npa + (double)a.N * a.kpad * 2.0 * npb +
                       M * a.N * 4.0 * ((a.out ? 1 : 0) + (a.res ? 1 : 0) + (a.accumulate ? 1 : 0)) +
                       (act ? M * round_up(a.N, 32) * 2.0 * npa : 0.0);
  if (a.out_plane) {  // only the wide-layer kernel has the plane-output epilogue
    if (a.res || a.accumulate || a.out_act || act || a.geglu_plane || strided || a.out ||
        (a.prec != PREC_F16 && a.prec != PREC_BF16) || (((uintptr_t)a.out_plane) & 7) || !wconv_try(a, P.w, flops, bytes, s))
      return set_error(ALCM_E_INVALID, "opconv: plane output needs F16/BF16, N % 4 == 0, Cp % 64 == 0, out == NULL "
                                       "and no res/accumulate/act/GEGLU/strided output");
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  if (a.geglu_plane) {  // only the wide-layer kernel has the GEGLU epilogue
    if (!wconv_try(a, P.w, flops, bytes, s))
      return set_error(ALCM_E_INVALID, "opconv: GEGLU plane epilogue needs F16/BF16, N % 128 == 0, Cp % 64 == 0, "
                                       "no res/accumulate/act, 4-byte aligned plane");
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  if (strided) {  // the two-workgroup wide-layer kernel, or opconv_kernel's LDS-staged epilogue (N <= 96)
    if (wconv_try(a, P.w, flops, bytes, s)) {
      ALCM_HIP(hipGetLastError());
      return 0;
    }
    if (a.N % 4 || a.N > 96)
      return set_error(ALCM_E_INVALID, "opconv: strided output needs the wide-layer kernel (F16/BF16, N % 192 == 0, "
                                       "Cp % 64 == 0, (k-1)*dil <= 64) or N <= 96 with N % 4 == 0");
  } else if ((!act && wconv_try(a, P.w, flops, bytes, s)) ||
      nconv_try(a, P.w, act ? &P.act : nullptr, flops, bytes, s)) {
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  const int N = a.N;
  // one tap per K step (two taps per step measured slower: the larger weight buffers cost occupancy)
  //                                                      BM   BN  WGM WGN TPS
  // small problems whose 128 x 128 tiles would leave CUs idle (the text encoders' N = 1024 projections at
  // M = 2464: 160 tiles for 256 CUs) take the 96-column tiles (220 tiles): text encode 13.5 -> 13.2 ms per B = 32
  // (profiles/r3v); ALCM_OPCONV_TILE=-1 keeps the 128 x 128 tiles (A/B)
  const int64_t tiles128 = (int64_t)a.B * ((a.T + 127) / 128) * ((N + 127) / 128);
  const bool underfill = !act && N % 128 == 0 && N > 96 && tiles128 < 256 && knobs().opconv_tile != -1;
  int rc;
  if (act && N > 96) rc = set_error(ALCM_E_INVALID, "opconv: fused activation on N > 96 needs the wide kernel");
  else if (N % 192 == 0 && N % 128 != 0) rc = launch_opconv<128, 192, 2, 2, 1>(P, a.B, a.prec, act, flops, bytes, s);
  else if (N % 128 == 0 && !underfill) rc = launch_opconv<128, 128, 2, 2, 1>(P, a.B, a.prec, act, flops, bytes, s);
  else if (N > 48) {
    const int v = tile_variant(a.prec);
    if (v == 1) rc = launch_opconv<256, 96, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
    else if (v == 2) rc = launch_opconv<256, 96, 4, 1, 2>(P, a.B, a.prec, act, flops, bytes, s);
    else rc = launch_opconv<128, 96, 2, 2, 1>(P, a.B, a.prec, act, flops, bytes, s);
  } else if (N > 32) {
    const int v = tile_variant(a.prec);
    if (v == 1) rc = launch_opconv<512, 48, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
    else if (v == 2) rc = launch_opconv<512, 48, 4, 1, 2>(P, a.B, a.prec, act, flops, bytes, s);
    else rc = launch_opconv<256, 48, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
  } else if (N > 16) {
    const int v = tile_variant(a.prec);
    if (v == 1) rc = launch_opconv<512, 32, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
    else if (v == 2) rc = launch_opconv<512, 32, 4, 1, 2>(P, a.B, a.prec, act, flops, bytes, s);
    else rc = launch_opconv<256, 32, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
  }
  else rc = launch_opconv<256, 16, 4, 1, 1>(P, a.B, a.prec, act, flops, bytes, s);
  if (rc) return rc;
  ALCM_HIP(hipGetLastError());
  return 0;
}

// out = (sum over i < n of conv_i + bias_i + res_i) * args[0].out_scale (+ out if args[0].accumulate): the fused
// sum-form launch where it applies (three wide terms), else the terms in order, each accumulating into out
int opconv_sum(const alcm_opconv_args* a, int n, hipStream_t s) {
  if (!a || n < 1 || n > 3) return set_error(ALCM_E_INVALID, "opconv_sum: 1 <= n <= 3 terms");
  if (!a[0].out && !a[0].out_plane) return set_error(ALCM_E_INVALID, "opconv_sum: args[0].out is required");
  if (a[0].out_plane && !wconv3_sum_ok(a, n))
    return set_error(ALCM_E_INVALID, "opconv_sum: a plane output needs the one-launch form (three F16 / BF16 terms, "
                                     "dilation 1, Cp % 64 == 0, N % 192 == 0, full 256-row tiles) and no accumulate");
  for (int i = 0; i < n; ++i)
    if (a[i].B != a[0].B || a[i].T != a[0].T || a[i].N != a[0].N || a[i].act_plane || (i > 0 && a[i].out_plane) ||
        a[i].geglu_plane || a[i].out_stride > 0 || a[i].out_act || (a[i].out && a[i].out != a[0].out))
      return set_error(ALCM_E_INVALID, "opconv_sum: terms need equal B, T, N, same-length fp32 outputs into "
                                       "args[0].out, no activation / plane / GEGLU / strided output");
  if (wconv3_sum_try(a, n, s)) {
    ALCM_HIP(hipGetLastError());
    return 0;
  }
  for (int i = 0; i < n; ++i) {
    alcm_opconv_args g = a[i];
    g.out = a[0].out;
    g.out_scale = a[0].out_scale;
    g.accumulate = i > 0 ? 1 : a[0].accumulate;
    ALCM_TRY(opconv(g, s));
  }
  return 0;
}

}  // namespace alcm

extern "C" int alcm_opconv_sum(const alcm_opconv_args* args, int n, alcm_stream_t stream) {
  return alcm::opconv_sum(args, n, (hipStream_t)stream);
}

extern "C" int alcm_activation1d_op(const float* x, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                                    const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                                    alcm_stream_t stream) {
  return alcm::activation1d_op(x, y, B, T, C, Cp, alpha_exp, inv_beta, up_filter, down_filter, prec,
                               (hipStream_t)stream);
}

extern "C" int alcm_activation1d_op_f16in(const void* x16, void* y, int B, int T, int C, int Cp,
                                          const float* alpha_exp, const float* inv_beta, const float* up_filter,
                                          const float* down_filter, int prec, alcm_stream_t stream) {
  return alcm::activation1d_op_h16(x16, y, B, T, C, Cp, alpha_exp, inv_beta, up_filter, down_filter, prec,
                                   (hipStream_t)stream);
}

extern "C" int alcm_opconv(const alcm_opconv_args* args, alcm_stream_t stream) {
  if (!args) return alcm::set_error(ALCM_E_INVALID, "null args");
  return alcm::opconv(*args, (hipStream_t)stream);
}
