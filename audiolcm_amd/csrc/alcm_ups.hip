// BigVGAN ConvTranspose1d upsampler of the narrow stages (stride 2, kernel 4: vocoder/bigvgan/models.py:160-165,
// 187-188) under the split precision, both output phases in ONE pass over the fp32 input.
//
// The phase decomposition (alcm_models.cpp, load_vocoder): output row 2 v + off[r] = sum over taps j in {0, 1} of
// W_r[j] x[v - pad[r] + j] + bias, i.e. two 2-tap convs of the same input rows.  The generic path ran them as two
// fp32-operand GEMM launches (alcm_gemm.hip), each re-reading x and converting it to bf16 hi / lo per 32-deep K step
// per N tile: 0.31 + 0.54 ms per phase pair at stages 4 / 5 against 0.09 of HBM time.
//
// Structure: persistent 512-thread workgroups (one per CU at stage 4, two at stage 5), both phases' packed bf16 hi / lo weight planes resident in
// LDS (rows of an odd number of 16-B slots); per tile of TM = 128 input rows the window [t0 - 1, t0 + 129) is split
// into bf16 hi / lo operand rows in LDS (rows outside [0, T) zero = the conv padding),
// while the next tile's window is already loading into registers; wave w computes input rows 16 w .. 16 w + 15 of
// both phases (bf16x3: lo*hi + hi*lo + hi*hi per 32-deep K slice, K = tap * cp + c as the packed weights, cp = cin: a
// lane's 8 channels never straddle a tap) and stores
// its fp32 outputs straight from the accumulators.
#include <cstdio>
#include <cstring>

#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

typedef __attribute__((address_space(3))) void up_lds_t;
typedef __attribute__((address_space(1))) void up_gbl_t;

__device__ __attribute__((aligned(16))) uint4 g_ups_zero[8];

struct Ups2Dev {
  const float* x;  // [B][T][cin] fp32
  float* out;      // [B][2 T][cout] fp32
  int T, cin, cout;
  const u16* w[2];  // phase r: bf16 hi plane [cout][kpad] (K = tap * cp + c), lo plane lo elements after it
  int64_t lo;
  int kpad;
  int pad[2], off[2];
  const float* bias;
  int tiles_per_batch, ntiles;
};

template <int CP, int NOUT>
struct UpsGeo {
  static constexpr int TM = 128, TR = TM + 2, NT = 512, NWAVE = 8;
  static constexpr int XSL = (CP / 8) % 2 ? CP / 8 : CP / 8 + 1;  // x row: odd number of 16-B slots
  static constexpr int XRS = XSL * 16;
  static constexpr int XPL = (TR * XRS + 1023) / 1024 * 1024;   // one x plane
  static constexpr int KD = 2 * CP;                              // K per phase
  static constexpr int WSL = (KD / 8) % 2 ? KD / 8 : KD / 8 + 1;
  static constexpr int WRS = WSL * 16;
  static constexpr int WPL = NOUT * WRS;                         // one weight plane
  static constexpr int WB = (4 * WPL + 1023) / 1024 * 1024;      // [phase][plane][row]
  static constexpr int SMEM = WB + 2 * XPL;
  static constexpr int OCC = SMEM <= 81920 ? 2 : 1;             // workgroups per CU (stage 5: two)
  static_assert(KD % 32 == 0 && CP % 8 == 0 && NOUT % 16 == 0 && SMEM <= 163840, "geometry");
};

template <int CP, int NOUT, int CIN>
__global__ __launch_bounds__(512, (UpsGeo<CP, NOUT>::OCC)) void ups2_kernel(const Ups2Dev P) {
  using G = UpsGeo<CP, NOUT>;
  constexpr int TM = G::TM, TR = G::TR, NT = G::NT, XRS = G::XRS, WRS = G::WRS, KD = G::KD;
  constexpr int NTN = NOUT / 16, NS = KD / 32;
  constexpr int CQ = CIN / 4;                          // float4 per input row
  constexpr int XPT = (TR * CQ + NT - 1) / NT;         // window float4 per thread
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  char* const wl = smem;
  char* const xh = smem + G::WB;
  char* const xl = xh + G::XPL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, l16 = lane & 15;
  const int T = P.T;

  // resident weights: instruction i covers bytes [1024 i, + 1024) of [phase][plane][row n][slot q]
  {
    constexpr int NI = G::WB / 1024;
    for (int i = wave; i < NI; i += G::NWAVE) {
      const int o = i * 1024 + lane * 16;
      const int pp = o / G::WPL, rr = o - pp * G::WPL;  // pp = 2 phase + plane
      const int n = rr / WRS, q = (rr - n * WRS) >> 4;
      const bool ok = pp < 4 && n < P.cout && q < KD / 8;
      const u16* src = ok ? P.w[pp >> 1] + (pp & 1) * P.lo + (int64_t)n * P.kpad + q * 8
                          : reinterpret_cast<const u16*>(g_ups_zero);
      __builtin_amdgcn_global_load_lds((up_gbl_t*)src, (up_lds_t*)(wl + i * 1024), 16, 0, 0);
    }
  }
  // channels cin .. CP - 1 of every window row stay zero (the packed K runs over cp channels per tap)
  if constexpr (CP > CIN) {
    constexpr int ZQ = (CP - CIN) / 4;
    for (int e = tid; e < TR * ZQ; e += NT) {
      const int r = e / ZQ, c = CIN + (e - r * ZQ) * 4;
      *reinterpret_cast<uint2*>(xh + r * XRS + c * 2) = make_uint2(0u, 0u);
      *reinterpret_cast<uint2*>(xl + r * XRS + c * 2) = make_uint2(0u, 0u);
    }
  }

  float4 xr[XPT];
  auto load_x = [&](int tile) {
    const int b = tile / P.tiles_per_batch, t0 = (tile - b * P.tiles_per_batch) * TM;
    const float* xb = P.x + (int64_t)b * T * CIN;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e = tid + i * NT;
      const int r = e / CQ, c4 = e - r * CQ;
      const int t = t0 - 1 + r;
      xr[i] = (e < TR * CQ && t >= 0 && t < T) ? *reinterpret_cast<const float4*>(xb + (int64_t)t * CIN + c4 * 4)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e = tid + i * NT;
      if (e >= TR * CQ) break;
      const int r = e / CQ, c = (e - r * CQ) * 4;
      const float f[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
      uint32_t hh[2], ll[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const __bf16 h0 = (__bf16)f[2 * j], h1 = (__bf16)f[2 * j + 1];
        const __bf16 l0 = (__bf16)(f[2 * j] - (float)h0), l1 = (__bf16)(f[2 * j + 1] - (float)h1);
        hh[j] = (uint32_t)__builtin_bit_cast(u16, h0) | ((uint32_t)__builtin_bit_cast(u16, h1) << 16);
        ll[j] = (uint32_t)__builtin_bit_cast(u16, l0) | ((uint32_t)__builtin_bit_cast(u16, l1) << 16);
      }
      *reinterpret_cast<uint2*>(xh + r * XRS + c * 2) = make_uint2(hh[0], hh[1]);
      *reinterpret_cast<uint2*>(xl + r * XRS + c * 2) = make_uint2(ll[0], ll[1]);
    }
  };

  float bias_r[NTN];
#pragma unroll
  for (int j = 0; j < NTN; ++j) bias_r[j] = (j * 16 + l16 < P.cout) ? P.bias[j * 16 + l16] : 0.f;

  int tile = blockIdx.x;
  if (tile < P.ntiles) load_x(tile);
  __builtin_amdgcn_s_waitcnt(7 << 4);  // vmcnt(0): the weight DMA (and the first window)
  for (; tile < P.ntiles; tile += gridDim.x) {
    store_x();
    __syncthreads();
    const int b = tile / P.tiles_per_batch, t0 = (tile - b * P.tiles_per_batch) * TM;
    if (tile + (int)gridDim.x < P.ntiles) load_x(tile + gridDim.x);  // lands under this tile's MFMAs and stores

    f32x4 acc[2][NTN];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph)
#pragma unroll
      for (int j = 0; j < NTN; ++j) acc[ph][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      // window row of input row v = t0 + 16 wave + l16 for tap j: v - pad + j - (t0 - 1)
      const int arow = wave * 16 + l16 + 1 - P.pad[ph];
      const char* wb = wl + ph * 2 * G::WPL + l16 * WRS;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int kk = s * 32 + q4 * 8;
        const int tap = kk / CP, c = kk - tap * CP;
        const int ao = (arow + tap) * XRS + c * 2;
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(xh + ao);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(xl + ao);
        bf16x8 bh[NTN], bl[NTN];
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          bh[j] = *reinterpret_cast<const bf16x8*>(wb + j * 16 * WRS + kk * 2);
          bl[j] = *reinterpret_cast<const bf16x8*>(wb + G::WPL + j * 16 * WRS + kk * 2);
        }
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          acc[ph][j] = mfma16<PREC_BF16>(al, bh[j], acc[ph][j]);
          acc[ph][j] = mfma16<PREC_BF16>(ah, bl[j], acc[ph][j]);
          acc[ph][j] = mfma16<PREC_BF16>(ah, bh[j], acc[ph][j]);
        }
      }
    }
    // outputs: lane holds input rows 16 wave + 4 q4 + r, column 16 j + l16 of each phase
    float* ob = P.out + (int64_t)b * 2 * T * P.cout;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = t0 + wave * 16 + q4 * 4 + r;
        float* orow = ob + (int64_t)(2 * v + P.off[ph]) * P.cout;
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          const int n = j * 16 + l16;
          if (v < T && n < P.cout) orow[n] = acc[ph][j][r] + bias_r[j];
        }
      }
    __syncthreads();  // every window read retired before the next store_x
  }
}

// ------------------------------------------------------------------------------------------------------ host
bool ups2_supported(int cin, int cout, int cpad, int rate, int taps) {
  if (rate != 2 || taps != 2) return false;
  return (cin == 96 && cpad == 96 && cout == 48) || (cin == 48 && cpad == 48 && cout == 24);
}

int ups2(const float* x, float* out, int B, int T, int cin, int cout, const u16* w0, const u16* w1, int64_t lo,
         int kpad, const int pad[2], const int off[2], const float* bias, hipStream_t s) {
  const int cpad = cin;
  if (!ups2_supported(cin, cout, cpad, 2, 2)) return set_error(ALCM_E_INVALID, "ups2: unsupported shape");
  if (!x || !out || !w0 || !w1 || !bias || B <= 0 || T <= 0 || kpad < 2 * cpad || (((uintptr_t)x) & 15) ||
      (((uintptr_t)w0) & 15) || (((uintptr_t)w1) & 15) || (lo % 8) || (kpad % 8))
    return set_error(ALCM_E_INVALID, "ups2: bad arguments");
  for (int r = 0; r < 2; ++r)
    if (pad[r] < 0 || pad[r] > 1 || off[r] < 0 || off[r] > 1) return set_error(ALCM_E_INVALID, "ups2: phase geometry");
  if ((int64_t)B * T * 2 * cout >= (1ll << 40)) return set_error(ALCM_E_INVALID, "ups2: problem too large");
  Ups2Dev P{};
  P.x = x; P.out = out; P.T = T; P.cin = cin; P.cout = cout;
  P.w[0] = w0; P.w[1] = w1; P.lo = lo; P.kpad = kpad;
  P.pad[0] = pad[0]; P.pad[1] = pad[1]; P.off[0] = off[0]; P.off[1] = off[1];
  P.bias = bias;
  P.tiles_per_batch = (T + 127) / 128;
  const int64_t nt = (int64_t)B * P.tiles_per_batch;
  if (nt >= (1ll << 30)) return set_error(ALCM_E_INVALID, "ups2: problem too large");
  P.ntiles = (int)nt;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0, n = 0;
    ncu = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
              ? n
              : 256;
  }
  const int grid = (int)std::min<int64_t>(nt, (int64_t)ncu * (cin == 96 ? UpsGeo<96, 48>::OCC : UpsGeo<48, 32>::OCC));
  void* tok = prof_start(s);
  if (cin == 96) hipLaunchKernelGGL((ups2_kernel<96, 48, 96>), dim3(grid), dim3(512), 0, s, P);
  else hipLaunchKernelGGL((ups2_kernel<48, 32, 48>), dim3(grid), dim3(512), 0, s, P);
  ALCM_HIP(hipGetLastError());
  if (tok) {
    const double M = (double)B * T;
    char name[64];
    std::snprintf(name, sizeof(name), "alcm::ups2_kernel<%d, %d, %d>", cpad, cin == 96 ? 48 : 32, cin);
    prof_stop(tok, s, name, 2.0 * 2.0 * M * cout * 2.0 * cin, M * cin * 4.0 + 2.0 * M * cout * 4.0);
  }
  return 0;
}

}  // namespace alcm
