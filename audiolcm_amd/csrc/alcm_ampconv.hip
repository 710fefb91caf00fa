// Fused anti-aliased activation + dilated conv1d for BigVGAN's narrow stages (C <= 96).
//
// One AMPBlock1 half-layer is  y = conv_{k,d}( Activation1d(x) ) + bias [+ residual]
// (vocoder/bigvgan/models.py:72-81, alias_free_torch/act.py:23-27).  At C = 24/48/96 these
// layers are HBM-bound; as separate kernels they moved x through HBM three times and re-read
// the conv input k times through L2.  Here one workgroup owns BM output rows x all channels:
//   1. the conv input window rows [t0 - pad, t0 + BM + (k-1)d - pad) are produced by the
//      Activation1d of x (up-FIR -> SnakeBeta -> down-FIR, evaluated from L1/L2-resident x),
//      zero outside [0, T) (the conv's zero padding), split to bf16 hi/lo straight into LDS;
//   2. the implicit GEMM runs over K = (tap, channel) reading A fragments from the window at
//      row offset tap*d and B fragments (packed weights, a few KB, L1/L2-hot) straight from
//      global memory: no barrier inside the K loop;
//   3. epilogue: bias, activation (tanh for conv_post), residual, scale/accumulate (mean of
//      the three resblocks), store.
// HBM traffic per layer: read x once (+ halo), write y once (+ residual read).
#include "alcm_common.h"
#include "alcm_internal.h"

namespace alcm {

struct Taps12A {
  float up[12], dn[12];
};

struct AmpDev {
  const float* x;
  int64_t x_sb;
  int T, Cin;
  const float* aexp;
  const float* ibeta;
  Taps12A f;
  const u16* w;
  int64_t w_lo;
  int kpad, Cout, ksize, dil, pad;
  const float* bias;
  const float* res;
  int64_t r_sb;
  float* out;
  int64_t o_sb;
  int out_act, accumulate;
  float out_scale;
  int tiles_per_batch;
};

__device__ __forceinline__ float amp_sin_sq(float x) {
  const float k = rintf(x * 0.63661977236758134f);
  float r = fmaf(-k, 1.5703125f, x);
  r = fmaf(-k, 4.837512969970703125e-4f, r);
  r = fmaf(-k, 7.54978995489188216e-8f, r);
  const float z = r * r;
  const float sn = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
  const float cs = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                  4.166664568298827e-2f), z, -0.5f), z, 1.0f);
  const float v = (((int)k) & 1) ? cs : sn;
  return v * v;
}

constexpr int AR = 16;  // activation outputs per work item

// Activation1d of channel c for window rows [w0, w0+AR): input time tt = tb + w, 0 outside [0,T).
template <bool ACT>
__device__ __forceinline__ void act_run(const float* __restrict__ xc, int64_t st, int T, int tb, int w0, int wr,
                                        float ea, float ib, const Taps12A& f, float (&o)[AR]) {
  const int j0 = tb + w0;
  if (!ACT) {
#pragma unroll
    for (int r = 0; r < AR; ++r) {
      const int j = j0 + r;
      o[r] = (j >= 0 && j < T && w0 + r < wr) ? xc[(int64_t)j * st] : 0.f;
    }
    return;
  }
  if (j0 >= 6 && j0 + AR + 6 <= T) {
    float win[AR + 12];
#pragma unroll
    for (int i = 0; i < AR + 12; ++i) win[i] = xc[(int64_t)(j0 - 6 + i) * st];
    float sv[2 * AR + 10];
#pragma unroll
    for (int q = 0; q < 2 * AR + 10; ++q) {
      float u = 0.f;
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        const int k = 2 * kk + (q & 1);
        u = fmaf(f.up[k], win[(q - k) / 2 + 6], u);
      }
      u *= 2.0f;
      sv[q] = u + ib * amp_sin_sq(u * ea);
    }
#pragma unroll
    for (int r = 0; r < AR; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 12; ++k) acc = fmaf(f.dn[k], sv[2 * r + k], acc);
      o[r] = acc;
    }
    return;
  }
  for (int r = 0; r < AR; ++r) {
    const int j = j0 + r;
    float acc = 0.f;
    if (j >= 0 && j < T && w0 + r < wr) {
      for (int k = 0; k < 12; ++k) {
        int m = 2 * j + k - 5;
        m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
        float u = 0.f;
        for (int kk = 0; kk < 6; ++kk) {
          const int ku = 2 * kk + ((m & 1) ? 0 : 1);
          int xi = (m + 5 - ku) / 2;
          xi = xi < 0 ? 0 : (xi > T - 1 ? T - 1 : xi);
          u = fmaf(f.up[ku], xc[(int64_t)xi * st], u);
        }
        u *= 2.0f;
        acc = fmaf(f.dn[k], u + ib * amp_sin_sq(u * ea), acc);
      }
    }
    o[r] = acc;
  }
}

// BM output rows per workgroup (4 waves x BM/4 rows), all Cout (<= TN*16) columns.
constexpr int AMP_WAVES = 8;  // 512-thread workgroups: one activation item per thread, more waves in flight
template <int BM, int TN, int CPAD, int PREC, bool ACT>
__global__ __launch_bounds__(64 * AMP_WAVES) void amp_conv_kernel(const AmpDev P) {
  constexpr int NT = 64 * AMP_WAVES;
  constexpr int WROWS = BM / AMP_WAVES;  // output rows per wave
  constexpr int TM = WROWS / 16;
  static_assert(TM >= 1 && WROWS % 16 == 0, "BM must give each wave a multiple of 16 rows");
  constexpr int S = CPAD + 8 + ((8 - (CPAD + 8) % 32 + 32) % 32);  // row stride (bf16) == 8 mod 32
  constexpr int WR_MAX = BM + 64;
  constexpr bool SPLIT = PREC == PREC_SPLIT;
  constexpr int NP = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 Wn[NP][WR_MAX * S];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / P.tiles_per_batch;
  const int t0 = (blockIdx.x - b * P.tiles_per_batch) * BM;
  const int WR = BM + (P.ksize - 1) * P.dil;
  const int tb = t0 - P.pad;
  const float* xb = P.x + (int64_t)b * P.x_sb;

  // ---- 1. activation window -> LDS (bf16 hi/lo)
  const int runs = (WR + AR - 1) / AR;
  const int items = runs * P.Cin;
  // residual of this lane's output elements: issued before the activation phase so its latency hides
  float resv[TM][4][TN];
  {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + wave * WROWS + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = j * 16 + (lane & 15);
          resv[i][r][j] = (P.res && t < P.T && n < P.Cout) ? P.res[(int64_t)b * P.r_sb + (int64_t)t * P.Cout + n] : 0.f;
        }
      }
  }
  for (int e = tid; e < items; e += NT) {
    const int c = e % P.Cin, run = e / P.Cin;
    float o[AR];
    act_run<ACT>(xb + c, P.Cin, P.T, tb, run * AR, WR, ACT ? P.aexp[c] : 0.f, ACT ? P.ibeta[c] : 0.f, P.f, o);
    // rows in [WR, runs*AR) are never read by the MFMAs; WR_MAX covers them, so no per-row guard
#pragma unroll
    for (int r = 0; r < AR; ++r) {
      const int w = run * AR + r;
      if constexpr (PREC == PREC_F16) {
        Wn[0][w * S + c] = __builtin_bit_cast(__bf16, (_Float16)o[r]);
      } else {
        const __bf16 h = (__bf16)o[r];
        Wn[0][w * S + c] = h;
        if (SPLIT) Wn[NP - 1][w * S + c] = (__bf16)(o[r] - (float)h);
      }
    }
  }
  __syncthreads();

  // ---- 2. implicit GEMM over K = (tap, channel), A from the window, B straight from global
  const int Kr = P.ksize * CPAD;
  const int row_base = wave * WROWS + (lane & 15);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const u16* wrow[TN];
  bool nok[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = j * 16 + (lane & 15);
    nok[j] = n < P.Cout;
    wrow[j] = P.w + (int64_t)(nok[j] ? n : 0) * P.kpad + 8 * (lane >> 4);
  }
  // B fragments are prefetched one K-step ahead (L1/L2 latency hidden behind the MFMAs)
  bf16x8 nbh[TN], nbl[SPLIT ? TN : 1];
  auto load_b = [&](int k0) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      uint4 h = make_uint4(0, 0, 0, 0), l = make_uint4(0, 0, 0, 0);
      if (nok[j]) {
        h = *reinterpret_cast<const uint4*>(wrow[j] + k0);
        if (SPLIT) l = *reinterpret_cast<const uint4*>(wrow[j] + k0 + P.w_lo);
      }
      nbh[j] = __builtin_bit_cast(bf16x8, h);
      if (SPLIT) nbl[j] = __builtin_bit_cast(bf16x8, l);
    }
  };
  load_b(0);
  for (int k0 = 0; k0 < P.kpad; k0 += 32) {
    bf16x8 bh[TN], bl[SPLIT ? TN : 1];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = nbh[j];
      if (SPLIT) bl[j] = nbl[j];
    }
    if (k0 + 32 < P.kpad) load_b(k0 + 32);
    const int k8 = k0 + 8 * (lane >> 4);
    const bool kok = k8 < Kr;
    const int tap = k8 / CPAD;
    const int ci = k8 - tap * CPAD;
    bf16x8 ah[TM], al[SPLIT ? TM : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (kok) {
        const int off = (row_base + i * 16 + tap * P.dil) * S + ci;
        ah[i] = *reinterpret_cast<const bf16x8*>(&Wn[0][off]);
        if (SPLIT) al[i] = *reinterpret_cast<const bf16x8*>(&Wn[NP - 1][off]);
      } else {
        ah[i] = bf16x8{};
        if (SPLIT) al[i] = bf16x8{};
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (SPLIT) {
          acc[i][j] = mfma16<PREC>(al[i], bh[j], acc[i][j]);
          acc[i][j] = mfma16<PREC>(ah[i], bl[j], acc[i][j]);
        }
        acc[i][j] = mfma16<PREC>(ah[i], bh[j], acc[i][j]);
      }
  }

  // ---- 3. epilogue
#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
    for (int r = 0; r < 4; ++r) {
      const int t = t0 + wave * WROWS + i * 16 + (lane >> 4) * 4 + r;
      if (t >= P.T) continue;
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + (lane & 15);
        if (n >= P.Cout) continue;
        float v = acc[i][j][r];
        if (P.bias) v += P.bias[n];
        if (P.out_act) v = alcm_act(v, P.out_act);
        v += resv[i][r][j];
        v *= P.out_scale;
        float* o = P.out + (int64_t)b * P.o_sb + (int64_t)t * P.Cout + n;
        if (P.accumulate) v += *o;
        *o = v;
      }
    }
  }
}

template <int BM, int TN, int CPAD, int PREC>
static void launch_amp_p(const AmpDev& Q, dim3 grid, bool act, hipStream_t s) {
  if (act) hipLaunchKernelGGL((amp_conv_kernel<BM, TN, CPAD, PREC, true>), grid, dim3(64 * AMP_WAVES), 0, s, Q);
  else hipLaunchKernelGGL((amp_conv_kernel<BM, TN, CPAD, PREC, false>), grid, dim3(64 * AMP_WAVES), 0, s, Q);
}

template <int BM, int TN, int CPAD>
static void launch_amp(const AmpDev& P, int B, int prec, bool act, hipStream_t s) {
  AmpDev Q = P;
  Q.tiles_per_batch = (P.T + BM - 1) / BM;
  dim3 grid(B * Q.tiles_per_batch);
  void* tok = prof_start(s);
  if (prec == PREC_SPLIT) launch_amp_p<BM, TN, CPAD, PREC_SPLIT>(Q, grid, act, s);
  else if (prec == PREC_F16) launch_amp_p<BM, TN, CPAD, PREC_F16>(Q, grid, act, s);
  else launch_amp_p<BM, TN, CPAD, PREC_BF16>(Q, grid, act, s);
  const bool split = prec == PREC_SPLIT;
  if (tok) {
    char name[128];
    std::snprintf(name, sizeof(name), "alcm::amp_conv_kernel<%d, %d, %d, %d, %s>", BM, TN, CPAD, prec,
                  act ? "true" : "false");
    const double elems = (double)B * P.T;
    const double flops = 2.0 * elems * P.Cout * (double)P.ksize * P.Cin;
    const double bytes = elems * (P.Cin + P.Cout * (1 + (P.res ? 1 : 0) + (P.accumulate ? 1 : 0))) * 4.0 +
                         (double)P.Cout * P.kpad * 2.0 * (split ? 2 : 1);
    prof_stop(tok, s, name, flops, bytes);
  }
}

int amp_conv(const alcm_amp_args& a, hipStream_t s) {
  if (!a.x || !a.w || !a.out || a.B <= 0 || a.T <= 0 || a.Cin <= 0 || a.Cout <= 0 || a.ksize <= 0 || a.dil <= 0)
    return set_error(ALCM_E_INVALID, "amp_conv: bad arguments");
  if (a.act && (!a.alpha_exp || !a.inv_beta || !a.up_filter || !a.down_filter))
    return set_error(ALCM_E_INVALID, "amp_conv: activation parameters missing");
  if ((a.ksize - 1) * a.dil > 64) return set_error(ALCM_E_INVALID, "amp_conv: receptive field too large");
  const int cpad = round_up(a.Cin, 8);
  if (a.kpad < a.ksize * cpad || a.kpad % 32) return set_error(ALCM_E_INVALID, "amp_conv: kpad mismatch");
  if (a.x == a.out) return set_error(ALCM_E_INVALID, "amp_conv: in-place not supported");
  AmpDev P{};
  P.x = a.x; P.x_sb = (int64_t)a.T * a.Cin; P.T = a.T; P.Cin = a.Cin;
  P.aexp = a.alpha_exp; P.ibeta = a.inv_beta;
  if (a.act)
    for (int k = 0; k < 12; ++k) {
      P.f.up[k] = a.up_filter[k];
      P.f.dn[k] = a.down_filter[k];
    }
  if (a.prec < PREC_BF16 || a.prec > PREC_F16) return set_error(ALCM_E_INVALID, "amp_conv: bad prec");
  // PREC_F16 reads the packed weight's fp16 plane (ptr + 2*w_lo_off)
  P.w = (const u16*)a.w + (a.prec == PREC_F16 ? 2 * a.w_lo_off : 0); P.w_lo = a.w_lo_off; P.kpad = a.kpad; P.Cout = a.Cout; P.ksize = a.ksize;
  P.dil = a.dil; P.pad = a.pad; P.bias = a.bias; P.res = a.res; P.r_sb = (int64_t)a.T * a.Cout;
  P.out = a.out; P.o_sb = (int64_t)a.T * a.Cout; P.out_act = a.out_act; P.accumulate = a.accumulate;
  P.out_scale = a.out_scale;
  const int split = a.prec;
  const bool act = a.act != 0;
  if (cpad != a.Cin) return set_error(ALCM_E_INVALID, "amp_conv: Cin must be a multiple of 8");
  if (a.Cin == 24 && a.Cout <= 16) launch_amp<256, 1, 24>(P, a.B, split, act, s);
  else if (a.Cin == 24 && a.Cout <= 32) launch_amp<256, 2, 24>(P, a.B, split, act, s);
  else if (a.Cin == 48 && a.Cout <= 48) launch_amp<128, 3, 48>(P, a.B, split, act, s);
  else if (a.Cin == 96 && a.Cout <= 96) launch_amp<128, 6, 96>(P, a.B, split, act, s);
  else return set_error(ALCM_E_INVALID, "amp_conv: unsupported channel count (24/48/96)");
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm

extern "C" int alcm_amp_conv(const alcm_amp_args* args, alcm_stream_t stream) {
  if (!args) return alcm::set_error(ALCM_E_INVALID, "null args");
  return alcm::amp_conv(*args, (hipStream_t)stream);
}
