// Fused anti-aliased activation + dilated conv1d for BigVGAN's narrow stages (C <= 96).
//
// One AMPBlock1 half-layer is  y = conv_{k,d}( Activation1d(x) ) + bias [+ residual]
// (vocoder/bigvgan/models.py:72-81, alias_free_torch/act.py:23-27), and conv_post is the same
// shape with Cout = 1 and tanh (models.py:201-203).  At C = 24/48/96 these layers move 1-2 GB
// through HBM per launch at B=32 and are HBM/VALU-bound once the MFMA part is efficient.
//
// Streaming design (one workgroup = 4 waves = one batch row b and a segment of R*BM output rows):
//   * the conv input window lives in an LDS *ring* of WRING rows (>= BM + (k-1)d) holding
//     Activation1d(x) as MFMA operand planes (bf16 hi/lo for PREC_SPLIT, fp16 for PREC_F16);
//     each sub-tile of BM output rows computes only the BM rows that enter the window
//     (the first sub-tile also the (k-1)d halo), so the activation runs ~once per element;
//   * the implicit GEMM runs over K = (tap, channel): A fragments are read from the ring at
//     row offset tap*d (per lane, modulo WRING), B (packed weights, L2-resident) is staged
//     per K-step into a double-buffered LDS tile shared by the 4 waves (one barrier per step);
//   * epilogue: bias, activation (tanh for conv_post), residual (prefetched before the K loop),
//     scale / accumulate (mean of the three resblocks), store.
// HBM traffic per layer: read x once (+ halo at segment starts), write y once (+ residual read).
#include <cstdio>
#include <cstdlib>

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
  int segs_per_batch, seg_tiles;
  int ablate;  // diagnostics only (env ALCM_AMP_ABLATE): bit0 skip activation, bit1 skip K loop, bit2 skip epilogue
};

// sin^2(x) with a Cody-Waite reduction to [-pi/4, pi/4] and minimax sin/cos polynomials (fp32, ~1 ulp)
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

// Activation1d (UpSample1d -> SnakeBeta -> DownSample1d, act.py:23-27) of one channel for AR
// consecutive output times j0 .. j0+AR-1 (xc = x + b*sb + c, row stride st); 0 outside [0, T)
// (that is the conv's zero padding, not the activation's replicate padding).
template <int AR, bool ACT>
__device__ __forceinline__ void act_run(const float* __restrict__ xc, int64_t st, int T, int j0, float ea, float ib,
                                        const Taps12A& f, float (&o)[AR]) {
  if (!ACT) {
#pragma unroll
    for (int r = 0; r < AR; ++r) {
      const int j = j0 + r;
      o[r] = (j >= 0 && j < T) ? xc[(int64_t)j * st] : 0.f;
    }
    return;
  }
  if (j0 >= 6 && j0 + AR + 6 <= T) {
    // interior: replicate padding never reached; upsampled sample q pairs with input window win
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
  // edges: explicit replicate padding of the up (pad 5) and down (pad 5/6) filters
  for (int r = 0; r < AR; ++r) {
    const int j = j0 + r;
    float acc = 0.f;
    if (j >= 0 && j < T) {
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

// LDS ring row stride (bf16 elements) == 8 mod 32: the 16 rows of an A-fragment read land on
// distinct 16-byte slots of each ds_read_b128 lane group for any start row
template <int CPAD>
struct RingRow {
  static constexpr int S = CPAD + 8 + ((8 - (CPAD + 8) % 32 + 32) % 32);
};

// B tile in LDS: NT rows x 32 k (64 B) per plane, 16-B chunk kq of row r at slot kq ^ ((r >> 2) & 2)
__device__ __forceinline__ int bt_off(int r, int kq) { return r * 32 + ((kq ^ ((r >> 2) & 2)) << 3); }

// Interior Activation1d from an LDS fp32 stage of x: xr points at the staged row of input time j0 - 6
// (channel c, row stride CPAD); the caller guarantees 6 <= j0 and j0 + AR + 6 <= T.
template <int AR, int CPAD>
__device__ __forceinline__ void act_run_lds(const float* xr, float ea, float ib, const Taps12A& f, float (&o)[AR]) {
  float win[AR + 12];
#pragma unroll
  for (int i = 0; i < AR + 12; ++i) win[i] = xr[i * CPAD];
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
}

// CPAD = Cin; wave grid WGM x WGN, each wave TM x TN 16x16 tiles; BM = WGM*TM*16 rows per sub-tile,
// NT = WGN*TN*16 >= Cout columns; AR activation rows per work item; WRING ring rows (power of 2);
// XR rows of x staged per activation chunk (XR >= BM + 12: one chunk per sub-tile after the first).
//
// Per sub-tile jt the workgroup runs  [activation of BM new rows from the x stage -> ring] ->
// [K loop; meanwhile the x rows of sub-tile jt+1 and this sub-tile's residual are loaded into
// registers] -> [epilogue through an LDS tile] -> [prefetched x -> x stage], so the HBM latency of
// the next activation and of the residual hides behind this sub-tile's MFMAs.
template <int CPAD, int WGM, int WGN, int TM, int TN, int AR, int WRING, int XR, int PREC, bool ACT>
__global__ __launch_bounds__(256) void amp_conv_kernel(const AmpDev P) {
  constexpr int BM = WGM * TM * 16;
  constexpr int NT = WGN * TN * 16;
  constexpr int NPA = PREC == PREC_SPLIT ? 2 : 1;                           // activation planes
  constexpr int NPB = (PREC == PREC_SPLIT || PREC == PREC_F16W2) ? 2 : 1;  // weight planes
  constexpr int S = RingRow<CPAD>::S;
  constexpr int BCH = NT * 4;  // 16-B chunks per B plane per K-step
  constexpr int BPER = (BCH + 255) / 256;
  constexpr int OTS = NT + 4;  // output-tile row stride (floats): spreads the acc writes over banks
  constexpr int CH = XR - 12;  // activation rows per x stage
  constexpr int C4 = CPAD / 4;
  constexpr int XPER = (XR * C4 + 255) / 256;         // prefetched float4 of x per thread
  constexpr int RPER = (BM * NT / 4 + 255) / 256;     // prefetched float4 of the residual per thread
  static_assert(WGM * WGN == 4, "4 waves");
  static_assert((WRING & (WRING - 1)) == 0 && WRING >= BM + 64, "ring must hold BM + max halo rows");
  static_assert(CPAD % 4 == 0 && CH >= BM, "x stage must hold one sub-tile of new rows");
  // scratch is time-shared: x stage (activation) / B double buffer (K loop) / output tile (epilogue)
  constexpr int SB_B = 2 * NPB * NT * 32 * 2, SB_X = XR * CPAD * 4, SB_O = BM * OTS * 4;
  constexpr int SB = SB_B > SB_X ? (SB_B > SB_O ? SB_B : SB_O) : (SB_X > SB_O ? SB_X : SB_O);
  __shared__ __attribute__((aligned(16))) __bf16 ring[NPA][WRING * S];
  __shared__ __attribute__((aligned(16))) char scratch[SB];
  __bf16* bsb = reinterpret_cast<__bf16*>(scratch);  // [2][NPB][NT*32]
  float* xs = reinterpret_cast<float*>(scratch);     // [XR][CPAD]
  float* ot = reinterpret_cast<float*>(scratch);     // [BM][OTS]
  auto bs = [&](int buf, int pl) { return bsb + (buf * NPB + pl) * NT * 32; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int b = blockIdx.x / P.segs_per_batch;
  const int seg = blockIdx.x - b * P.segs_per_batch;
  const int t_begin = seg * P.seg_tiles * BM;
  const int halo = (P.ksize - 1) * P.dil;
  const int tw0 = t_begin - P.pad;  // input time of relative window row 0
  const float* xb = P.x + (int64_t)b * P.x_sb;
  const int Kr = P.ksize * CPAD;
  const int nks = P.kpad / 32;
  const int Cout = P.Cout;
  const bool vec_out = (Cout % 4) == 0;

  // B staging (per K-step: rows n < Cout of the packed weight, k0 .. k0+31; zero rows beyond Cout)
  const u16* bsrc[BPER];
  bool bok[BPER];
#pragma unroll
  for (int i = 0; i < BPER; ++i) {
    const int c = tid + i * 256;
    const int n = c >> 2;
    bok[i] = c < BCH && n < Cout;
    bsrc[i] = P.w + (int64_t)(bok[i] ? n : 0) * P.kpad + (c & 3) * 8;
  }
  uint4 bh[BPER], bl[BPER];
  auto load_b = [&](int k0) {
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      bh[i] = make_uint4(0, 0, 0, 0);
      bl[i] = make_uint4(0, 0, 0, 0);
      if (bok[i]) {
        bh[i] = *reinterpret_cast<const uint4*>(bsrc[i] + k0);
        if (NPB == 2) bl[i] = *reinterpret_cast<const uint4*>(bsrc[i] + k0 + P.w_lo);
      }
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int c = tid + i * 256;
      if (c >= BCH) continue;
      const int off = bt_off(c >> 2, c & 3);
      *reinterpret_cast<uint4*>(bs(buf, 0) + off) = bh[i];
      if (NPB == 2) *reinterpret_cast<uint4*>(bs(buf, NPB - 1) + off) = bl[i];
    }
  };
  auto put_ring = [&](int row, int c, float v) {
    const int slot = row & (WRING - 1);
    if constexpr (PREC == PREC_F16 || PREC == PREC_F16W2) {
      ring[0][slot * S + c] = __builtin_bit_cast(__bf16, (_Float16)v);
    } else {
      const __bf16 h = (__bf16)v;
      ring[0][slot * S + c] = h;
      if (NPA == 2) ring[NPA - 1][slot * S + c] = (__bf16)(v - (float)h);
    }
  };
  // x rows [jx0, jx0 + nrows) -> registers (rows outside [0, T) read as 0)
  float4 xp[XPER];
  auto load_x = [&](int jx0, int nrows) {
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int e = tid + i * 256;
      const int rr = e / C4, c4 = e - rr * C4;
      const int j = jx0 + rr;
      xp[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rr < nrows && j >= 0 && j < P.T) xp[i] = *reinterpret_cast<const float4*>(xb + (int64_t)j * CPAD + c4 * 4);
    }
  };
  auto store_x = [&](int nrows) {
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int e = tid + i * 256;
      if (e < nrows * C4) *reinterpret_cast<float4*>(xs + e * 4) = xp[i];
    }
  };
  // activation of window rows [w, w + rows) from the x stage (staged row 0 = input time tw0 + w - 6)
  auto act_chunk = [&](int w, int rows) {
    const int runs = (rows + AR - 1) / AR;
    for (int e = tid; e < runs * CPAD; e += 256) {
      const int c = e % CPAD, run = e / CPAD;
      const int w0 = w + run * AR;
      const int j0 = tw0 + w0;
      float o[AR];
      if (!ACT) {
#pragma unroll
        for (int r = 0; r < AR; ++r) o[r] = xs[(run * AR + r + 6) * CPAD + c];
      } else if (j0 >= 6 && j0 + AR + 6 <= P.T) {
        act_run_lds<AR, CPAD>(xs + run * AR * CPAD + c, P.aexp[c], P.ibeta[c], P.f, o);
      } else {
        act_run<AR, true>(xb + c, CPAD, P.T, j0, P.aexp[c], P.ibeta[c], P.f, o);
      }
#pragma unroll
      for (int r = 0; r < AR; ++r)
        if (w0 + r < w + rows) put_ring(w0 + r, c, o[r]);
    }
  };

  // prologue: the first sub-tile's window rows [0, BM + halo), staged in chunks of CH rows
  int have = 0;
  {
    const int need = BM + halo;
    for (int w = 0; w < need; w += CH) {
      const int rows = min(CH, need - w);
      load_x(tw0 + w - 6, rows + 12);
      store_x(rows + 12);
      __syncthreads();
      if (!(P.ablate & 1)) act_chunk(w, rows);
      __syncthreads();
    }
    have = need;
  }

  for (int jt = 0; jt < P.seg_tiles; ++jt) {
    const int t0 = t_begin + jt * BM;
    if (t0 >= P.T) break;
    const bool next = jt + 1 < P.seg_tiles && t0 + BM < P.T;
    if (jt > 0) {
      // BM new rows [have, have + BM), staged at the end of the previous sub-tile
      if (!(P.ablate & 1)) act_chunk(have, BM);
      have += BM;
      __syncthreads();  // ring rows visible; x stage free for the B buffers
    }

    // ---- K loop, with the next sub-tile's x rows and this sub-tile's residual prefetched
    load_b(0);
    if (next) load_x(tw0 + have - 6, BM + 12);
    float4 rp[RPER];
    const int mrows = min(BM, P.T - t0);
    const float* rbp = P.res ? P.res + (int64_t)b * P.r_sb + (int64_t)t0 * Cout : nullptr;
    if (vec_out) {
      const int q4 = Cout / 4;
#pragma unroll
      for (int i = 0; i < RPER; ++i) {
        const int e = tid + i * 256;
        rp[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rbp && e < mrows * q4) rp[i] = *reinterpret_cast<const float4*>(rbp + (int64_t)e * 4);
      }
    }
    store_b(0);
    __syncthreads();
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int mrow = jt * BM + wm * TM * 16 + (lane & 15);  // relative window row of this lane's A rows (tap 0)
    for (int ks = 0; ks < ((P.ablate & 2) ? 0 : nks); ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nks) load_b((ks + 1) * 32);
      const int k8 = ks * 32 + 8 * (lane >> 4);
      const bool kok = k8 < Kr;
      const int tap = k8 / CPAD;
      const int ci = k8 - tap * CPAD;
      bf16x8 ah[TM], al[NPA == 2 ? TM : 1];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int off = ((mrow + i * 16 + tap * P.dil) & (WRING - 1)) * S + ci;
        if (kok) {
          ah[i] = *reinterpret_cast<const bf16x8*>(&ring[0][off]);
          if (NPA == 2) al[i] = *reinterpret_cast<const bf16x8*>(&ring[NPA - 1][off]);
        } else {
          ah[i] = bf16x8{};
          if (NPA == 2) al[i] = bf16x8{};
        }
      }
      bf16x8 fh[TN], fl[NPB == 2 ? TN : 1];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int off = bt_off(wn * TN * 16 + j * 16 + (lane & 15), lane >> 4);
        fh[j] = *reinterpret_cast<const bf16x8*>(bs(cur, 0) + off);
        if (NPB == 2) fl[j] = *reinterpret_cast<const bf16x8*>(bs(cur, NPB - 1) + off);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (PREC == PREC_SPLIT) {
            acc[i][j] = mfma16<PREC_BF16>(al[i], fh[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_BF16>(ah[i], fl[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_BF16>(ah[i], fh[j], acc[i][j]);
          } else if constexpr (PREC == PREC_F16W2) {
            acc[i][j] = mfma16<PREC_F16>(ah[i], fl[j], acc[i][j]);
            acc[i][j] = mfma16<PREC_F16>(ah[i], fh[j], acc[i][j]);
          } else {
            acc[i][j] = mfma16<PREC>(ah[i], fh[j], acc[i][j]);
          }
        }
      if (ks + 1 < nks) store_b(cur ^ 1);
      __syncthreads();  // also orders this sub-tile's ring reads before the next sub-tile's writes
    }
    if (P.ablate & 2) __syncthreads();

    // ---- epilogue: acc (+bias, out_act) -> LDS tile -> coalesced 16-B rows (+res, *scale, +out)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = wn * TN * 16 + j * 16 + (lane & 15);
          float v = acc[i][j][r];
          if (P.bias && n < Cout) v += P.bias[n];
          if (P.out_act) v = alcm_act(v, P.out_act);
          ot[m * OTS + n] = v;
        }
      }
    __syncthreads();
    float* ob = P.out + (int64_t)b * P.o_sb + (int64_t)t0 * Cout;
    if (!(P.ablate & 4)) {
      if (vec_out) {
        const int q4 = Cout / 4;
#pragma unroll
        for (int i = 0; i < RPER; ++i) {
          const int e = tid + i * 256;
          if (e >= mrows * q4) continue;
          const int m = e / q4, n = (e - m * q4) * 4;
          float4 v = *reinterpret_cast<const float4*>(ot + m * OTS + n);
          v.x += rp[i].x; v.y += rp[i].y; v.z += rp[i].z; v.w += rp[i].w;
          v.x *= P.out_scale; v.y *= P.out_scale; v.z *= P.out_scale; v.w *= P.out_scale;
          if (P.accumulate) {
            const float4 pv = *reinterpret_cast<const float4*>(ob + (int64_t)e * 4);
            v.x += pv.x; v.y += pv.y; v.z += pv.z; v.w += pv.w;
          }
          *reinterpret_cast<float4*>(ob + (int64_t)e * 4) = v;
        }
      } else {
        for (int e = tid; e < mrows * Cout; e += 256) {
          const int m = e / Cout, n = e - m * Cout;
          float v = ot[m * OTS + n];
          if (rbp) v += rbp[e];
          v *= P.out_scale;
          if (P.accumulate) v += ob[e];
          ob[e] = v;
        }
      }
    }
    __syncthreads();  // output tile (scratch) becomes the next sub-tile's x stage
    if (next) {
      store_x(BM + 12);
      __syncthreads();
    }
  }
}

template <int CPAD, int WGM, int WGN, int TM, int TN, int AR, int WRING, int XR, int PREC>
static void launch_amp_p(const AmpDev& Q, dim3 grid, bool act, hipStream_t s) {
  if (act)
    hipLaunchKernelGGL((amp_conv_kernel<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC, true>), grid, dim3(256), 0, s,
                       Q);
  else
    hipLaunchKernelGGL((amp_conv_kernel<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC, false>), grid, dim3(256), 0, s,
                       Q);
}

template <int CPAD, int WGM, int WGN, int TM, int TN, int AR, int WRING, int XR>
static void launch_amp(const AmpDev& P, int B, int prec, bool act, int force_tiles, hipStream_t s) {
  constexpr int BM = WGM * TM * 16;
  AmpDev Q = P;
  const int tiles = (P.T + BM - 1) / BM;
  // sub-tiles per workgroup: ~2.5k workgroups over the chip (>= 8 per CU), few halo recomputes
  int st = force_tiles > 0 ? force_tiles : std::max(1, (int)(((int64_t)tiles * B + 2559) / 2560));
  st = std::min(st, tiles);
  Q.seg_tiles = st;
  Q.segs_per_batch = (tiles + st - 1) / st;
  dim3 grid(B * Q.segs_per_batch);
  void* tok = prof_start(s);
  if (prec == PREC_SPLIT) launch_amp_p<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC_SPLIT>(Q, grid, act, s);
  else if (prec == PREC_F16) launch_amp_p<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC_F16>(Q, grid, act, s);
  else if (prec == PREC_F16W2) launch_amp_p<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC_F16W2>(Q, grid, act, s);
  else launch_amp_p<CPAD, WGM, WGN, TM, TN, AR, WRING, XR, PREC_BF16>(Q, grid, act, s);
  if (tok) {
    char name[128];
    std::snprintf(name, sizeof(name), "alcm::amp_conv_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %d, %s>", CPAD, WGM,
                  WGN, TM, TN, AR, WRING, XR, prec, act ? "true" : "false");
    const double elems = (double)B * P.T;
    const double flops = 2.0 * elems * P.Cout * (double)P.ksize * P.Cin;
    const double bytes = elems * (P.Cin + P.Cout * (1 + (P.res ? 1 : 0) + (P.accumulate ? 1 : 0))) * 4.0 +
                         (double)P.Cout * P.kpad * 2.0 * (prec == PREC_SPLIT || prec == PREC_F16W2 ? 2 : 1);
    prof_stop(tok, s, name, flops, bytes);
  }
}

int amp_conv(const alcm_amp_args& a, hipStream_t s) {
  if (!a.x || !a.w || !a.out || a.B <= 0 || a.T <= 0 || a.Cin <= 0 || a.Cout <= 0 || a.ksize <= 0 || a.dil <= 0)
    return set_error(ALCM_E_INVALID, "amp_conv: bad arguments");
  if (a.act && (!a.alpha_exp || !a.inv_beta || !a.up_filter || !a.down_filter))
    return set_error(ALCM_E_INVALID, "amp_conv: activation parameters missing");
  if ((a.ksize - 1) * a.dil > 64) return set_error(ALCM_E_INVALID, "amp_conv: receptive field too large");
  if (a.pad < 0 || a.pad > (a.ksize - 1) * a.dil) return set_error(ALCM_E_INVALID, "amp_conv: bad padding");
  const int cpad = round_up(a.Cin, 8);
  if (a.kpad < a.ksize * cpad || a.kpad % 32) return set_error(ALCM_E_INVALID, "amp_conv: kpad mismatch");
  if (a.x == a.out) return set_error(ALCM_E_INVALID, "amp_conv: in-place not supported");
  if (a.prec < PREC_BF16 || a.prec > PREC_F16W2) return set_error(ALCM_E_INVALID, "amp_conv: bad prec");
  if (a.seg_tiles < 0) return set_error(ALCM_E_INVALID, "amp_conv: seg_tiles must be >= 0");
  if ((int64_t)a.B * a.T * std::max(a.Cin, a.Cout) >= (1ll << 31))
    return set_error(ALCM_E_INVALID, "amp_conv: problem too large");
  AmpDev P{};
  P.x = a.x; P.x_sb = (int64_t)a.T * a.Cin; P.T = a.T; P.Cin = a.Cin;
  P.aexp = a.alpha_exp; P.ibeta = a.inv_beta;
  if (a.act)
    for (int k = 0; k < 12; ++k) {
      P.f.up[k] = a.up_filter[k];
      P.f.dn[k] = a.down_filter[k];
    }
  // PREC_F16 / PREC_F16W2 read the packed weight's fp16 hi (+ lo) planes (ptr + 2*w_lo_off, + 3*w_lo_off)
  P.w = (const u16*)a.w + ((a.prec == PREC_F16 || a.prec == PREC_F16W2) ? 2 * a.w_lo_off : 0);
  P.w_lo = a.w_lo_off;
  P.kpad = a.kpad; P.Cout = a.Cout; P.ksize = a.ksize;
  P.dil = a.dil; P.pad = a.pad; P.bias = a.bias; P.res = a.res; P.r_sb = (int64_t)a.T * a.Cout;
  P.out = a.out; P.o_sb = (int64_t)a.T * a.Cout; P.out_act = a.out_act; P.accumulate = a.accumulate;
  P.out_scale = a.out_scale;
  const int prec = a.prec;
  const bool act = a.act != 0;
  const int ft = a.seg_tiles;
  if (const char* ab = std::getenv("ALCM_AMP_ABLATE")) P.ablate = std::atoi(ab);
  if (cpad != a.Cin) return set_error(ALCM_E_INVALID, "amp_conv: Cin must be a multiple of 8");
  //                                            CPAD WGM WGN TM TN AR WRING XR
  if (a.Cin == 24 && a.Cout <= 16) launch_amp<24, 4, 1, 2, 1, 16, 256, 140>(P, a.B, prec, act, ft, s);
  else if (a.Cin == 24 && a.Cout <= 32) launch_amp<24, 4, 1, 2, 2, 16, 256, 140>(P, a.B, prec, act, ft, s);
  else if (a.Cin == 48 && a.Cout <= 48) launch_amp<48, 4, 1, 1, 3, 16, 128, 76>(P, a.B, prec, act, ft, s);
  else if (a.Cin == 96 && a.Cout <= 96) launch_amp<96, 2, 2, 2, 3, 8, 128, 76>(P, a.B, prec, act, ft, s);
  else return set_error(ALCM_E_INVALID, "amp_conv: unsupported channel count (24/48/96)");
  ALCM_HIP(hipGetLastError());
  return 0;
}

}  // namespace alcm

extern "C" int alcm_amp_conv(const alcm_amp_args* args, alcm_stream_t stream) {
  if (!args) return alcm::set_error(ALCM_E_INVALID, "null args");
  return alcm::amp_conv(*args, (hipStream_t)stream);
}
