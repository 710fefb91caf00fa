// MFMA implicit-GEMM for every contraction on the AudioLCM hot path (gfx950 / CDNA4).
//
//   C[m][n] = epilogue( sum_k A[m][k] * B[n][k] )
//
// One kernel template covers: conv1d of any kernel size / dilation / zero padding
// (implicit GEMM, K = tap*Cpad + ci), nearest-x2 upsample folded into the input index
// (Upsample1D, autoencoder1d.py:280-295), ConvTranspose1d as per-phase convolutions
// (BigVGAN ups, models.py:160-165), Linear layers, and the batched attention products
// Q K^T and P V (new_attention.py:114-126, autoencoder1d.py:265-274).
//
// Activations are fp32, channels-last (b, t, c) in HBM; operands are rounded to bf16 while
// they are staged into LDS and fed to v_mfma_f32_16x16x32_bf16 with fp32 accumulate.  With
// SPLIT each fp32 operand is carried as hi = bf16(x), lo = bf16(x - hi) and the product is
// hi*hi + hi*lo + lo*hi (3 MFMAs): ~2^-16 relative error, i.e. fp32-reference parity at 3x
// the bf16 MFMA cost (still 5.3x the f32-input MFMA rate).  PREC_F16 rounds both operands to fp16
// (11-bit significand, 8x smaller rounding error than bf16) and runs v_mfma_f32_16x16x32_f16 once:
// the per-layer precision policy (alcm_models.cpp) uses it where the parity budget allows.
//
// Prologue (A operand, applied on load): GroupNorm/LayerNorm affine + SiLU, so norm+act+conv
// is one pass over HBM.  Epilogue: bias, acc scale, activation, GEGLU pair gating
// (new_attention.py:48-55), residual add, output scale, accumulate (BigVGAN mean of
// resblocks, models.py:193-199), strided store (channels-last or NCT, conv-transpose phases).
#include <cstdio>
#include <cstring>

#include "alcm_common.h"
#include "audiolcm_hip.h"
#include "alcm_internal.h"

namespace alcm {

constexpr int BK = 32;
// GEMM tiles in LDS: rows of BK=32 bf16 (64 B, unpadded); the 16-B chunk kq of row r sits at chunk
// slot kq ^ ((r >> 2) & 2).  A ds_read_b128 fragment read (lane l: row l&15 of an aligned 16-row
// block, chunk l>>4) then hits 16 distinct 16-B bank slots in each of its four 16-lane groups
// ({0-3,12-15,20-27}, ...), i.e. it is conflict-free; the 80-B padded rows used before were 2-way.
constexpr int LDS_ROW = 32;
__device__ __forceinline__ int lds_off(int r, int kq) { return r * LDS_ROW + ((kq ^ ((r >> 2) & 2)) << 3); }
// Conv input window rows: 48 bf16 (96 B).  Fragment reads start at any row (offset tap*dil), so the
// layout must be conflict-free under translation: a 6-slot row stride is (16 rows x 4 chunks land on
// distinct slots per lane group for every start row), unlike 4 (64 B) or 5 (80 B).
constexpr int AW_ROW = 48;

// Prologue activation: the path only fuses SiLU (GroupNorm/LayerNorm + swish) into operand loads.
__device__ __forceinline__ float pro_act(float x, int act) { return act == ACT_SILU ? x / (1.0f + expf(-x)) : x; }

struct ActDev {
  const float* p;
  int64_t sb, st, sc;
  int T_in, C_in, Cpad, ksize, dil, pad, up, Kreal, M;
  FastDiv rpb, cpad;
  int64_t zs1, zs2;
  const float* ps;
  const float* ph;
  int64_t psb;
  const float* pm;
  const float* pr;
  int pact;
};
struct ActTDev {
  const float* p;
  int64_t st, sc;
  int Kext, rows;
  int64_t zs1, zs2;
};
struct WDev {
  const u16* p;
  int64_t lo;
  int rows, Kpad;
};
struct EpiDev {
  const float* bias;
  float acc_scale, out_scale;
  int act, accumulate, geglu;
  const float* res;
  int64_t r_sb, r_st, r_sc, r_zs1, r_zs2;
  float* out;
  int64_t o_sb, o_st, o_sc, o_zs1, o_zs2;
  FastDiv orpb;
  int out_step, out_off;
};
struct GemmDev {
  int M, N, Kpad;
  FastDiv zdiv;
  ActDev a;
  ActDev bact;
  ActTDev bT;
  WDev w;
  EpiDev e;
};

enum { BK_W = 0, BK_ACT = 1, BK_ACTT = 2 };

__device__ __forceinline__ int64_t zoff(const FastDiv& zd, int z, int64_t s1, int64_t s2) {
  uint32_t q, r;
  zd.divmod((uint32_t)z, q, r);
  return (int64_t)q * s1 + (int64_t)r * s2;
}

// fp32 -> MFMA operand planes: bf16 hi (+ bf16 lo for PREC_SPLIT) or fp16 (PREC_F16, in the hi plane)
template <int PREC>
__device__ __forceinline__ void prec_store(const float (&v)[8], __bf16* hi, __bf16* lo) {
  if constexpr (PREC == PREC_F16) {
    f16x8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)v[j];
    *reinterpret_cast<f16x8*>(hi) = h;
  } else {
    bf16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 bh = (__bf16)v[j];
      h[j] = bh;
      if (PREC == PREC_SPLIT) l[j] = (__bf16)(v[j] - (float)bh);
    }
    *reinterpret_cast<bf16x8*>(hi) = h;
    if (PREC == PREC_SPLIT) *reinterpret_cast<bf16x8*>(lo) = l;
  }
}

// ---------------------------------------------------------------- fp32 activation tile (conv taps)
template <int ROWS, bool VEC>
struct ActTile {
  static constexpr int CHUNKS = ROWS * 4;
  static constexpr int PER = (CHUNKS + 255) / 256;
  const float* base[PER];
  int t[PER];
  int b[PER];
  bool ok[PER];
  float v[PER][8];

  __device__ __forceinline__ void init(const ActDev& A, int tid, int row0, int64_t zo) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      const int r = row0 + (c >> 2);
      ok[i] = (c < CHUNKS) && (r < A.M);
      uint32_t bb = 0, tt = 0;
      if (ok[i]) A.rpb.divmod((uint32_t)r, bb, tt);
      b[i] = (int)bb;
      t[i] = (int)tt;
      base[i] = A.p + zo + (int64_t)bb * A.sb;
    }
  }
  __device__ __forceinline__ void load(const ActDev& A, int tid, int k0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      const int c = tid + i * 256;
      const int k = k0 + (c & 3) * 8;
      if (!ok[i] || k >= A.Kreal) continue;
      const int tap = (int)A.cpad.div((uint32_t)k);
      const int ci = k - tap * A.Cpad;
      int ts = t[i] + tap * A.dil - A.pad;
      if (A.up == 2) {
        if (ts < 0 || ts >= 2 * A.T_in) continue;
        ts >>= 1;
      } else if (ts < 0 || ts >= A.T_in) {
        continue;
      }
      const float* src = base[i] + (int64_t)ts * A.st;
      if (VEC) {
        const float4 x0 = *reinterpret_cast<const float4*>(src + ci);
        const float4 x1 = *reinterpret_cast<const float4*>(src + ci + 4);
        v[i][0] = x0.x; v[i][1] = x0.y; v[i][2] = x0.z; v[i][3] = x0.w;
        v[i][4] = x1.x; v[i][5] = x1.y; v[i][6] = x1.z; v[i][7] = x1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (ci + j < A.C_in) v[i][j] = src[(int64_t)(ci + j) * A.sc];
      }
      if (A.pm) {
        const int64_t ri = (int64_t)b[i] * A.T_in + ts;
        const float mu = A.pm[ri], rs = A.pr[ri];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (v[i][j] - mu) * rs;
      }
      if (A.ps) {
        const float* sc = A.ps + (int64_t)b[i] * A.psb + ci;
        const float* sh = A.ph + (int64_t)b[i] * A.psb + ci;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (VEC || ci + j < A.C_in) v[i][j] = v[i][j] * sc[j] + sh[j];
      }
      if (A.pact) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (VEC || ci + j < A.C_in) v[i][j] = pro_act(v[i][j], A.pact);
      }
    }
  }
  template <int PREC>
  __device__ __forceinline__ void store(__bf16* hi, __bf16* lo, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      if (c >= CHUNKS) continue;
      const int off = lds_off(c >> 2, c & 3);
      prec_store<PREC>(v[i], hi + off, lo + off);
    }
  }
};

// ---------------------------------------------------------------- fp32 N-contiguous tile (P V's V operand)
template <int ROWS>
struct ActTTile {
  static constexpr int CHUNKS = ROWS * 4;
  static constexpr int PER = (CHUNKS + 255) / 256;
  const float* base;
  float v[PER][8];
  __device__ __forceinline__ void init(const ActTDev& B, int tid, int row0, int64_t zo) { base = B.p + zo; }
  __device__ __forceinline__ void load(const ActTDev& B, int tid, int row0, int k0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      const int n = row0 + (c % ROWS);
      const int kk = k0 + (c / ROWS) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = (c < CHUNKS) && (n < B.rows) && (kk + j < B.Kext);
        v[i][j] = ok ? base[(int64_t)(kk + j) * B.st + (int64_t)n * B.sc] : 0.f;
      }
    }
  }
  template <int PREC>
  __device__ __forceinline__ void store(__bf16* hi, __bf16* lo, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      if (c >= CHUNKS) continue;
      const int off = lds_off(c % ROWS, c / ROWS);
      prec_store<PREC>(v[i], hi + off, lo + off);
    }
  }
};

// ---------------------------------------------------------------- packed bf16 weight tile
template <int ROWS>
struct WTile {
  static constexpr int CHUNKS = ROWS * 4;
  static constexpr int PER = (CHUNKS + 255) / 256;
  uint4 h[PER], l[PER];
  const u16* src[PER];
  bool ok[PER];
  __device__ __forceinline__ void init(const WDev& W, int tid, int row0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      const int r = row0 + (c >> 2);
      ok[i] = c < CHUNKS && r < W.rows;
      src[i] = W.p + (int64_t)(ok[i] ? r : 0) * W.Kpad + (c & 3) * 8;
    }
  }
  __device__ __forceinline__ void load(const WDev& W, int k0, bool split) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      h[i] = make_uint4(0, 0, 0, 0);
      l[i] = make_uint4(0, 0, 0, 0);
      if (ok[i]) {
        h[i] = *reinterpret_cast<const uint4*>(src[i] + k0);
        if (split) l[i] = *reinterpret_cast<const uint4*>(src[i] + k0 + W.lo);
      }
    }
  }
  template <int PREC>
  __device__ __forceinline__ void store(__bf16* hi, __bf16* lo, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 256;
      if (c >= CHUNKS) continue;
      const int off = lds_off(c >> 2, c & 3);
      *reinterpret_cast<uint4*>(hi + off) = h[i];
      if (PREC == PREC_SPLIT) *reinterpret_cast<uint4*>(lo + off) = l[i];
    }
  }
};

// ---------------------------------------------------------------- the kernel
template <int BM, int BN, int WM, int WN, bool AVEC, int BKIND, int PREC>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmDev P) {
  constexpr int TM = BM / (WM * 16);
  constexpr int TN = BN / (WN * 16);
  constexpr bool SPLIT = PREC == PREC_SPLIT;
  constexpr int NP = SPLIT ? 2 : 1;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) __bf16 As[2][NP][BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][NP][BN * LDS_ROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int row0 = blockIdx.x * BM;
  const int col0 = blockIdx.y * BN;
  const int z = blockIdx.z;

  ActTile<BM, AVEC> at;
  at.init(P.a, tid, row0, zoff(P.zdiv, z, P.a.zs1, P.a.zs2));
  ActTile<BN, true> bt_act;
  ActTTile<BN> bt_t;
  WTile<BN> bt_w;
  if constexpr (BKIND == BK_ACT) bt_act.init(P.bact, tid, col0, zoff(P.zdiv, z, P.bact.zs1, P.bact.zs2));
  if constexpr (BKIND == BK_ACTT) bt_t.init(P.bT, tid, col0, zoff(P.zdiv, z, P.bT.zs1, P.bT.zs2));
  if constexpr (BKIND == BK_W) bt_w.init(P.w, tid, col0);

  auto load_tiles = [&](int k0) {
    at.load(P.a, tid, k0);
    if constexpr (BKIND == BK_W) bt_w.load(P.w, k0, SPLIT);
    if constexpr (BKIND == BK_ACT) bt_act.load(P.bact, tid, k0);
    if constexpr (BKIND == BK_ACTT) bt_t.load(P.bT, tid, col0, k0);
  };
  auto store_tiles = [&](int buf) {
    at.template store<PREC>(As[buf][0], As[buf][NP - 1], tid);
    if constexpr (BKIND == BK_W) bt_w.template store<PREC>(Bs[buf][0], Bs[buf][NP - 1], tid);
    if constexpr (BKIND == BK_ACT) bt_act.template store<PREC>(Bs[buf][0], Bs[buf][NP - 1], tid);
    if constexpr (BKIND == BK_ACTT) bt_t.template store<PREC>(Bs[buf][0], Bs[buf][NP - 1], tid);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = P.Kpad / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int a_off = lds_off(wm * TM * 16 + (lane & 15), lane >> 4);
  const int b_off = lds_off(wn * TN * 16 + (lane & 15), lane >> 4);

  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) load_tiles((ks + 1) * BK);

    bf16x8 ah[TM], bh[TN];
    bf16x8 al[SPLIT ? TM : 1], bl[SPLIT ? TN : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(&As[cur][0][a_off + i * 16 * LDS_ROW]);
      if constexpr (SPLIT) al[i] = *reinterpret_cast<const bf16x8*>(&As[cur][NP - 1][a_off + i * 16 * LDS_ROW]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][0][b_off + j * 16 * LDS_ROW]);
      if constexpr (SPLIT) bl[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][NP - 1][b_off + j * 16 * LDS_ROW]);
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

    if (ks + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const EpiDev& E = P.e;
  const int64_t ozo = zoff(P.zdiv, z, E.o_zs1, E.o_zs2);
  const int64_t rzo = E.res ? zoff(P.zdiv, z, E.r_zs1, E.r_zs2) : 0;
#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
      const bool mok = m < P.M;
      uint32_t bb = 0, tt = 0;
      if (mok) E.orpb.divmod((uint32_t)m, bb, tt);
      const int64_t to = (int64_t)tt * E.out_step + E.out_off;
      const int64_t obase = ozo + (int64_t)bb * E.o_sb + to * E.o_st;
      const int64_t rbase = rzo + (int64_t)bb * E.r_sb + to * E.r_st;
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j) {
        const int n = col0 + wn * TN * 16 + j * 16 + (lane & 15);
        float v = acc[i][j][r] * E.acc_scale;
        if (E.bias && n < P.N) v += E.bias[n];
        int nout = n;
        bool st = mok && n < P.N;
        if (E.geglu) {
          const float g = __shfl_xor(v, 1);
          v = v * alcm_act(g, E.geglu == 2 ? ACT_GELU_TANH : ACT_GELU_ERF);
          st = st && ((lane & 1) == 0);
          nout = n >> 1;
        } else if (E.act) {
          v = alcm_act(v, E.act);
        }
        if (st) {
          if (E.res) v += E.res[rbase + (int64_t)nout * E.r_sc];
          v *= E.out_scale;
          float* o = E.out + obase + (int64_t)nout * E.o_sc;
          if (E.accumulate) v += *o;
          *o = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- skinny GEMM (M <= 64 rows, k = 1)
// The DiT embedder MLPs run at M = B rows (concatDiT.py TimestepEmbedder / proj_w: Linear -> SiLU -> Linear): on the
// MFMA tiles a 32-row problem is 1-5 workgroups walking K serially (45 us a launch, latency-bound).  Here a
// workgroup owns 32 output columns x 32 rows: A (32 x Kpad fp32, zero past C_in) staged once in LDS, 256 threads =
// 32 columns x 8 K slices, fp32 FMAs of the A element (rounded to the operand format for BF16 / F16 like the MFMA
// path; SPLIT keeps fp32) with the weight's value in that format (SPLIT: bf16 hi + lo), the slices' partials added in
// slice order, then the MFMA kernels' epilogue (acc_scale, bias, act, residual, out_scale, accumulate).
// Rows in blocks of SK_M (grid.y), so which rows share a launch never changes a row's arithmetic: the result is
// invariant to how a batch is split (eligibility depends on K and the layer, not on M up to SK_MAXM rows).
constexpr int SK_N = 32, SK_M = 32, SK_KMAX = 768, SK_MAXM = 1024;  // columns / rows per workgroup, K and M limits
template <int PREC>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const GemmDev P) {
  __shared__ __attribute__((aligned(16))) float sm[SK_M * SK_KMAX];
  const int tid = threadIdx.x, c = tid & 31, ks = tid >> 5;
  const int n = blockIdx.x * SK_N + c;
  const int m0 = blockIdx.y * SK_M;
  const int M = min(P.M - m0, SK_M), K = P.Kpad;
  const ActDev& A = P.a;
  // A staged as float4 pieces (rows channel-contiguous, C_in % 4 == 0: checked by the host), eight loads in flight per
  // thread before their stores (one at a time, each store waited on its load: 72 serialised L2 trips a launch)
  const int K4 = K >> 2, n4 = M * K4;
  for (int e0 = tid; e0 < n4; e0 += 256 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < n4) {
        const int m = e / K4, k = (e - m * K4) * 4;
        if (k < A.C_in) {
          uint32_t b, t;
          A.rpb.divmod((uint32_t)(m0 + m), b, t);
          v[u] = *reinterpret_cast<const float4*>(A.p + (int64_t)b * A.sb + (int64_t)t * A.st + k);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256;
      if (e >= n4) continue;
      float4 x = v[u];
      if constexpr (PREC == PREC_F16) {
        x.x = (float)(_Float16)x.x; x.y = (float)(_Float16)x.y; x.z = (float)(_Float16)x.z; x.w = (float)(_Float16)x.w;
      }
      if constexpr (PREC == PREC_BF16) {
        x.x = (float)(__bf16)x.x; x.y = (float)(__bf16)x.y; x.z = (float)(__bf16)x.z; x.w = (float)(__bf16)x.w;
      }
      *reinterpret_cast<float4*>(sm + 4 * e) = x;
    }
  }
  __syncthreads();
  float acc[SK_M];
#pragma unroll
  for (int m = 0; m < SK_M; ++m) acc[m] = 0.f;
  const bool nok = n < P.N;
  // the weight pieces one K step ahead (the next step's loads in flight under this step's FMAs)
  const u16* wrow = P.w.p + (int64_t)(nok ? n : 0) * K;
  bf16x8 hn = {}, ln = {};
  if (nok && 8 * ks < K) {
    hn = *reinterpret_cast<const bf16x8*>(wrow + 8 * ks);
    if constexpr (PREC == PREC_SPLIT) ln = *reinterpret_cast<const bf16x8*>(wrow + P.w.lo + 8 * ks);
  }
  for (int k0 = 8 * ks; k0 < K; k0 += 64) {
    const bf16x8 h = hn, l = ln;
    if (nok && k0 + 64 < K) {
      hn = *reinterpret_cast<const bf16x8*>(wrow + k0 + 64);
      if constexpr (PREC == PREC_SPLIT) ln = *reinterpret_cast<const bf16x8*>(wrow + P.w.lo + k0 + 64);
    }
    float w[8];
    if constexpr (PREC == PREC_F16) {
      const f16x8 hf = __builtin_bit_cast(f16x8, h);
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = (float)hf[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = (float)h[j];
      if constexpr (PREC == PREC_SPLIT) {
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] += (float)l[j];
      }
    }
#pragma unroll
    for (int m = 0; m < SK_M; ++m) {
      if (m < M) {
        const float4 a0 = *reinterpret_cast<const float4*>(sm + m * K + k0);
        const float4 a1 = *reinterpret_cast<const float4*>(sm + m * K + k0 + 4);
        float v = acc[m];
        v = fmaf(a0.x, w[0], v); v = fmaf(a0.y, w[1], v); v = fmaf(a0.z, w[2], v); v = fmaf(a0.w, w[3], v);
        v = fmaf(a1.x, w[4], v); v = fmaf(a1.y, w[5], v); v = fmaf(a1.z, w[6], v); v = fmaf(a1.w, w[7], v);
        acc[m] = v;
      }
    }
  }
  __syncthreads();  // every A read done: the buffer takes the 8 slices' partials [slice][row][column]
#pragma unroll
  for (int m = 0; m < SK_M; ++m)
    if (m < M) sm[(ks * SK_M + m) * SK_N + c] = acc[m];
  __syncthreads();
  const EpiDev& E = P.e;
  for (int m = ks; m < M; m += 8) {
    float v = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) v += sm[(s2 * SK_M + m) * SK_N + c];
    if (!nok) continue;
    uint32_t bb = 0, tt = 0;
    E.orpb.divmod((uint32_t)(m0 + m), bb, tt);
    const int64_t to = (int64_t)tt * E.out_step + E.out_off;
    v *= E.acc_scale;
    if (E.bias) v += E.bias[n];
    if (E.act) v = alcm_act(v, E.act);
    if (E.res) v += E.res[(int64_t)bb * E.r_sb + to * E.r_st + (int64_t)n * E.r_sc];
    v *= E.out_scale;
    float* o = E.out + (int64_t)bb * E.o_sb + to * E.o_st + (int64_t)n * E.o_sc;
    if (E.accumulate) v += *o;
    *o = v;
  }
}

// ---------------------------------------------------------------- window convolution (ksize > 1)
// Implicit GEMM for conv1d with k taps where the A operand of every tap is a shifted view of
// one input window: for each 32-channel chunk the rows [t0 - pad, t0 + BM + (k-1)*dil - pad)
// are loaded, normalised/activated (prologue) and split to bf16 hi/lo ONCE into LDS, and the k
// taps then read it at row offset tap*dil.  Compared with the tap-by-tap loader this cuts the A
// global loads, the fp32->bf16 conversions and the A LDS writes by k (k = 3..11 on the path).
// Tiles never straddle a batch (grid.x = B * ceil(T_out / BM)); K order = (chunk, tap).
constexpr int HALO_MAX = 64;

template <int BM, int BN, int WM, int WN, int PREC, bool PRO>
__global__ __launch_bounds__(256) void conv_kernel(const GemmDev P, int tiles_per_batch, int T_out) {
  constexpr int TM = BM / (WM * 16);
  constexpr int TN = BN / (WN * 16);
  constexpr bool SPLIT = PREC == PREC_SPLIT;
  constexpr int NP = SPLIT ? 2 : 1;
  constexpr int WR_MAX = BM + HALO_MAX;
  constexpr int WCH = WR_MAX * 4;
  constexpr int WPER = (WCH + 255) / 256;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) __bf16 Aw[NP][WR_MAX * AW_ROW];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][NP][BN * LDS_ROW];

  const ActDev& A = P.a;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int b = blockIdx.x / tiles_per_batch;
  const int t0 = (blockIdx.x - b * tiles_per_batch) * BM;
  const int col0 = blockIdx.y * BN;
  const int WR = BM + (A.ksize - 1) * A.dil;
  const int nC = A.Cpad / 32;
  const int K = A.ksize;

  // per-thread window rows (fixed across channel chunks): source pointer or null for zero padding
  const float* wsrc[WPER];
  int wrow[WPER];
#pragma unroll
  for (int i = 0; i < WPER; ++i) {
    const int c = tid + i * 256;
    const int w = c >> 2;
    const int tu = t0 + w - A.pad;
    int ts = -1;
    if (c < WCH && w < WR) {
      if (A.up == 2) ts = (tu >= 0 && tu < 2 * A.T_in) ? (tu >> 1) : -1;
      else ts = (tu >= 0 && tu < A.T_in) ? tu : -1;
    }
    wrow[i] = ts;
    wsrc[i] = ts >= 0 ? A.p + (int64_t)b * A.sb + (int64_t)ts * A.st + (c & 3) * 8 : nullptr;
  }
  float wv[WPER][8];
  auto load_window = [&](int cc) {
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      if (wsrc[i]) {
        const float4 x0 = *reinterpret_cast<const float4*>(wsrc[i] + cc * 32);
        const float4 x1 = *reinterpret_cast<const float4*>(wsrc[i] + cc * 32 + 4);
        wv[i][0] = x0.x; wv[i][1] = x0.y; wv[i][2] = x0.z; wv[i][3] = x0.w;
        wv[i][4] = x1.x; wv[i][5] = x1.y; wv[i][6] = x1.z; wv[i][7] = x1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) wv[i][j] = 0.f;
      }
    }
  };
  // prologue (normalise / affine / SiLU) is applied at store time so the loads stay in flight
  // behind the previous chunk's MFMAs; zero-padding rows stay exactly zero
  auto store_window = [&](int cc) {
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int c = tid + i * 256;
      const int w = c >> 2, kc = c & 3;
      if (c >= WCH || w >= WR) continue;
      if constexpr (PRO) {
        if (wrow[i] >= 0) {
          const int ci = cc * 32 + kc * 8;
          if (A.pm) {
            const int64_t ri = (int64_t)b * A.T_in + wrow[i];
            const float mu = A.pm[ri], rs = A.pr[ri];
#pragma unroll
            for (int j = 0; j < 8; ++j) wv[i][j] = (wv[i][j] - mu) * rs;
          }
          if (A.ps) {
            const float* sc = A.ps + (int64_t)b * A.psb + ci;
            const float* sh = A.ph + (int64_t)b * A.psb + ci;
#pragma unroll
            for (int j = 0; j < 8; ++j) wv[i][j] = wv[i][j] * sc[j] + sh[j];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) wv[i][j] = pro_act(wv[i][j], A.pact);
        }
      }
      prec_store<PREC>(wv[i], Aw[0] + w * AW_ROW + kc * 8, Aw[NP - 1] + w * AW_ROW + kc * 8);
    }
  };

  WTile<BN> bt;
  bt.init(P.w, tid, col0);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_window(0);
  bt.load(P.w, 0, SPLIT);
  store_window(0);
  bt.template store<PREC>(Bs[0][0], Bs[0][NP - 1], tid);
  __syncthreads();

  const int a_base = (wm * TM * 16 + (lane & 15)) * AW_ROW + (lane >> 4) * 8;
  const int b_off = lds_off(wn * TN * 16 + (lane & 15), lane >> 4);
  int cur = 0;
  for (int cc = 0; cc < nC; ++cc) {
    const bool next_win = cc + 1 < nC;
    if (next_win) load_window(cc + 1);
    for (int tap = 0; tap < K; ++tap) {
      const bool last_tap = tap + 1 == K;
      const bool more = !last_tap || next_win;
      if (more) bt.load(P.w, last_tap ? (cc + 1) * 32 : (tap + 1) * A.Cpad + cc * 32, SPLIT);

      const int a_off = a_base + tap * A.dil * AW_ROW;
      bf16x8 ah[TM], bh[TN];
      bf16x8 al[SPLIT ? TM : 1], bl[SPLIT ? TN : 1];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const bf16x8*>(&Aw[0][a_off + i * 16 * AW_ROW]);
        if constexpr (SPLIT) al[i] = *reinterpret_cast<const bf16x8*>(&Aw[NP - 1][a_off + i * 16 * AW_ROW]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][0][b_off + j * 16 * LDS_ROW]);
        if constexpr (SPLIT) bl[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][NP - 1][b_off + j * 16 * LDS_ROW]);
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

      if (more) bt.template store<PREC>(Bs[cur ^ 1][0], Bs[cur ^ 1][NP - 1], tid);
      if (last_tap && next_win) {
        __syncthreads();
        store_window(cc + 1);
      }
      __syncthreads();
      cur ^= 1;
    }
  }

  // epilogue (rows are (b, t0 + local) directly)
  const EpiDev& E = P.e;
#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
    for (int r = 0; r < 4; ++r) {
      const int tt = t0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
      const bool mok = tt < T_out;
      const int64_t to = (int64_t)tt * E.out_step + E.out_off;
      const int64_t obase = (int64_t)b * E.o_sb + to * E.o_st;
      const int64_t rbase = (int64_t)b * E.r_sb + to * E.r_st;
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j) {
        const int n = col0 + wn * TN * 16 + j * 16 + (lane & 15);
        float v = acc[i][j][r] * E.acc_scale;
        if (E.bias && n < P.N) v += E.bias[n];
        int nout = n;
        bool st = mok && n < P.N;
        if (E.geglu) {
          const float g = __shfl_xor(v, 1);
          v = v * alcm_act(g, E.geglu == 2 ? ACT_GELU_TANH : ACT_GELU_ERF);
          st = st && ((lane & 1) == 0);
          nout = n >> 1;
        } else if (E.act) {
          v = alcm_act(v, E.act);
        }
        if (st) {
          if (E.res) v += E.res[rbase + (int64_t)nout * E.r_sc];
          v *= E.out_scale;
          float* o = E.out + obase + (int64_t)nout * E.o_sc;
          if (E.accumulate) v += *o;
          *o = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- host side
static bool fill_act(const alcm_operand& o, int M, ActDev& d, std::string& err) {
  d.p = (const float*)o.ptr;
  d.sb = o.sb; d.st = o.st; d.sc = o.sc;
  d.T_in = o.T_in; d.C_in = o.C_in; d.Cpad = o.Cpad; d.ksize = o.ksize; d.dil = o.dil;
  d.pad = o.pad; d.up = o.up ? o.up : 1;
  d.Kreal = o.ksize * o.Cpad;
  d.M = M;
  d.rpb = FastDiv((uint32_t)(o.rows_per_batch > 0 ? o.rows_per_batch : 1));
  d.cpad = FastDiv((uint32_t)(o.Cpad > 0 ? o.Cpad : 1));
  d.zs1 = o.zs1; d.zs2 = o.zs2;
  d.ps = o.pro_scale; d.ph = o.pro_shift; d.psb = o.pro_sb;
  d.pm = o.pro_mean; d.pr = o.pro_rstd; d.pact = o.pro_act;
  if (!o.ptr || o.Cpad <= 0 || o.Cpad % 8 || o.C_in > o.Cpad || o.ksize <= 0 || o.T_in <= 0 ||
      (d.up != 1 && d.up != 2) || o.rows_per_batch <= 0) {
    err = "bad ACT operand geometry";
    return false;
  }
  if (o.pro_act != ACT_NONE && o.pro_act != ACT_SILU) {
    err = "prologue activation must be NONE or SILU";
    return false;
  }
  if ((o.pro_scale == nullptr) != (o.pro_shift == nullptr) || (o.pro_mean == nullptr) != (o.pro_rstd == nullptr)) {
    err = "prologue scale/shift and mean/rstd must come in pairs";
    return false;
  }
  return true;
}

static bool act_vec_ok(const alcm_operand& o) {
  const bool al = (((uintptr_t)o.ptr) & 15) == 0;
  return al && o.sc == 1 && o.C_in == o.Cpad && o.Cpad % 8 == 0 && o.st % 4 == 0 && o.sb % 4 == 0 &&
         o.zs1 % 4 == 0 && o.zs2 % 4 == 0;
}

struct LaunchCost {
  double flops, bytes;
};
static thread_local LaunchCost g_cost;

template <int BM, int BN, int WM, int WN, bool AVEC, int BKIND, int PREC>
static void launch_one(const GemmDev& P, int batch, int ncols, hipStream_t s) {
  dim3 grid((P.M + BM - 1) / BM, (ncols + BN - 1) / BN, batch);
  void* tok = prof_start(s);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AVEC, BKIND, PREC>), grid, dim3(256), 0, s, P);
  if (tok) {
    // the demangled name rocprofv3 prints for this instantiation
    char name[128];
    std::snprintf(name, sizeof(name), "alcm::gemm_kernel<%d, %d, %d, %d, %s, %d, %d>", BM, BN, WM, WN,
                  AVEC ? "true" : "false", BKIND, PREC);
    if (knobs().prof_shapes)  // diagnostics: split the statistics per problem shape
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " M%d N%d K%d x%d", P.M, ncols,
                    P.Kpad, batch);
    prof_stop(tok, s, name, g_cost.flops, g_cost.bytes);
  }
}

template <int BM, int BN, int WM, int WN, bool AVEC, int BKIND>
static void launch_split(const GemmDev& P, int batch, int ncols, int prec, hipStream_t s) {
  if (prec == PREC_SPLIT) launch_one<BM, BN, WM, WN, AVEC, BKIND, PREC_SPLIT>(P, batch, ncols, s);
  else if (prec == PREC_F16) launch_one<BM, BN, WM, WN, AVEC, BKIND, PREC_F16>(P, batch, ncols, s);
  else launch_one<BM, BN, WM, WN, AVEC, BKIND, PREC_BF16>(P, batch, ncols, s);
}

template <int BM, int BN, int WM, int WN, int PREC, bool PRO>
static void launch_conv(const GemmDev& P, int nbatch, int T_out, hipStream_t s) {
  const int tpb = (T_out + BM - 1) / BM;
  dim3 grid(nbatch * tpb, (P.N + BN - 1) / BN, 1);
  void* tok = prof_start(s);
  hipLaunchKernelGGL((conv_kernel<BM, BN, WM, WN, PREC, PRO>), grid, dim3(256), 0, s, P, tpb, T_out);
  if (tok) {
    char name[128];
    std::snprintf(name, sizeof(name), "alcm::conv_kernel<%d, %d, %d, %d, %d, %s>", BM, BN, WM, WN, PREC,
                  PRO ? "true" : "false");
    if (knobs().prof_shapes)
      std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " T%d N%d K%d k%d up%d x%d", T_out,
                    P.N, P.Kpad, P.a.ksize, P.a.up, nbatch);
    prof_stop(tok, s, name, g_cost.flops, g_cost.bytes);
  }
}

template <int BM, int BN, int WM, int WN, bool PRO>
static void launch_conv_sp(const GemmDev& P, int nbatch, int T_out, int prec, hipStream_t s) {
  if (prec == PREC_SPLIT) launch_conv<BM, BN, WM, WN, PREC_SPLIT, PRO>(P, nbatch, T_out, s);
  else if (prec == PREC_F16) launch_conv<BM, BN, WM, WN, PREC_F16, PRO>(P, nbatch, T_out, s);
  else launch_conv<BM, BN, WM, WN, PREC_BF16, PRO>(P, nbatch, T_out, s);
}

int gemm(const alcm_gemm_args& g, hipStream_t s) {
  std::string err;
  if (g.M <= 0 || g.N <= 0) return 0;
  if (g.Kpad <= 0 || g.Kpad % BK) return set_error(ALCM_E_INVALID, "Kpad must be a positive multiple of 32");
  if (g.a.kind != ALCM_OPND_ACT) return set_error(ALCM_E_INVALID, "A operand must be ACT");
  if (!g.out) return set_error(ALCM_E_INVALID, "null output");
  if (g.geglu && (g.N % 2)) return set_error(ALCM_E_INVALID, "geglu needs even N");
  GemmDev P{};
  P.M = g.M; P.N = g.N; P.Kpad = g.Kpad;
  const int batch = g.batch > 0 ? g.batch : 1;
  P.zdiv = FastDiv((uint32_t)(g.zdiv > 0 ? g.zdiv : 1));
  if (!fill_act(g.a, g.M, P.a, err)) return set_error(ALCM_E_INVALID, "A: " + err);
  if (P.a.Kreal > g.Kpad) return set_error(ALCM_E_INVALID, "Kpad smaller than ksize*Cpad of A");
  int bkind;
  if (g.b.kind == ALCM_OPND_WEIGHT) {
    bkind = BK_W;
    // PREC_F16 reads the fp16 plane (third plane of the packed weight) in place of bf16 hi
    P.w.p = (const u16*)g.b.ptr + (g.prec == PREC_F16 ? 2 * g.b.w_lo_off : 0);
    P.w.lo = g.b.w_lo_off; P.w.rows = g.b.rows; P.w.Kpad = g.Kpad;
    if (!g.b.ptr || g.b.rows < g.N) return set_error(ALCM_E_INVALID, "weight operand rows < N");
    if ((((uintptr_t)g.b.ptr) & 15) || (g.b.w_lo_off % 8)) return set_error(ALCM_E_INVALID, "weight alignment");
  } else if (g.b.kind == ALCM_OPND_ACT) {
    bkind = BK_ACT;
    if (!fill_act(g.b, g.N, P.bact, err)) return set_error(ALCM_E_INVALID, "B: " + err);
    if (!act_vec_ok(g.b) || g.b.ksize != 1 || g.b.pro_scale || g.b.pro_mean)
      return set_error(ALCM_E_INVALID, "B ACT operand must be channel-contiguous, 16B aligned, k=1, no prologue");
    if (P.bact.Kreal > g.Kpad) return set_error(ALCM_E_INVALID, "Kpad smaller than B K");
  } else if (g.b.kind == ALCM_OPND_ACT_T) {
    bkind = BK_ACTT;
    P.bT.p = (const float*)g.b.ptr; P.bT.st = g.b.st; P.bT.sc = g.b.sc; P.bT.Kext = g.b.T_in;
    P.bT.rows = g.b.rows; P.bT.zs1 = g.b.zs1; P.bT.zs2 = g.b.zs2;
    if (!g.b.ptr || g.b.rows < g.N) return set_error(ALCM_E_INVALID, "ACT_T operand rows < N");
  } else {
    return set_error(ALCM_E_INVALID, "unknown B operand kind");
  }
  EpiDev& E = P.e;
  E.bias = g.bias; E.acc_scale = g.acc_scale; E.out_scale = g.out_scale; E.act = g.act;
  E.accumulate = g.accumulate; E.geglu = g.geglu; E.res = g.res;
  E.r_sb = g.r_sb; E.r_st = g.r_st; E.r_sc = g.r_sc; E.r_zs1 = g.r_zs1; E.r_zs2 = g.r_zs2;
  E.out = g.out; E.o_sb = g.o_sb; E.o_st = g.o_st; E.o_sc = g.o_sc; E.o_zs1 = g.o_zs1; E.o_zs2 = g.o_zs2;
  E.orpb = FastDiv((uint32_t)(g.out_rows_per_batch > 0 ? g.out_rows_per_batch : 1));
  E.out_step = g.out_step ? g.out_step : 1;
  E.out_off = g.out_off;

  const bool avec = act_vec_ok(g.a);
  if (g.prec < PREC_BF16 || g.prec > PREC_F16) return set_error(ALCM_E_INVALID, "prec must be 0 (bf16), 1 (split) or 2 (f16)");
  const int split = g.prec;  // precision code passed down to the launchers
  const int N = g.N;
  if (prof_enabled()) {
    // algorithmic work of this launch: 2*M*N*K_real MACs; unique A rows, B operand, output (+residual/acc)
    const double Kr = (double)g.a.ksize * g.a.C_in;
    const double nb = (double)batch;
    const double a_rows = (double)g.a.T_in * ((double)g.M / std::max(1, g.a.rows_per_batch));
    double bbytes;
    if (bkind == BK_W) bbytes = (double)N * g.Kpad * 2.0 * (split == PREC_SPLIT ? 2 : 1);
    else if (bkind == BK_ACT) bbytes = nb * (double)g.b.T_in * g.b.C_in * 4.0;
    else bbytes = nb * (double)g.b.rows * g.b.T_in * 4.0;
    const double nout = g.geglu ? N / 2 : N;
    const double obytes = nb * (double)g.M * nout * 4.0 * (1 + (g.res ? 1 : 0) + (g.accumulate ? 1 : 0));
    g_cost.flops = 2.0 * nb * (double)g.M * N * Kr;
    g_cost.bytes = nb * a_rows * g.a.C_in * 4.0 + bbytes + obytes;
  }
  const bool window_conv = bkind == BK_W && avec && batch == 1 && g.a.ksize > 1 && g.a.Cpad % 32 == 0 &&
                           g.a.C_in == g.a.Cpad && (g.a.ksize - 1) * g.a.dil <= HALO_MAX &&
                           g.out_rows_per_batch == g.a.rows_per_batch && g.M % g.a.rows_per_batch == 0 &&
                           !g.disable_window;
  if (window_conv) {
    const int nb = g.M / g.a.rows_per_batch, T_out = g.a.rows_per_batch;
    // 64-wide N tiles when 128-wide tiles would waste a third of the MFMA work (N = 192, 320, ...)
    const bool narrow = g.tile_n == 64 || (g.tile_n == 0 && (N <= 64 || (N % 128 != 0 && N % 64 == 0)));
    const bool pro = g.a.pro_scale || g.a.pro_mean || g.a.pro_act;
    if (narrow) {
      if (pro) launch_conv_sp<128, 64, 4, 1, true>(P, nb, T_out, split, s);
      else launch_conv_sp<128, 64, 4, 1, false>(P, nb, T_out, split, s);
    } else {
      if (pro) launch_conv_sp<128, 128, 2, 2, true>(P, nb, T_out, split, s);
      else launch_conv_sp<128, 128, 2, 2, false>(P, nb, T_out, split, s);
    }
  } else if (bkind == BK_W && batch == 1 && g.M <= SK_MAXM && g.a.ksize == 1 && P.a.pad == 0 && P.a.up != 2 &&
             !P.a.pm && !P.a.ps && !P.a.pact && !g.geglu && g.Kpad <= SK_KMAX && g.Kpad % 8 == 0 &&
             g.a.sc == 1 && g.a.C_in % 4 == 0 && g.a.st % 4 == 0 && g.a.sb % 4 == 0 && (((uintptr_t)g.a.ptr) & 15) == 0 &&
             knobs().gemm_skinny) {
    // the embedder MLPs' M = B rows (gemm_skinny_kernel)
    const dim3 grid((unsigned)((N + SK_N - 1) / SK_N), (unsigned)((g.M + SK_M - 1) / SK_M));
    void* tok = prof_start(s);
    if (split == PREC_SPLIT) hipLaunchKernelGGL((gemm_skinny_kernel<PREC_SPLIT>), grid, dim3(256), 0, s, P);
    else if (split == PREC_F16) hipLaunchKernelGGL((gemm_skinny_kernel<PREC_F16>), grid, dim3(256), 0, s, P);
    else hipLaunchKernelGGL((gemm_skinny_kernel<PREC_BF16>), grid, dim3(256), 0, s, P);
    if (tok) {
      char name[96];
      std::snprintf(name, sizeof(name), "alcm::gemm_skinny_kernel<%d>", split);
      if (knobs().prof_shapes)
        std::snprintf(name + std::strlen(name), sizeof(name) - std::strlen(name), " M%d N%d K%d", g.M, N, g.Kpad);
      prof_stop(tok, s, name, g_cost.flops, g_cost.bytes);
    }
  } else if (bkind == BK_W) {
    // (N <= 32 on fewer than 128 tiles of 256 rows: 64-row tiles, 4x the workgroups — the DiT final layer, M = B T rows
    // x N = 20: 39 -> 156 workgroups; the same K order per output, bit-identical)
    if (N <= 32 && (int64_t)((g.M + 255) / 256) * batch < 128 && knobs().gemm_skinny) {
      if (avec) launch_split<64, 32, 4, 1, true, BK_W>(P, batch, N, split, s);
      else launch_split<64, 32, 4, 1, false, BK_W>(P, batch, N, split, s);
    } else if (N <= 32) {
      if (avec) launch_split<256, 32, 4, 1, true, BK_W>(P, batch, N, split, s);
      else launch_split<256, 32, 4, 1, false, BK_W>(P, batch, N, split, s);
    } else if (N <= 64) {
      if (avec) launch_split<256, 64, 4, 1, true, BK_W>(P, batch, N, split, s);
      else launch_split<256, 64, 4, 1, false, BK_W>(P, batch, N, split, s);
    } else {
      if (avec) launch_split<128, 128, 2, 2, true, BK_W>(P, batch, N, split, s);
      else launch_split<128, 128, 2, 2, false, BK_W>(P, batch, N, split, s);
    }
  } else {
    if (!avec) return set_error(ALCM_E_INVALID, "attention GEMM A operand must be vectorisable");
    if (bkind == BK_ACT) {
      if (N <= 64) launch_split<256, 64, 4, 1, true, BK_ACT>(P, batch, N, split, s);
      else launch_split<128, 128, 2, 2, true, BK_ACT>(P, batch, N, split, s);
    } else {
      if (N <= 64) launch_split<256, 64, 4, 1, true, BK_ACTT>(P, batch, N, split, s);
      else launch_split<128, 128, 2, 2, true, BK_ACTT>(P, batch, N, split, s);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(ALCM_E_HIP, std::string("gemm launch: ") + hipGetErrorString(e));
  return 0;
}

// ---------------------------------------------------------------- weight packing (device)
// W[co][ci][k] fp32 -> planes bf16 hi, bf16 lo, fp16 hi, fp16 lo [co][Kpad], K index = tap*cpad + ci.  For ConvTranspose1d
// (weight [ci][co][k], stride s, phase r) tap j = r + s*(Q-1-tap).
__global__ void pack_weight_kernel(const float* w, int c_out, int c_in, int ksz, int cpad, int kpad, int transposed,
                                   int stride, int phase, u16* out) {
  const int64_t total = (int64_t)c_out * kpad;
  const int Q = transposed ? ksz / stride : ksz;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(idx / kpad);
    const int k = (int)(idx % kpad);
    const int tap = k / cpad, ci = k % cpad;
    float v = 0.f;
    if (tap < Q && ci < c_in) {
      if (transposed) {
        const int j = phase + stride * (Q - 1 - tap);
        v = w[((int64_t)ci * c_out + co) * ksz + j];
      } else {
        v = w[((int64_t)co * c_in + ci) * ksz + tap];
      }
    }
    const __bf16 h = (__bf16)v;
    const __bf16 l = (__bf16)(v - (float)h);
    out[idx] = __builtin_bit_cast(u16, h);
    out[idx + total] = __builtin_bit_cast(u16, l);
    const _Float16 fh = (_Float16)v;
    out[idx + 2 * total] = __builtin_bit_cast(u16, fh);
    out[idx + 3 * total] = __builtin_bit_cast(u16, (_Float16)(v - (float)fh));
  }
}

int pack_conv_weight(const float* w, int c_out, int c_in, int k, int cpad, int kpad, int transposed, int stride,
                     int phase, void* out, hipStream_t s) {
  if (!w || !out || c_out <= 0 || c_in <= 0 || k <= 0 || cpad < c_in || cpad % 8 || kpad % BK)
    return set_error(ALCM_E_INVALID, "pack_conv_weight: bad geometry");
  const int Q = transposed ? k / stride : k;
  if (transposed && (stride <= 0 || k % stride || phase < 0 || phase >= stride))
    return set_error(ALCM_E_INVALID, "pack_conv_weight: bad transposed stride/phase");
  if (Q * cpad > kpad) return set_error(ALCM_E_INVALID, "pack_conv_weight: kpad too small");
  const int64_t total = (int64_t)c_out * kpad;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(blocks), dim3(256), 0, s, w, c_out, c_in, k, cpad, kpad, transposed,
                     stride, phase, (u16*)out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(ALCM_E_HIP, std::string("pack launch: ") + hipGetErrorString(e));
  return 0;
}

}  // namespace alcm

extern "C" int alcm_gemm(const alcm_gemm_args* args, alcm_stream_t stream) {
  if (!args) return alcm::set_error(ALCM_E_INVALID, "null args");
  return alcm::gemm(*args, (hipStream_t)stream);
}

extern "C" int alcm_pack_conv_weight(const float* w, int c_out, int c_in, int k, int cpad, int kpad, int transposed,
                                     int stride, int phase, void* out, alcm_stream_t stream) {
  return alcm::pack_conv_weight(w, c_out, c_in, k, cpad, kpad, transposed, stride, phase, out, (hipStream_t)stream);
}
