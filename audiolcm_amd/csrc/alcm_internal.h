// Internal (non-ABI) declarations shared by the libaudiolcm_hip.so translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "audiolcm_hip.h"

namespace alcm {

int set_error(int code, const std::string& msg);

#define ALCM_HIP(expr)                                                                         \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return ::alcm::set_error(ALCM_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e));   \
  } while (0)

#define ALCM_TRY(expr)      \
  do {                      \
    int _r = (expr);        \
    if (_r) return _r;      \
  } while (0)

int gemm(const alcm_gemm_args& g, hipStream_t s);
int pack_conv_weight(const float* w, int c_out, int c_in, int k, int cpad, int kpad, int transposed, int stride,
                     int phase, void* out, hipStream_t s);

int group_norm_affine(const float* x, int B, int T, int C, int64_t sb, int64_t st, int groups, float eps,
                      const float* gamma, const float* beta, float* scale, float* shift, hipStream_t s);
int row_stats(const float* x, int rows, int C, int64_t ld, float eps, float* mean, float* rstd, hipStream_t s);
int layer_norm(const float* x, int rows, int C, int64_t ld_in, float eps, const float* gamma, const float* beta,
               const float* add, int64_t ld_add, float* y, int64_t ld_out, hipStream_t s, int rpb = 0,
               int64_t out_bs = 0);
int softmax_rows(float* x, int rows, int n, int64_t ld, hipStream_t s);
int layer_norm_plane(const float* x, int rows, int C, int64_t ld, float eps, const float* gamma, const float* beta,
                     void* plane, int prec, hipStream_t s);
// plane[b][t'][c] = (silu?)(x[b][t'/up][c] * scale[b][c] + shift[b][c]) (scale == nullptr: identity)
int affine_plane(const float* x, int B, int T, int C, int up, const float* scale, const float* shift, int silu,
                 void* plane, int prec, hipStream_t s);
int activation1d(const float* x, float* y, int B, int T, int C, int64_t sb, int64_t st, const float* alpha_exp,
                 const float* inv_beta, const float* up_filter, const float* down_filter, hipStream_t s);
int lcm_step(const float* x, const float* eps, const float* eps_u, float cfg, const float* noise,
             const float* coeffs, float* prev, float* den, int64_t n, hipStream_t s);
int fill_f32(float* p, int64_t n, float v, hipStream_t s);
int nct_to_cl(const float* x, int B, int C, int T, int Cp, float* y, hipStream_t s);
// fp32 rows [rows][C] -> operand planes [rows][Cp] in the format of `prec` (SPLIT: lo plane rows * Cp after hi)
int to_planes(const float* x, void* y, int64_t rows, int C, int Cp, int prec, hipStream_t s);
// BigVGAN output head: Activation1d -> conv_post (k7, C -> 1, weights [tap][C] fp32) -> tanh, fp32 (alcm_act.hip)
struct Taps12O;
int act_conv_post(const float* x, float* wav, int B, int T, int C, const float* alpha_exp, const float* inv_beta,
                  const Taps12O& f, const float* w_tc, float bias, hipStream_t s);
int activation1d_x3(const float* x, void* const y[3], int B, int T, int C, int Cp, const float* const alpha_exp[3],
                    const float* const inv_beta[3], const float* up_filter, const float* down_filter, int prec,
                    hipStream_t s);
int activation1d_op(const float* x, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                    const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                    hipStream_t s);
// Activation1d with both FIRs on MFMA, fp16 planes out (alcm_act.hip; C >= 192, C % 64 == 0, PREC_F16, Cp == C)
bool act_mfma_ok(int C, int Cp, int prec);
// x16: x is an fp16 plane [B][T][C] (the wide-stage conv1 output, alcm_opconv's out_plane) instead of fp32
int act_mfma3(const float* x, void* const y[3], int B, int T, int C, int Cp, const float* const alpha_exp[3],
              const float* const inv_beta[3], const Taps12O& f, hipStream_t s);
int act_mfma(const void* x, bool x16, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
             const float* inv_beta, const Taps12O& f, hipStream_t s);
// Activation1d of an fp16 plane x16 [B][T][C] into fp16 planes (act_mfma shapes only; ALCM_E_INVALID otherwise)
int activation1d_op_h16(const void* x16, void* y, int B, int T, int C, int Cp, const float* alpha_exp,
                        const float* inv_beta, const float* up_filter, const float* down_filter, int prec,
                        hipStream_t s);
int nconv_try(const alcm_opconv_args& a, const unsigned short* wplane, const void* actepi, double flops, double bytes,
              hipStream_t s);
int opconv(const alcm_opconv_args& a, hipStream_t s);
// o_plane != nullptr: write the output as an fp16 / bf16 operand plane [B][L][H] instead of fp32 O
// bias != nullptr: + bias[(head * bld + query) * bld + key] on the scores (L <= 512); scale > 0 replaces 1/sqrt(dh);
// qkv_plane != nullptr (then qkv == nullptr): q / k / v rows as PREC operand elements (L <= 512)
int flash_attention(const float* qkv, float* O, int B, int L, int H, int nh, int prec, hipStream_t s,
                    void* o_plane = nullptr, const float* bias = nullptr, int bld = 0, float scale = 0.f,
                    const void* qkv_plane = nullptr);
// whether opconv can fuse Activation1d into its epilogue for N output channels at this precision
bool opconv_act_supported(int prec, int N, int Cp_in);
bool wconv3_sum_ok(const alcm_opconv_args* a, int n);
int wconv3_sum_try(const alcm_opconv_args* a, int n, hipStream_t s);
int opconv_sum(const alcm_opconv_args* a, int n, hipStream_t s);
int wconv_try(const alcm_opconv_args& a, const unsigned short* wplane, double flops, double bytes,
              hipStream_t s);

// narrow AMPBlock conv with resident dense weights (alcm_tconv.hip); actepi: const ActEpiDev* or nullptr
bool tconv_supported(int prec, int C, int N, int ksize, int dil);
struct ActEpiDev;
int tconv(const alcm_opconv_args& a, const unsigned short* wd, int64_t wd_lo, int kd, const ActEpiDev* act,
          double flops, double bytes, hipStream_t s);

struct Taps12O;

// BigVGAN stride-2 / kernel-4 upsampler, both phases in one split-precision pass (alcm_ups.hip)
bool ups2_supported(int cin, int cout, int cpad, int rate, int taps);
int ups2(const float* x, float* out, int B, int T, int cin, int cout, const unsigned short* w0, const unsigned short* w1,
         int64_t lo, int kpad, const int pad[2], const int off[2], const float* bias, hipStream_t s);
// bf16x3 1x1 conv on split operand planes (alcm_sgemm.hip)
bool sgemm_planes_ok(int K, int N, int kpad);
int sgemm_planes(const unsigned short* a, int64_t a_lo, int M, int K, const unsigned short* w, int64_t w_lo, int kpad,
                 int N, const float* bias, const float* res, int64_t ldr, float* out, int64_t ldo, float out_scale,
                 hipStream_t s);
// single-plane 1x1 conv / linear (alcm_sgemm.hip, ALCM_LIN1); 1 when it launched, 0 when not eligible
int lin_plane_try(const alcm_opconv_args& a, const unsigned short* wplane, double flops, double bytes, hipStream_t s);
int split_planes(const float* x, int64_t rows, int C, int T, const float* scale, const float* shift,
                 unsigned short* y, hipStream_t s);

// diagnostic / A-B switches, read from ALCM_* environment variables at library load (alcm_knobs.cpp)
struct Knobs {
  int wconv = 8;                 // ALCM_WCONV: > 0 = the wide-layer kernels (alcm_wconv.hip), 0 = opconv_kernel (A/B)
  int wconv3 = -1;               // ALCM_WCONV3: persistent 8-wave 256 x 192 wide conv (alcm_wconv.hip): -1 by shape, 0 off, 1 on
  int wconv3_grid = 0;           // ALCM_WCONV3_GRID: cap on wconv3's persistent workgroups (tests; 0 = one per CU)
  int nconv = -1;                // ALCM_NCONV: 0 = opconv_kernel for the narrow tail, 2 = nconv for every width
  int opconv_tile = 0;           // ALCM_OPCONV_TILE: narrow-layer tile variant
  bool serial_resblocks = false; // ALCM_SERIAL_RESBLOCKS: default of alcm_model_set_resblock_streams
  bool prof_shapes = false;      // ALCM_PROF_SHAPES: split profile rows per layer shape
  int tconv_ablate = 0;          // ALCM_TCONV_ABLATE: timing-only ablation bits of the tail convs (1 no epilogue,
                                 // 2 no MFMA, 4 no window DMA, 8 no plane stores, 16 no fp32 state stores); selects
                                 // their diagnostics instantiation
  bool tconv_trace = false;      // ALCM_TCONV_TRACE: per-phase shader-clock trace of the tail convs (alcm_debug_tconv_trace;
                                 // diagnostics instantiation)
  int lin1 = -1;                 // ALCM_LIN1: single-plane 1x1 convs on lin_plane_kernel (1: 32-deep 4-stage ring, 2: 64-deep
                                 // double-buffered, -1: 64-deep for plane outputs), 0 = wconv2
  int tconv = 1;                 // ALCM_TCONV: narrow conv for BigVGAN stages 3-5: 1 by shape, 2 streamed weights,
                                 // 3 resident weights (alcm_tconv.hip), 0 = opconv / nconv
  int act_defer = 1;             // ALCM_ACT_DEFER: act_mfma issues a tile's plane stores one tile late, before the next
                                 // prefetch (0 = at the end of the tile)
  int act_mfma = 1;              // ALCM_ACT_MFMA: Activation1d FIRs on MFMA for the wide stages (0 = VALU act_coop)
  int conv1_h16 = 1;             // ALCM_CONV1_H16: wide-stage AMPBlock conv1 writes an fp16 plane for its Activation1d
  int act_x3_mfma = 1;           // ALCM_ACT_X3_MFMA: the wide stages' three first Activation1d in one MFMA-FIR pass (0 = three)
  int nct_cl = 1;                // ALCM_NCT_CL: NCT conv inputs (DiT proj_in, BigVGAN conv_pre) transposed to channels-last
                                 // first (0 = strided gather in the conv)
  int ups_t160 = 1;              // ALCM_UPS_T160: strided (upsampler phase) wconv2 launches may take 160-row tiles
  int gemm_skinny = 1;           // ALCM_GEMM_SKINNY: M <= 64-row k = 1 GEMMs on gemm_skinny_kernel (0 = MFMA tiles)
  int wconv_sum = 1;             // ALCM_WCONV_SUM: the wide stages' three chains' last conv2 + residual in one sum-form
                                 // launch writing the next stage's upsampler planes (2 = fp32 output + to_planes,
                                 // 0 = three accumulating launches)
  int ksplit = 1;                // ALCM_KSPLIT: wconv3 K parts on under-filled grids where a workspace is given (0 = never)
  int xp[4] = {0, 0, 0, 0};      // ALCM_XP0..3: scratch switches for an experiment in flight (no default path reads them)
};
const Knobs& knobs();

bool prof_enabled();
void* prof_start(hipStream_t s);
void prof_stop(void* tok, hipStream_t s, const std::string& name, double flops, double bytes);

constexpr int kBK = 32;
inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace alcm
