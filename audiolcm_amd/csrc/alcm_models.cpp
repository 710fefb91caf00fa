// Model-level orchestration of the AudioLCM hot path on MI355X: weight ingestion from
// reference state_dict tensors, weight packing (weight-norm fold, bf16 hi/lo split, fused
// QKV / GEGLU-interleaved / conv-transpose-phase layouts), workspace planning, and the launch
// sequences of ConcatDiT2MLP, Decoder1D and BigVGAN.
//
// Activations live in HBM as fp32 channels-last (b, t, c) tensors; the reference's NCT layout
// is only used at the boundary (latents x/z/eps, mel, waveform) and is read/written through
// strided GEMM operands, so no transpose kernels run.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "alcm_common.h"
#include "alcm_internal.h"
#include "alcm_actepi.h"

namespace alcm {

thread_local std::string g_err;
int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int sincos_embedding(const float* v, float vscale, const float* freqs, int B, int half, int cos_first, float* out,
                     hipStream_t s);
// alcm_mel.hip
int reflect_pad_clamp(const float* x, int B, int L, int p, float* y, hipStream_t s);
int stft_magnitude(const float* spec, int F, int64_t rows, float* mag, hipStream_t s);
int log10_nct(const float* x, int B, int T, int C, float* out, hipStream_t s);
int rows_stride2(const float* in, int B, int T, int To, int C, float* out, hipStream_t s);
// alcm_text.hip
int embed_gather(const int64_t* ids, int rows, const float* table, int64_t vocab, int D, const float* add, int L,
                 float* out, hipStream_t s);
int rms_stats(const float* x, int rows, int C, float eps, float* mean, float* rstd, hipStream_t s);
int rms_norm(const float* x, int rows, int C, float eps, const float* w, int L, int64_t out_sb, float* out,
             hipStream_t s);
int rms_norm_plane(const float* x, int rows, int C, float eps, const float* w, void* out, int prec, hipStream_t s);
int geglu_pairs(const float* y, int64_t rows, int F, float* out, hipStream_t s);
int geglu_split_planes(const float* y, int64_t rows, int F, void* plane, int64_t lo_off, hipStream_t s);
int softmax_rows_bias(float* x, int rows, int n, int64_t ld, int L, int heads, const float* bias, int bld,
                      hipStream_t s);
int i64_to_f32(const int64_t* t, float* o, int n, hipStream_t s);

// ------------------------------------------------------------------ weights
struct Packed {
  u16* p = nullptr;
  int rows = 0, cin = 0, cpad = 0, taps = 0, kpad = 0;
  int64_t lo = 0;
};
struct ConvW {
  Packed w;
  Packed dw;  // BigVGAN narrow stages: dense K = tap * C + c packing for the resident-weight conv (alcm_tconv.hip)
  float* b = nullptr;
};
struct NormW {
  float* g = nullptr;
  float* b = nullptr;
};

struct DitBlock {
  NormW gn, ln1, ln2, ln3;
  ConvW proj_in, proj_out, qkv1, out1, qkv2, out2, ff0, ff2;
};
struct DitW {
  int in_ch = 20, ctx_dim = 1024, hidden = 576, heads = 8, depth = 4, max_len = 1000, ctx_tokens = 154;
  int ff_k = 9, pin_k = 5;
  ConvW proj_w, mlp0, mlp2, c0[2], c2[2], proj_in, fin;
  NormW cln[2], fin_gn;
  float* pos = nullptr;
  float* t_freqs = nullptr;
  std::vector<DitBlock> blocks;
};

struct ResW {
  NormW n1, n2;
  ConvW c1, c2, nin;
  bool has_nin = false;
  int cin = 0, cout = 0;
};
struct VaeEncW {  // Encoder1D + quant_conv (autoencoder1d.py:319-413, :31-33), present when encoder.* keys are
  bool present = false;
  int in_ch = 80;
  ConvW conv_in, conv_out, quant, attn_qkv, attn_out;
  std::vector<std::vector<ResW>> lv;  // lv[level]
  std::vector<ConvW> down;            // down[level] (w.p == nullptr if none)
  ResW mid1, mid2;
  NormW attn_n, norm_out;
};
struct VaeW {
  VaeEncW enc;
  int z_ch = 20, embed = 20, out_ch = 80, ksz = 5, ch = 384, nrb = 2;
  std::vector<int> mult;
  std::vector<int> up_levels;
  ConvW pqc, conv_in, attn_qkv, attn_out, conv_out;
  ResW mid1, mid2;
  NormW attn_n, norm_out;
  std::vector<std::vector<ResW>> lv;  // lv[level]
  std::vector<ConvW> up;              // up[level] (w.p == nullptr if none)
};

struct MelW {  // log-mel front-end (NAT_mel.py:42-85): STFT as a GEMM over frames + mel projection
  int n_fft = 1024, hop = 256, win = 1024, n_mels = 80, n_freq = 513;
  ConvW dft;     // [2 n_freq][n_fft]: window * cos / -window * sin, K = tap * hop + c over n_fft / hop taps
  ConvW basis;   // [n_mels][n_freq]
};

struct ActW {
  float* aexp = nullptr;
  float* ibeta = nullptr;
  float fup[12] = {0}, fdn[12] = {0};  // host copies: the kernel takes the taps as arguments
};
struct AmpW {
  int k = 3;
  std::vector<int> dil;
  std::vector<ConvW> c1, c2;
  std::vector<ActW> act;
};
struct StageW {
  int cin = 0, cout = 0, rate = 1, kernel = 1;
  std::vector<ConvW> phase;
  std::vector<int> pad, off;
  std::vector<AmpW> rb;
};
struct VocW {
  int num_mels = 80, c0 = 1536;
  ConvW pre, post;
  float* post_w32 = nullptr;  // conv_post weight [tap][C] fp32 (the fused output head, act_conv_post)
  float post_bias = 0.f;
  std::vector<StageW> st;
  ActW post_act;
};

// text conditioning (FrozenCLAPFLANEmbedder, ldm/modules/encoders/modules.py:529-582)
struct BertLayerW {  // transformers BertLayer (post-LN)
  ConvW qkv, ao, inter, out;
  NormW ln1, ln2;
};
struct T5BlockW {  // transformers T5Block of the encoder (pre-RMSNorm, no biases)
  float* ln0 = nullptr;
  float* ln1 = nullptr;
  ConvW qkv, o, wi, wo;
};
struct TextW {
  int b_vocab = 30522, b_hidden = 768, b_layers = 12, b_heads = 12, b_inter = 3072, b_maxpos = 512;
  int p_out = 1024;
  int t_vocab = 32128, t_d = 1024, t_dkv = 64, t_heads = 16, t_ff = 2816, t_layers = 24;
  int max_len = 77;
  float b_eps = 1e-12f, p_eps = 1e-5f, t_eps = 1e-6f;
  float* b_word = nullptr;      // (vocab, hidden)
  float* b_pos_type = nullptr;  // position_embeddings[t] + token_type_embeddings[0]  (maxpos, hidden)
  NormW b_emb_ln;
  std::vector<BertLayerW> bl;
  ConvW p1, p2;  // CLAP Projection linear1 / linear2 (no bias)
  NormW p_ln;
  float* t_emb = nullptr;   // shared (vocab, d)
  float* t_bias = nullptr;  // relative position bias (heads, max_len, max_len)
  std::vector<T5BlockW> tb;
  float* t_fin = nullptr;
  float* zeros = nullptr;  // max(d, hidden) zeros: the RMSNorm prologue's shift
};

}  // namespace alcm

struct alcm_model {
  int kind = -1;
  int policy = ALCM_POLICY_SPLIT;  // ALCM_POLICY_*
  std::vector<void*> allocs;
  size_t weight_bytes = 0;
  alcm::DitW dit;
  alcm::VaeW vae;
  alcm::VocW voc;
  alcm::TextW text;
  alcm::MelW mel;
  // BigVGAN: the three resblocks of a stage are independent chains until their mean; they run on the
  // caller's stream plus two auxiliary streams ordered by events, so the VALU / HBM bound Activation1d
  // kernels of one chain overlap the MFMA-bound convs of another.  The auxiliary streams and events belong
  // to the CALLER's stream (created on its first call, kept until destroy): concurrent calls on one handle
  // from different caller streams fork and join on disjoint resources, so they never order against (or
  // race on) each other's chains.
  struct AuxSet {
    hipStream_t s[2] = {nullptr, nullptr};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  };
  std::mutex aux_mu;
  std::map<hipStream_t, AuxSet> aux;
  bool resblock_streams = true;  // alcm_model_set_resblock_streams (default: !ALCM_SERIAL_RESBLOCKS)
};

namespace alcm {

// MFMA precision of one layer under the model's policy; f16_ok marks the layers the parity budget lets
// run as one fp16 MFMA (measured by scripts/precision_emulate.py).
static int prec_of(const alcm_model* m, bool f16_ok) {
  if (m->policy == ALCM_POLICY_BF16) return PREC_BF16;
  return (m->policy == ALCM_POLICY_MIXED && f16_ok) ? PREC_F16 : PREC_SPLIT;
}

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct Ingest {
  std::map<std::string, const alcm_named_tensor*> by;
  alcm_model* m;
  hipStream_t s = nullptr;

  Ingest(alcm_model* mm, const alcm_named_tensor* t, int n) : m(mm) {
    for (int i = 0; i < n; ++i)
      if (t[i].name) by[t[i].name] = &t[i];
  }
  bool has(const std::string& k) const { return by.count(k) != 0; }
  std::vector<float> get(const std::string& k, std::vector<int64_t> shape) {
    auto it = by.find(k);
    if (it == by.end()) throw Error(ALCM_E_MISSING, "missing weight tensor '" + k + "'");
    const alcm_named_tensor* t = it->second;
    int64_t n = 1;
    for (int i = 0; i < t->ndim; ++i) n *= t->shape[i];
    int64_t want = 1;
    for (auto v : shape) want *= v;
    bool same = (int)shape.size() == t->ndim;
    for (int i = 0; same && i < t->ndim; ++i) same = t->shape[i] == shape[i];
    if (!same || n != want) {
      std::string got;
      for (int i = 0; i < t->ndim; ++i) got += std::to_string(t->shape[i]) + (i + 1 < t->ndim ? "x" : "");
      std::string exp;
      for (size_t i = 0; i < shape.size(); ++i) exp += std::to_string(shape[i]) + (i + 1 < shape.size() ? "x" : "");
      throw Error(ALCM_E_INVALID, "weight '" + k + "' has shape " + got + ", expected " + exp);
    }
    if (!t->data) throw Error(ALCM_E_INVALID, "weight '" + k + "' has null data");
    return std::vector<float>(t->data, t->data + n);
  }
  void* dalloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) throw Error(ALCM_E_HIP, "hipMalloc failed");
    m->allocs.push_back(p);
    m->weight_bytes += bytes;
    return p;
  }
  float* upload(const std::vector<float>& v) {
    float* p = (float*)dalloc(v.size() * sizeof(float));
    if (hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      throw Error(ALCM_E_HIP, "hipMemcpy H2D failed");
    return p;
  }
  // pack W[co][ci][k] (or ConvTranspose [ci][co][k] phase) into bf16 hi / bf16 lo / fp16 [rows][kpad]
  Packed pack(const std::vector<float>& w, int cout, int cin, int k, int transposed = 0, int stride = 1,
              int phase = 0, int cpad_to = 8) {
    Packed P;
    P.rows = cout;
    P.cin = cin;
    P.cpad = round_up(cin, cpad_to);
    P.taps = transposed ? k / stride : k;
    P.kpad = round_up(P.taps * P.cpad, kBK);
    P.lo = (int64_t)cout * P.kpad;
    P.p = (u16*)dalloc((size_t)4 * cout * P.kpad * sizeof(u16));  // bf16 hi, bf16 lo, fp16 hi, fp16 lo planes
    void* tmp = nullptr;
    if (hipMalloc(&tmp, w.size() * sizeof(float)) != hipSuccess) throw Error(ALCM_E_HIP, "hipMalloc tmp failed");
    (void)hipMemcpy(tmp, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice);
    int r = pack_conv_weight((const float*)tmp, cout, cin, k, P.cpad, P.kpad, transposed, stride, phase, P.p, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(tmp);
    if (r) throw Error(r, g_err);
    return P;
  }
  ConvW conv(const std::string& p, int cout, int cin, int k, bool bias = true) {
    ConvW c;
    c.w = pack(get(p + "weight", {cout, cin, k}), cout, cin, k);
    if (bias) c.b = upload(get(p + "bias", {cout}));
    return c;
  }
  ConvW linear(const std::string& p, int cout, int cin, bool bias = true) {
    ConvW c;
    c.w = pack(get(p + "weight", {cout, cin}), cout, cin, 1);
    if (bias) c.b = upload(get(p + "bias", {cout}));
    return c;
  }
  NormW norm(const std::string& p, int c) {
    NormW n;
    n.g = upload(get(p + "weight", {c}));
    n.b = upload(get(p + "bias", {c}));
    return n;
  }
  // weight_norm(dim=0) fold: w = g * v / ||v||  (torch.nn.utils.weight_norm, used by every BigVGAN conv)
  std::vector<float> wn(const std::string& p, std::vector<int64_t> vshape) {
    std::vector<float> v = get(p + "weight_v", vshape);
    std::vector<float> g = get(p + "weight_g", {vshape[0], 1, 1});
    const int64_t d0 = vshape[0], inner = (int64_t)v.size() / d0;
    for (int64_t o = 0; o < d0; ++o) {
      double ss = 0.0;
      for (int64_t i = 0; i < inner; ++i) ss += (double)v[o * inner + i] * v[o * inner + i];
      const float scale = (float)((double)g[o] / std::sqrt(ss));
      for (int64_t i = 0; i < inner; ++i) v[o * inner + i] *= scale;
    }
    return v;
  }
};

// ------------------------------------------------------------------ builders
static void build_dit(Ingest& I, const int* ic, int nic) {
  DitW& D = I.m->dit;
  if (nic >= 9) {
    D.in_ch = ic[0]; D.ctx_dim = ic[1]; D.hidden = ic[2]; D.heads = ic[3]; D.depth = ic[4];
    D.max_len = ic[5]; D.ctx_tokens = ic[6]; D.ff_k = ic[7]; D.pin_k = ic[8];
  }
  const int H = D.hidden, C = D.ctx_dim;
  if (H % D.heads || (H / D.heads) % 8 || D.ctx_tokens % 2 || H % 32)
    throw Error(ALCM_E_INVALID, "unsupported DiT geometry");
  D.proj_w = I.linear("t_embedder.proj_w.", 256, 256, false);
  D.mlp0 = I.linear("t_embedder.mlp.0.", H, 256);
  D.mlp2 = I.linear("t_embedder.mlp.2.", H, H);
  for (int e = 0; e < 2; ++e) {
    const std::string p = std::string(e ? "c2_embedder" : "c1_embedder") + ".mlp.";
    D.c0[e] = I.linear(p + "0.", H, C);
    D.c2[e] = I.linear(p + "2.", H, H);
    D.cln[e] = I.norm(p + "3.", H);
  }
  D.proj_in = I.conv("proj_in.", H, D.in_ch, D.pin_k);
  D.pos = I.upload(I.get("pos_emb.weight", {D.max_len, H}));
  if (I.has("_alcm.t_freqs")) {
    D.t_freqs = I.upload(I.get("_alcm.t_freqs", {128}));
  } else {
    std::vector<float> f(128);
    for (int i = 0; i < 128; ++i) f[i] = expf(-logf(10000.f) * (float)i / 128.f);
    D.t_freqs = I.upload(f);
  }
  const int inner = 4 * H;
  for (int i = 0; i < D.depth; ++i) {
    DitBlock b;
    const std::string p = "blocks." + std::to_string(i) + ".";
    const std::string tb = p + "transformer_blocks.0.";
    b.gn = I.norm(p + "norm.", H);
    b.proj_in = I.conv(p + "proj_in.", H, H, 1);
    b.proj_out = I.conv(p + "proj_out.", H, H, 1);
    b.ln1 = I.norm(tb + "norm1.", H);
    b.ln2 = I.norm(tb + "norm2.", H);
    b.ln3 = I.norm(tb + "norm3.", H);
    for (int a = 0; a < 2; ++a) {
      const std::string ap = tb + (a ? "attn2." : "attn1.");
      std::vector<float> q = I.get(ap + "to_q.weight", {H, H}), k = I.get(ap + "to_k.weight", {H, H}),
                         v = I.get(ap + "to_v.weight", {H, H});
      std::vector<float> qkv;
      qkv.reserve(3 * (size_t)H * H);
      qkv.insert(qkv.end(), q.begin(), q.end());
      qkv.insert(qkv.end(), k.begin(), k.end());
      qkv.insert(qkv.end(), v.begin(), v.end());
      ConvW cq;
      cq.w = I.pack(qkv, 3 * H, H, 1);
      (a ? b.qkv2 : b.qkv1) = cq;
      (a ? b.out2 : b.out1) = I.linear(ap + "to_out.0.", H, H);
    }
    // GEGLU: interleave value/gate rows so the epilogue pairs lanes n, n^1 (new_attention.py:48-55)
    {
      const int K = D.ff_k;
      std::vector<float> w = I.get(tb + "ff.net.0.proj.weight", {2 * inner, H, K});
      std::vector<float> bb = I.get(tb + "ff.net.0.proj.bias", {2 * inner});
      std::vector<float> wi(w.size()), bi(bb.size());
      const size_t row = (size_t)H * K;
      for (int j = 0; j < inner; ++j) {
        std::memcpy(&wi[(2 * j) * row], &w[j * row], row * sizeof(float));
        std::memcpy(&wi[(2 * j + 1) * row], &w[(inner + j) * row], row * sizeof(float));
        bi[2 * j] = bb[j];
        bi[2 * j + 1] = bb[inner + j];
      }
      b.ff0.w = I.pack(wi, 2 * inner, H, K);
      b.ff0.b = I.upload(bi);
      b.ff2 = I.conv(tb + "ff.net.2.", H, inner, K);
    }
    D.blocks.push_back(b);
  }
  D.fin_gn = I.norm("final_layer.norm_final.", H);
  D.fin = I.conv("final_layer.conv1d.", D.in_ch, H, 1);
}

static ResW build_res(Ingest& I, const std::string& p, int cin, int cout, int k = 3) {
  ResW r;
  r.cin = cin;
  r.cout = cout;
  r.n1 = I.norm(p + "norm1.", cin);
  r.c1 = I.conv(p + "conv1.", cout, cin, k);
  r.n2 = I.norm(p + "norm2.", cout);
  r.c2 = I.conv(p + "conv2.", cout, cout, k);
  r.has_nin = cin != cout;
  if (r.has_nin) r.nin = I.conv(p + "nin_shortcut.", cout, cin, 1);
  return r;
}

static void build_vae(Ingest& I, const int* ic, int nic) {
  VaeW& V = I.m->vae;
  V.mult = {1, 2, 4};
  V.up_levels = {1};
  if (nic >= 7) {
    V.z_ch = ic[0]; V.embed = ic[1]; V.out_ch = ic[2]; V.ksz = ic[3]; V.ch = ic[4]; V.nrb = ic[5];
    const int nl = ic[6];
    if (nic < 8 + nl) throw Error(ALCM_E_INVALID, "vae iconfig too short");
    V.mult.assign(ic + 7, ic + 7 + nl);
    const int nu = ic[7 + nl];
    if (nic < 8 + nl + nu) throw Error(ALCM_E_INVALID, "vae iconfig too short");
    V.up_levels.assign(ic + 8 + nl, ic + 8 + nl + nu);
  }
  const int nl = (int)V.mult.size();
  int block_in = V.ch * V.mult[nl - 1];
  V.pqc = I.conv("post_quant_conv.", V.z_ch, V.embed, 1);
  const std::string d = "decoder.";
  V.conv_in = I.conv(d + "conv_in.", block_in, V.z_ch, V.ksz);
  V.mid1 = build_res(I, d + "mid.block_1.", block_in, block_in);
  {
    const std::string a = d + "mid.attn_1.";
    V.attn_n = I.norm(a + "norm.", block_in);
    const int C = block_in;
    std::vector<float> w, b;
    for (const char* q : {"q", "k", "v"}) {
      auto wq = I.get(a + q + ".weight", {C, C, 1});
      auto bq = I.get(a + q + ".bias", {C});
      w.insert(w.end(), wq.begin(), wq.end());
      b.insert(b.end(), bq.begin(), bq.end());
    }
    V.attn_qkv.w = I.pack(w, 3 * C, C, 1);
    V.attn_qkv.b = I.upload(b);
    V.attn_out = I.conv(a + "proj_out.", C, C, 1);
  }
  V.mid2 = build_res(I, d + "mid.block_2.", block_in, block_in);
  V.lv.assign(nl, {});
  V.up.assign(nl, ConvW{});
  for (int lvl = nl - 1; lvl >= 0; --lvl) {
    const int block_out = V.ch * V.mult[lvl];
    for (int ib = 0; ib <= V.nrb; ++ib) {
      V.lv[lvl].push_back(build_res(I, d + "up." + std::to_string(lvl) + ".block." + std::to_string(ib) + ".",
                                    block_in, block_out));
      block_in = block_out;
    }
    for (int u : V.up_levels)
      if (u == lvl) V.up[lvl] = I.conv(d + "up." + std::to_string(lvl) + ".upsample.conv.", block_in, block_in, 3);
  }
  V.norm_out = I.norm(d + "norm_out.", block_in);
  V.conv_out = I.conv(d + "conv_out.", V.out_ch, block_in, V.ksz);
  // Encoder1D (the audio-to-latent direction): built when the checkpoint carries it
  if (I.has("encoder.conv_in.weight")) {
    VaeEncW& E = V.enc;
    E.present = true;
    const std::string e = "encoder.";
    E.in_ch = (int)I.by.at(e + "conv_in.weight")->shape[1];
    E.conv_in = I.conv(e + "conv_in.", V.ch, E.in_ch, V.ksz);
    int bi = V.ch;
    E.lv.assign(nl, {});
    E.down.assign(nl, ConvW{});
    for (int lvl = 0; lvl < nl; ++lvl) {
      const int bo = V.ch * V.mult[lvl];
      for (int ib = 0; ib < V.nrb; ++ib) {
        E.lv[lvl].push_back(build_res(I, e + "down." + std::to_string(lvl) + ".block." + std::to_string(ib) + ".", bi,
                                      bo, V.ksz));
        bi = bo;
      }
      for (int u : V.up_levels)  // down_layers = up_levels - 1
        if (u - 1 == lvl) E.down[lvl] = I.conv(e + "down." + std::to_string(lvl) + ".downsample.conv.", bi, bi, 3);
    }
    E.mid1 = build_res(I, e + "mid.block_1.", bi, bi, V.ksz);
    {
      const std::string a = e + "mid.attn_1.";
      E.attn_n = I.norm(a + "norm.", bi);
      std::vector<float> w, b;
      for (const char* q : {"q", "k", "v"}) {
        auto wq = I.get(a + q + ".weight", {bi, bi, 1});
        auto bq = I.get(a + q + ".bias", {bi});
        w.insert(w.end(), wq.begin(), wq.end());
        b.insert(b.end(), bq.begin(), bq.end());
      }
      E.attn_qkv.w = I.pack(w, 3 * bi, bi, 1);
      E.attn_qkv.b = I.upload(b);
      E.attn_out = I.conv(a + "proj_out.", bi, bi, 1);
    }
    E.mid2 = build_res(I, e + "mid.block_2.", bi, bi, V.ksz);
    E.norm_out = I.norm(e + "norm_out.", bi);
    E.conv_out = I.conv(e + "conv_out.", 2 * V.z_ch, bi, V.ksz);
    E.quant = I.conv("quant_conv.", 2 * V.embed, 2 * V.z_ch, 1);
  }
}

static void build_mel(Ingest& I, const int* ic, int nic) {
  MelW& Mw = I.m->mel;
  if (nic >= 4) {
    Mw.n_fft = ic[0]; Mw.hop = ic[1]; Mw.win = ic[2]; Mw.n_mels = ic[3];
  }
  Mw.n_freq = Mw.n_fft / 2 + 1;
  if (Mw.n_fft % Mw.hop || (Mw.n_fft - Mw.hop) % 2 || Mw.win > Mw.n_fft || Mw.hop % 8)
    throw Error(ALCM_E_INVALID, "mel: n_fft must be a multiple of hop, (n_fft - hop) even, win <= n_fft");
  auto window = I.get("window", {Mw.win});
  std::vector<float> wfull(Mw.n_fft, 0.f);  // torch.stft centres a shorter window inside n_fft
  const int off = (Mw.n_fft - Mw.win) / 2;
  for (int i = 0; i < Mw.win; ++i) wfull[off + i] = window[i];
  // conv weight [co][ci][tap]: co = bin (re | im), ci = sample within a hop-row, tap = hop-row within the frame
  const int taps = Mw.n_fft / Mw.hop, F = Mw.n_freq;
  std::vector<float> w((size_t)2 * F * Mw.hop * taps);
  for (int k = 0; k < F; ++k)
    for (int c = 0; c < Mw.hop; ++c)
      for (int t = 0; t < taps; ++t) {
        const int n = t * Mw.hop + c;
        const double ang = 2.0 * M_PI * (double)((int64_t)k * n % Mw.n_fft) / Mw.n_fft;
        w[((size_t)k * Mw.hop + c) * taps + t] = (float)(wfull[n] * std::cos(ang));
        w[((size_t)(F + k) * Mw.hop + c) * taps + t] = (float)(-wfull[n] * std::sin(ang));
      }
  Mw.dft.w = I.pack(w, 2 * F, Mw.hop, taps);
  Mw.basis.w = I.pack(I.get("mel_basis", {Mw.n_mels, F}), Mw.n_mels, F, 1);
}

static ActW build_act(Ingest& I, const std::string& p, int C) {
  ActW a;
  auto al = I.get(p + "act.alpha", {C});
  auto be = I.get(p + "act.beta", {C});
  // SnakeBeta with alpha_logscale (activations.py:111-119): a = exp(alpha), 1/(exp(beta) + 1e-9)
  for (int c = 0; c < C; ++c) {
    al[c] = expf(al[c]);
    be[c] = 1.0f / (expf(be[c]) + 0.000000001f);
  }
  a.aexp = I.upload(al);
  a.ibeta = I.upload(be);
  auto fu = I.get(p + "upsample.filter", {1, 1, 12});
  auto fd = I.get(p + "downsample.lowpass.filter", {1, 1, 12});
  for (int k = 0; k < 12; ++k) {
    a.fup[k] = fu[k];
    a.fdn[k] = fd[k];
  }
  return a;
}

static void build_voc(Ingest& I, const int* ic, int nic) {
  VocW& G = I.m->voc;
  std::vector<int> rates = {4, 4, 2, 2, 2, 2}, kernels = {8, 8, 4, 4, 4, 4}, rk = {3, 7, 11}, dil = {1, 3, 5};
  if (nic >= 3) {
    G.num_mels = ic[0];
    G.c0 = ic[1];
    int n = ic[2], p = 3;
    if (nic < p + 2 * n + 1) throw Error(ALCM_E_INVALID, "bigvgan iconfig too short");
    rates.assign(ic + p, ic + p + n);
    kernels.assign(ic + p + n, ic + p + 2 * n);
    p += 2 * n;
    int nr = ic[p++];
    rk.assign(ic + p, ic + p + nr);
    p += nr;
    int nd = ic[p++];
    dil.assign(ic + p, ic + p + nd);
  }
  // (input channels padded to 32: the channels-last mel copy then takes the window conv, one staged window per
  // 32-channel chunk shared by the 7 taps)
  G.pre.w = I.pack(I.wn("conv_pre.", {G.c0, G.num_mels, 7}), G.c0, G.num_mels, 7, 0, 1, 0, 32);
  G.pre.b = I.upload(I.get("conv_pre.bias", {G.c0}));
  const int nk = (int)rk.size();
  for (size_t i = 0; i < rates.size(); ++i) {
    StageW S;
    S.cin = G.c0 >> i;
    S.cout = G.c0 >> (i + 1);
    S.rate = rates[i];
    S.kernel = kernels[i];
    const int s = S.rate, k = S.kernel, pad = (k - s) / 2, Q = k / s;
    if (k % s) throw Error(ALCM_E_INVALID, "upsample kernel must be a multiple of the rate");
    const std::string p = "ups." + std::to_string(i) + ".0.";
    std::vector<float> w = I.wn(p, {S.cin, S.cout, k});
    float* bias = I.upload(I.get(p + "bias", {S.cout}));
    for (int r = 0; r < s; ++r) {
      // output t = s*v + o, o = (r - pad) mod s; input u = v + c - q, c = (o + pad - r)/s
      const int o = ((r - pad) % s + s) % s;
      const int c = (o + pad - r) / s;
      ConvW cw;
      cw.w = I.pack(w, S.cout, S.cin, k, 1, s, r);
      cw.b = bias;
      S.phase.push_back(cw);
      S.pad.push_back(Q - 1 - c);
      S.off.push_back(o);
    }
    for (int j = 0; j < nk; ++j) {
      AmpW A;
      A.k = rk[j];
      A.dil = dil;
      const std::string rp = "resblocks." + std::to_string(i * nk + j) + ".";
      for (size_t l = 0; l < dil.size(); ++l) {
        for (int which = 0; which < 2; ++which) {
          const std::string cp = rp + (which ? "convs2." : "convs1.") + std::to_string(l) + ".";
          ConvW cw;
          // K = tap*Cp + ci with Cp = round_up(C, 32): the layout of the operand planes alcm_opconv reads
          const std::vector<float> wv = I.wn(cp, {S.cout, S.cout, A.k});
          cw.w = I.pack(wv, S.cout, S.cout, A.k, 0, 1, 0, 32);
          if (S.cout <= 96 && S.cout % 8 == 0) cw.dw = I.pack(wv, S.cout, S.cout, A.k, 0, 1, 0, 8);
          cw.b = I.upload(I.get(cp + "bias", {S.cout}));
          (which ? A.c2 : A.c1).push_back(cw);
        }
      }
      for (size_t a = 0; a < 2 * dil.size(); ++a)
        A.act.push_back(build_act(I, rp + "activations." + std::to_string(a) + ".", S.cout));
      S.rb.push_back(A);
    }
    G.st.push_back(S);
  }
  const int ch = G.st.back().cout;
  G.post_act = build_act(I, "activation_post.", ch);
  const std::vector<float> pw = I.wn("conv_post.", {1, ch, 7});
  G.post.w = I.pack(pw, 1, ch, 7, 0, 1, 0, 32);
  const std::vector<float> pb = I.get("conv_post.bias", {1});
  G.post.b = I.upload(pb);
  std::vector<float> ptc((size_t)7 * ch);
  for (int c = 0; c < ch; ++c)
    for (int k = 0; k < 7; ++k) ptc[(size_t)k * ch + c] = pw[(size_t)c * 7 + k];
  G.post_w32 = I.upload(ptc);
  G.post_bias = pb[0];
}

// ------------------------------------------------------------------ launch helpers
struct View {  // fp32 activation view, element (b, t, c) at p + b*sb + t*st + c*sc
  const float* p;
  int64_t sb, st, sc;
  int T, C;
};
struct Out {
  float* p;
  int64_t sb, st, sc;
  int step, off;
};
struct Res {
  const float* p = nullptr;
  int64_t sb = 0, st = 0, sc = 1;
};
struct Pro {
  const float* scale = nullptr;
  const float* shift = nullptr;
  int64_t sb = 0;
  const float* mean = nullptr;
  const float* rstd = nullptr;
  int act = 0;
};
inline View cl(const float* p, int T, int C, int64_t ld = -1) {  // channels-last (B, T, C) contiguous rows
  const int64_t l = ld < 0 ? C : ld;
  return View{p, (int64_t)T * l, l, 1, T, C};
}
inline Out ocl(float* p, int T, int C) { return Out{p, (int64_t)T * C, C, 1, 1, 0}; }

struct ConvOpts {
  int dil = 1, pad = 0, up = 1;
  Pro pro;
  Res res;
  int act = 0, accumulate = 0, geglu = 0;
  float out_scale = 1.f, acc_scale = 1.f;
};

static int conv(hipStream_t s, int split, int B, int rows_per_batch, const View& x, const ConvW& w, const Out& o,
                const ConvOpts& op) {
  alcm_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.M = B * rows_per_batch;
  g.N = w.w.rows;
  g.Kpad = w.w.kpad;
  g.batch = 1;
  g.zdiv = 1;
  alcm_operand& a = g.a;
  a.kind = ALCM_OPND_ACT;
  a.ptr = x.p;
  a.sb = x.sb; a.st = x.st; a.sc = x.sc;
  a.T_in = x.T; a.C_in = x.C; a.Cpad = w.w.cpad; a.ksize = w.w.taps; a.dil = op.dil; a.pad = op.pad; a.up = op.up;
  a.rows_per_batch = rows_per_batch;
  a.pro_scale = op.pro.scale; a.pro_shift = op.pro.shift; a.pro_sb = op.pro.sb;
  a.pro_mean = op.pro.mean; a.pro_rstd = op.pro.rstd; a.pro_act = op.pro.act;
  // (x.C == cpad > cin: a channels-last copy whose padding channels the caller zeroed, read as whole vectors)
  if (x.C != w.w.cin && !(x.C == w.w.cpad && x.sc == 1))
    return set_error(ALCM_E_INVALID, "conv: input channels do not match weight");
  alcm_operand& b = g.b;
  b.kind = ALCM_OPND_WEIGHT;
  b.ptr = w.w.p;
  b.rows = w.w.rows;
  b.w_lo_off = w.w.lo;
  g.bias = w.b;
  g.acc_scale = op.acc_scale;
  g.out_scale = op.out_scale;
  g.act = op.act;
  g.accumulate = op.accumulate;
  g.geglu = op.geglu;
  g.res = op.res.p; g.r_sb = op.res.sb; g.r_st = op.res.st; g.r_sc = op.res.sc;
  g.out = o.p; g.o_sb = o.sb; g.o_st = o.st; g.o_sc = o.sc;
  g.out_rows_per_batch = rows_per_batch;
  g.out_step = o.step;
  g.out_off = o.off;
  g.prec = split;
  return gemm(g, s);
}

static int lin(hipStream_t s, int prec, int R, const float* x, int C, const ConvW& w, float* y, const ConvOpts& o);

struct Bump {
  char* base;
  size_t cap, off = 0;
  Bump(void* b, size_t c) : base((char*)b), cap(c) {}
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? (T*)(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

// ------------------------------------------------------------------ DiT
struct DitWs {
  float *h, *u, *o, *qkv, *S, *g, *mean, *rstd, *gsc, *gsh, *tv, *tf, *t1;
  float* kp;  // K-split partial sums of the FFN down-projection (4 parts)
  int64_t kp_floats;
};
static DitWs plan_dit(const DitW& D, Bump& bp, int B, int T) {
  const int H = D.hidden, L = 1 + D.ctx_tokens + T, Lp = round_up(L, 8);
  DitWs w;
  w.h = bp.take<float>((size_t)B * L * H);
  w.u = bp.take<float>((size_t)B * L * H);
  w.o = bp.take<float>((size_t)B * L * H);
  w.qkv = bp.take<float>((size_t)B * L * 3 * H);
  w.S = bp.take<float>((size_t)B * D.heads * L * Lp);
  w.g = bp.take<float>((size_t)B * L * 4 * H);
  w.mean = bp.take<float>((size_t)B * L);
  w.rstd = bp.take<float>((size_t)B * L);
  w.gsc = bp.take<float>((size_t)B * H);
  w.gsh = bp.take<float>((size_t)B * H);
  w.tv = bp.take<float>((size_t)B);
  w.tf = bp.take<float>((size_t)B * 256);
  w.t1 = bp.take<float>((size_t)B * H);
  w.kp_floats = (int64_t)4 * B * L * H;
  w.kp = bp.take<float>((size_t)w.kp_floats);
  return w;
}

// attention core over a fused qkv buffer (B, L, 3H): O[b, t, h*dh + d] (new_attention.py:107-126)
static int dit_attention(hipStream_t s, int split, const DitW& D, int B, int L, const float* qkv, float* S, float* O) {
  const int H = D.hidden, nh = D.heads, dh = H / nh, Lp = round_up(L, 8);
  // single-rounding policies: fused kernel, scores never leave the chip (alcm_attn.hip)
  if ((split == PREC_F16 || split == PREC_BF16) && dh <= 72 && dh % 4 == 0)
    return flash_attention(qkv, O, B, L, H, nh, split, s);
  alcm_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  // S = (Q K^T) * dh^-1/2, batched over z = b*nh + head
  g.M = L; g.N = L; g.Kpad = round_up(dh, kBK); g.batch = B * nh; g.zdiv = nh;
  g.a.kind = ALCM_OPND_ACT; g.a.ptr = qkv; g.a.sb = 0; g.a.st = 3 * H; g.a.sc = 1;
  g.a.T_in = L; g.a.C_in = dh; g.a.Cpad = dh; g.a.ksize = 1; g.a.dil = 1; g.a.up = 1; g.a.rows_per_batch = L;
  g.a.zs1 = (int64_t)L * 3 * H; g.a.zs2 = dh;
  g.b = g.a;
  g.b.ptr = qkv + H;
  g.acc_scale = 1.0f / sqrtf((float)dh);
  g.out_scale = 1.f;
  g.out = S; g.o_sb = 0; g.o_st = Lp; g.o_sc = 1; g.o_zs1 = (int64_t)nh * L * Lp; g.o_zs2 = (int64_t)L * Lp;
  g.out_rows_per_batch = L; g.out_step = 1;
  g.prec = split;
  ALCM_TRY(gemm(g, s));
  ALCM_TRY(softmax_rows(S, B * nh * L, L, Lp, s));
  // O = P V
  alcm_gemm_args p;
  std::memset(&p, 0, sizeof(p));
  p.M = L; p.N = dh; p.Kpad = round_up(Lp, kBK); p.batch = B * nh; p.zdiv = nh;
  p.a.kind = ALCM_OPND_ACT; p.a.ptr = S; p.a.sb = 0; p.a.st = Lp; p.a.sc = 1; p.a.T_in = L; p.a.C_in = Lp;
  p.a.Cpad = Lp; p.a.ksize = 1; p.a.dil = 1; p.a.up = 1; p.a.rows_per_batch = L;
  p.a.zs1 = (int64_t)nh * L * Lp; p.a.zs2 = (int64_t)L * Lp;
  p.b.kind = ALCM_OPND_ACT_T; p.b.ptr = qkv + 2 * H; p.b.st = 3 * H; p.b.sc = 1; p.b.T_in = L; p.b.rows = dh;
  p.b.zs1 = (int64_t)L * 3 * H; p.b.zs2 = dh;
  p.acc_scale = 1.f; p.out_scale = 1.f;
  p.out = O; p.o_sb = 0; p.o_st = H; p.o_sc = 1; p.o_zs1 = (int64_t)L * H; p.o_zs2 = dh;
  p.out_rows_per_batch = L; p.out_step = 1;
  p.prec = split;
  return gemm(p, s);
}

static int dit_embed_context(alcm_model* m, const float* ctx, int B, float* cemb, void* ws, size_t wsb,
                             hipStream_t s) {
  const DitW& D = m->dit;
  const int H = D.hidden, n = D.ctx_tokens / 2, CT = D.ctx_tokens;
  Bump bp(ws, wsb);
  float* t0 = bp.take<float>((size_t)B * n * H);
  float* t1 = bp.take<float>((size_t)B * n * H);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "dit_embed_context: workspace too small");
  for (int e = 0; e < 2; ++e) {
    // ConditionEmbedder: Linear -> GELU(tanh) -> Linear -> LayerNorm (concatDiT.py:91-102)
    View x{ctx + (int64_t)e * n * D.ctx_dim, (int64_t)CT * D.ctx_dim, D.ctx_dim, 1, n, D.ctx_dim};
    ConvOpts o1;
    o1.act = ACT_GELU_TANH;
    ALCM_TRY(conv(s, prec_of(m, false), B, n, x, D.c0[e], ocl(t0, n, H), o1));
    ALCM_TRY(conv(s, prec_of(m, false), B, n, cl(t0, n, H), D.c2[e], ocl(t1, n, H), ConvOpts{}));
    // LayerNorm, plus the learned position rows 1+e*n .. (PositionEmbedding MODE_ADD, new_attention.py:245-248),
    // one launch for all clips: row b * n + t -> token row b * CT + e * n + t
    ALCM_TRY(layer_norm(t1, B * n, H, H, 1e-5f, D.cln[e].g, D.cln[e].b, D.pos + (int64_t)(1 + e * n) * H, H,
                        cemb + (int64_t)e * n * H, H, s, n, CT));
  }
  return 0;
}

static int dit_forward(alcm_model* m, const float* x, const int64_t* t, const float* cemb, const float* w_emb,
                       float* eps, int B, int T, void* ws, size_t wsb, hipStream_t s) {
  const DitW& D = m->dit;
  const int split = prec_of(m, false);
  // fp16-tolerant DiT layers (scripts/precision_emulate.py dit: latent rel-L2 per group in fp16):
  // GEGLU FFN convs 9e-5 (89% of the DiT FLOPs), attention QK^T/PV 1.6e-5, to_q/k/v 3.1e-5,
  // to_out 3.6e-5; the TemporalTransformer 1x1 proj_in/out (2.5e-4) and the embedders / proj_in k5 /
  // final layer (3.0e-4) stay bf16x3
  const int pff = prec_of(m, true);
  const int H = D.hidden, E = 1 + D.ctx_tokens, L = E + T;
  if (B <= 0 || T <= 0) return set_error(ALCM_E_INVALID, "dit_forward: empty batch");
  if (L > D.max_len)
    return set_error(ALCM_E_INVALID, "dit_forward: latent length exceeds PositionEmbedding max_len (concatDiT.py:261)");
  Bump bp(ws, wsb);
  DitWs w = plan_dit(D, bp, B, T);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "dit_forward: workspace too small");

  // --- t-token: [cos|sin](t*f) + proj_w(w) -> Linear -> SiLU -> Linear (+pos[0]) -> h[:, 0]
  ALCM_TRY(i64_to_f32(t, w.tv, B, s));
  ALCM_TRY(sincos_embedding(w.tv, 1.0f, D.t_freqs, B, 128, 1, w.tf, s));
  if (w_emb) {
    ConvOpts o;
    o.res = Res{w.tf, 0, 256, 1};
    ALCM_TRY(conv(s, split, 1, B, View{w_emb, 0, 256, 1, B, 256}, D.proj_w, Out{w.tf, 0, 256, 1, 1, 0}, o));
  }
  {
    ConvOpts o;
    o.act = ACT_SILU;
    ALCM_TRY(conv(s, split, 1, B, View{w.tf, 0, 256, 1, B, 256}, D.mlp0, Out{w.t1, 0, H, 1, 1, 0}, o));
    ConvOpts o2;
    o2.res = Res{D.pos, 0, 0, 1};
    ALCM_TRY(conv(s, split, 1, B, View{w.t1, 0, H, 1, B, H}, D.mlp2, Out{w.h, 0, (int64_t)L * H, 1, 1, 0}, o2));
  }
  // --- condition tokens (cached, LayerNorm + pos already applied)
  ALCM_HIP(hipMemcpy2DAsync(w.h + H, (size_t)L * H * sizeof(float), cemb, (size_t)D.ctx_tokens * H * sizeof(float),
                            (size_t)D.ctx_tokens * H * sizeof(float), B, hipMemcpyDeviceToDevice, s));
  // --- latent tokens: proj_in conv k5 on NCT x, + pos[E + t]
  {
    ConvOpts o;
    o.pad = D.pin_k / 2;
    o.res = Res{D.pos, 0, H, 1};
    // the NCT latent as channels-last rows of cpad channels (zero padded) in w.o (free until the first block), so
    // the conv reads whole vectors instead of a stride-T gather per element (ALCM_NCT_CL=0: the gather)
    const int cp = D.proj_in.w.cpad;
    const bool tcl = knobs().nct_cl && cp % 4 == 0 && (size_t)B * T * cp <= (size_t)B * L * H;
    View xv{x, (int64_t)D.in_ch * T, 1, T, T, D.in_ch};
    if (tcl) {
      ALCM_TRY(nct_to_cl(x, B, D.in_ch, T, cp, w.o, s));
      xv = View{w.o, (int64_t)T * cp, cp, 1, T, cp};
    }
    ALCM_TRY(conv(s, split, B, T, xv, D.proj_in, Out{w.h, (int64_t)L * H, H, 1, 1, E}, o));
  }
  const View hv = cl(w.h, L, H), uv = cl(w.u, L, H), ov = cl(w.o, L, H);
  const Out ho = ocl(w.h, L, H), uo = ocl(w.u, L, H);
  const Res ur{w.u, (int64_t)L * H, H, 1}, hr{w.h, (int64_t)L * H, H, 1};
  for (const DitBlock& blk : D.blocks) {
    // TemporalTransformer (concatDiT.py:159-171): GN32 -> 1x1 -> block -> 1x1 -> +x
    ALCM_TRY(group_norm_affine(w.h, B, L, H, (int64_t)L * H, H, 32, 1e-6f, blk.gn.g, blk.gn.b, w.gsc, w.gsh, s));
    // bf16x3 1x1 convs on split planes (alcm_sgemm.hip): the GroupNorm affine applied once while the planes are
    // written; w.g is free outside the feed-forward
    const bool sg = split == PREC_SPLIT && sgemm_planes_ok(H, H, blk.proj_in.w.kpad) &&
                    sgemm_planes_ok(H, H, blk.proj_out.w.kpad) && blk.proj_in.w.cpad == H && blk.proj_out.w.cpad == H;
    u16* spl = reinterpret_cast<u16*>(w.g);
    if (sg) {
      ALCM_TRY(split_planes(w.h, (int64_t)B * L, H, L, w.gsc, w.gsh, spl, s));
      ALCM_TRY(sgemm_planes(spl, (int64_t)B * L * H, B * L, H, blk.proj_in.w.p, blk.proj_in.w.lo, blk.proj_in.w.kpad,
                            H, blk.proj_in.b, nullptr, 0, w.u, H, 1.f, s));
    } else {
      ConvOpts o;
      o.pro = Pro{w.gsc, w.gsh, H, nullptr, nullptr, 0};
      ALCM_TRY(conv(s, split, B, L, hv, blk.proj_in, uo, o));
    }
    // BasicTransformerBlock (concatDiT.py:120-125)
    const bool planes = (pff == PREC_F16 || pff == PREC_BF16) && (H / D.heads) <= 72 && (H / D.heads) % 4 == 0;
    for (int a = 0; a < 2 && planes; ++a) {
      // attention sub-block on operand planes: LayerNorm -> plane, fused q/k/v projection (k = 1 on the
      // wide-layer kernel), flash attention writing the to_out operand plane, to_out + bias + residual in place
      const NormW& ln = a ? blk.ln2 : blk.ln1;
      const ConvW& wq = a ? blk.qkv2 : blk.qkv1;
      const ConvW& wo = a ? blk.out2 : blk.out1;
      u16* pln = reinterpret_cast<u16*>(w.g);  // w.g is free until the feed-forward below
      u16* opl = pln + (size_t)B * L * H;
      ALCM_TRY(layer_norm_plane(w.u, B * L, H, H, 1e-5f, ln.g, ln.b, pln, pff, s));
      alcm_opconv_args g;
      std::memset(&g, 0, sizeof(g));
      g.a = pln; g.B = B; g.T = L; g.C = H; g.Cp = wq.w.cpad; g.ksize = 1; g.dil = 1; g.pad = 0;
      g.w = wq.w.p; g.w_lo_off = wq.w.lo; g.kpad = wq.w.kpad; g.N = wq.w.rows;
      g.bias = wq.b; g.out = w.qkv; g.out_scale = 1.f; g.prec = pff;
      // q / k / v as an operand plane (attention rounds them to pff anyway): half the bytes written and staged
      const bool qp = wq.w.rows % 4 == 0 && L <= 512;
      if (qp) {
        g.out = nullptr;
        g.out_plane = w.qkv;
      }
      ALCM_TRY(opconv(g, s));
      if (qp) ALCM_TRY(flash_attention(nullptr, nullptr, B, L, H, D.heads, pff, s, opl, nullptr, 0, 0.f, w.qkv));
      else ALCM_TRY(flash_attention(w.qkv, nullptr, B, L, H, D.heads, pff, s, opl));
      std::memset(&g, 0, sizeof(g));
      g.a = opl; g.B = B; g.T = L; g.C = H; g.Cp = wo.w.cpad; g.ksize = 1; g.dil = 1; g.pad = 0;
      g.w = wo.w.p; g.w_lo_off = wo.w.lo; g.kpad = wo.w.kpad; g.N = wo.w.rows;
      g.bias = wo.b; g.res = w.u; g.out = w.u; g.out_scale = 1.f; g.prec = pff;
      ALCM_TRY(opconv(g, s));
    }
    for (int a = 0; a < 2 && !planes; ++a) {
      const NormW& ln = a ? blk.ln2 : blk.ln1;
      ALCM_TRY(row_stats(w.u, B * L, H, H, 1e-5f, w.mean, w.rstd, s));
      ConvOpts oq;
      oq.pro = Pro{ln.g, ln.b, 0, w.mean, w.rstd, 0};
      ALCM_TRY(conv(s, pff, B, L, uv, a ? blk.qkv2 : blk.qkv1, ocl(w.qkv, L, 3 * H), oq));
      ALCM_TRY(dit_attention(s, pff, D, B, L, w.qkv, w.S, w.o));
      ConvOpts oo;
      oo.res = ur;
      ALCM_TRY(conv(s, pff, B, L, ov, a ? blk.out2 : blk.out1, uo, oo));
    }
    if (pff == PREC_F16 || pff == PREC_BF16) {
      // Conv1dFeedForward on operand planes and the wide-layer kernel (alcm_wconv.hip): LayerNorm -> plane,
      // conv k9 576 -> 2x2304 with the GEGLU epilogue writing the 2304-channel plane, conv k9 2304 -> 576
      // + bias + residual in place (non-overlapping tiles)
      const int inner = blk.ff0.w.rows / 2;
      u16* p2 = reinterpret_cast<u16*>(w.g);
      u16* p1 = p2 + (size_t)B * L * inner;
      ALCM_TRY(layer_norm_plane(w.u, B * L, H, H, 1e-5f, blk.ln3.g, blk.ln3.b, p1, pff, s));
      alcm_opconv_args g;
      std::memset(&g, 0, sizeof(g));
      g.a = p1; g.a_lo_off = 0; g.B = B; g.T = L; g.C = H; g.Cp = blk.ff0.w.cpad;
      g.ksize = D.ff_k; g.dil = 1; g.pad = D.ff_k / 2;
      g.w = blk.ff0.w.p; g.w_lo_off = blk.ff0.w.lo; g.kpad = blk.ff0.w.kpad; g.N = blk.ff0.w.rows;
      g.bias = blk.ff0.b; g.out_scale = 1.f; g.prec = pff; g.geglu_plane = p2;
      ALCM_TRY(opconv(g, s));
      std::memset(&g, 0, sizeof(g));
      g.a = p2; g.a_lo_off = 0; g.B = B; g.T = L; g.C = inner; g.Cp = blk.ff2.w.cpad;
      g.ksize = D.ff_k; g.dil = 1; g.pad = D.ff_k / 2;
      g.w = blk.ff2.w.p; g.w_lo_off = blk.ff2.w.lo; g.kpad = blk.ff2.w.kpad; g.N = blk.ff2.w.rows;
      g.bias = blk.ff2.b; g.res = w.u; g.out = w.u; g.out_scale = 1.f; g.prec = pff;
      // 192 tiles of 256 x 192 at B = 32: K parts fill the chip (alcm_wconv.hip wconv3_parts)
      g.ksplit_ws = w.kp; g.ksplit_ws_floats = w.kp_floats;
      ALCM_TRY(opconv(g, s));
    } else {
      ALCM_TRY(row_stats(w.u, B * L, H, H, 1e-5f, w.mean, w.rstd, s));
      ConvOpts o;
      o.pad = D.ff_k / 2;
      o.pro = Pro{blk.ln3.g, blk.ln3.b, 0, w.mean, w.rstd, 0};
      o.geglu = 1;
      ALCM_TRY(conv(s, pff, B, L, uv, blk.ff0, ocl(w.g, L, 4 * H), o));
      ConvOpts o2;
      o2.pad = D.ff_k / 2;
      o2.res = ur;
      ALCM_TRY(conv(s, pff, B, L, cl(w.g, L, 4 * H), blk.ff2, uo, o2));
    }
    if (sg) {
      ALCM_TRY(split_planes(w.u, (int64_t)B * L, H, 0, nullptr, nullptr, spl, s));
      ALCM_TRY(sgemm_planes(spl, (int64_t)B * L * H, B * L, H, blk.proj_out.w.p, blk.proj_out.w.lo,
                            blk.proj_out.w.kpad, H, blk.proj_out.b, w.h, H, w.h, H, 1.f, s));
    } else {
      ConvOpts o;
      o.res = hr;
      ALCM_TRY(conv(s, split, B, L, uv, blk.proj_out, ho, o));
    }
  }
  // final layer on the latent tokens: GN16(eps 1e-5) -> 1x1 -> eps (NCT)  (concatDiT.py:77-89, 302-303)
  const float* hl = w.h + (int64_t)E * H;
  ALCM_TRY(group_norm_affine(hl, B, T, H, (int64_t)L * H, H, 16, 1e-5f, D.fin_gn.g, D.fin_gn.b, w.gsc, w.gsh, s));
  ConvOpts o;
  o.pro = Pro{w.gsc, w.gsh, H, nullptr, nullptr, 0};
  ALCM_TRY(conv(s, split, B, T, View{hl, (int64_t)L * H, H, 1, T, H}, D.fin,
                Out{eps, (int64_t)D.in_ch * T, 1, T, 1, 0}, o));
  return 0;
}

// ------------------------------------------------------------------ VAE decoder
struct VaeWs {
  float *a, *b, *c, *d, *qkv, *S, *gsc, *gsh, *pqs, *pqh;
  u16* pl;  // operand plane of the k3 conv inputs (F16 / BF16 layers)
};
// the VAE's k3 convs read operand planes on the wide-layer kernel
static bool vae_planes(int pk3) {
  return pk3 == PREC_F16 || pk3 == PREC_BF16;
}
// conv k3 (same length) on an operand plane: out = conv(plane) + bias (+ res); out may alias res
static int plane_conv3(hipStream_t s, int prec, int B, int T, int C, const u16* plane, const ConvW& cw,
                       const float* res, float* out) {
  if (cw.w.cpad != C || cw.w.cin != C) return set_error(ALCM_E_INVALID, "plane_conv3: plane width != packed Cin");
  alcm_opconv_args g;
  std::memset(&g, 0, sizeof(g));
  g.a = plane; g.a_lo_off = 0; g.B = B; g.T = T; g.C = C; g.Cp = cw.w.cpad;
  g.ksize = cw.w.taps; g.dil = 1; g.pad = cw.w.taps / 2;
  g.w = cw.w.p; g.w_lo_off = cw.w.lo; g.kpad = cw.w.kpad; g.N = cw.w.rows;
  g.bias = cw.b; g.res = res; g.out = out; g.out_scale = 1.f; g.prec = prec;
  return opconv(g, s);
}
static VaeWs plan_vae(const VaeW& V, Bump& bp, int B, int T) {
  // largest channels x time of any activation on the decode path
  const int nl = (int)V.mult.size();
  int tcur = T, maxc = V.ch * V.mult[nl - 1];
  size_t big = (size_t)T * maxc;
  for (int lvl = nl - 1; lvl >= 0; --lvl) {
    const int c = V.ch * V.mult[lvl];
    maxc = std::max(maxc, c);
    big = std::max(big, (size_t)tcur * c);
    for (int u : V.up_levels)
      if (u == lvl) tcur *= 2;
    big = std::max(big, (size_t)tcur * c);
  }
  big = std::max(big, (size_t)tcur * V.out_ch);
  const int Cm = V.ch * V.mult.back(), Tp = round_up(T, 8);
  VaeWs w;
  w.a = bp.take<float>((size_t)B * big);
  w.b = bp.take<float>((size_t)B * big);
  w.c = bp.take<float>((size_t)B * big);
  w.d = bp.take<float>((size_t)B * big);
  w.qkv = bp.take<float>((size_t)B * T * 3 * Cm);
  w.S = bp.take<float>((size_t)B * T * Tp);
  w.gsc = bp.take<float>((size_t)B * maxc);
  w.gsh = bp.take<float>((size_t)B * maxc);
  w.pqs = bp.take<float>((size_t)V.z_ch);
  w.pqh = bp.take<float>((size_t)V.z_ch);
  w.pl = bp.take<u16>((size_t)B * big);
  return w;
}

// bf16x3 1x1 conv through split operand planes (alcm_sgemm.hip) when the layer qualifies: out[b,t,:] =
// W (x[b,t,:] (* scale[b] + shift[b])) + bias (+ res), rows of ld C in / ldo out; `scratch` holds B*T*C*4 bytes of
// planes.  Returns 1 when it ran, 0 when the caller should use conv(), or an error code (negative never)
static int split_1x1(hipStream_t s, int prec, int B, int T, const float* x, int C, const float* scale,
                     const float* shift, const ConvW& cw, const float* res, float* out, int ldo, u16* scratch,
                     int* rc) {
  *rc = 0;
  if (prec != PREC_SPLIT || !scratch || cw.w.taps != 1 || cw.w.cpad != C || cw.w.cin != C ||
      !sgemm_planes_ok(C, cw.w.rows, cw.w.kpad))
    return 0;
  const int64_t rows = (int64_t)B * T;
  if ((*rc = split_planes(x, rows, C, T, scale, shift, scratch, s))) return 1;
  *rc = sgemm_planes(scratch, rows * C, (int)rows, C, cw.w.p, cw.w.lo, cw.w.kpad, cw.w.rows, cw.b, res, ldo, out,
                     ldo, 1.f, s);
  return 1;
}

// ResnetBlock1D (autoencoder1d.py:212-235): out = x' + conv2(swish(GN(conv1(swish(GN(x))))))
static int vae_res(hipStream_t s, int split, int pk3, int B, int T, const ResW& r, const float* x, float* tmp,
                   float* sc, float* out, VaeWs& w) {
  ALCM_TRY(group_norm_affine(x, B, T, r.cin, (int64_t)T * r.cin, r.cin, 32, 1e-6f, r.n1.g, r.n1.b, w.gsc, w.gsh, s));
  if (vae_planes(pk3)) {
    // GN affine + swish -> plane, conv1 on the wide-layer kernel; again for conv2 with bias + residual
    ALCM_TRY(affine_plane(x, B, T, r.cin, 1, w.gsc, w.gsh, 1, w.pl, pk3, s));
    ALCM_TRY(plane_conv3(s, pk3, B, T, r.cin, w.pl, r.c1, nullptr, tmp));
    ALCM_TRY(group_norm_affine(tmp, B, T, r.cout, (int64_t)T * r.cout, r.cout, 32, 1e-6f, r.n2.g, r.n2.b, w.gsc,
                               w.gsh, s));
    const float* resid = x;
    if (r.has_nin) {
      int rc;  // `out` is free until conv2 writes it: the split planes of x go there
      if (!split_1x1(s, split, B, T, x, r.cin, nullptr, nullptr, r.nin, nullptr, sc, r.cout,
                     reinterpret_cast<u16*>(out), &rc))
        ALCM_TRY(conv(s, split, B, T, cl(x, T, r.cin), r.nin, ocl(sc, T, r.cout), ConvOpts{}));
      ALCM_TRY(rc);
      resid = sc;
    }
    ALCM_TRY(affine_plane(tmp, B, T, r.cout, 1, w.gsc, w.gsh, 1, w.pl, pk3, s));
    return plane_conv3(s, pk3, B, T, r.cout, w.pl, r.c2, resid, out);
  }
  ConvOpts o1;
  o1.pad = r.c1.w.taps / 2;
  o1.pro = Pro{w.gsc, w.gsh, r.cin, nullptr, nullptr, ACT_SILU};
  ALCM_TRY(conv(s, pk3, B, T, cl(x, T, r.cin), r.c1, ocl(tmp, T, r.cout), o1));
  ALCM_TRY(group_norm_affine(tmp, B, T, r.cout, (int64_t)T * r.cout, r.cout, 32, 1e-6f, r.n2.g, r.n2.b, w.gsc, w.gsh, s));
  const float* resid = x;
  if (r.has_nin) {
    int rc;
    if (!split_1x1(s, split, B, T, x, r.cin, nullptr, nullptr, r.nin, nullptr, sc, r.cout, reinterpret_cast<u16*>(out),
                   &rc))
      ALCM_TRY(conv(s, split, B, T, cl(x, T, r.cin), r.nin, ocl(sc, T, r.cout), ConvOpts{}));
    ALCM_TRY(rc);
    resid = sc;
  }
  ConvOpts o2;
  o2.pad = r.c2.w.taps / 2;
  o2.pro = Pro{w.gsc, w.gsh, r.cout, nullptr, nullptr, ACT_SILU};
  o2.res = Res{resid, (int64_t)T * r.cout, r.cout, 1};
  return conv(s, pk3, B, T, cl(tmp, T, r.cout), r.c2, ocl(out, T, r.cout), o2);
}

static int vae_attn(hipStream_t s, int split, int B, int T, int C, const NormW& nw, const ConvW& qkvw, const ConvW& ow,
                    float* h, float* o_scratch, VaeWs& w);

static int vae_decode(alcm_model* m, const float* z, float inv_scale, float* mel, int B, int T, void* ws, size_t wsb,
                      hipStream_t s) {
  const VaeW& V = m->vae;
  const int split = prec_of(m, false);
  const int pk3 = prec_of(m, true);  // k3 ResnetBlock1D / upsample convs
  if (B <= 0 || T <= 0) return set_error(ALCM_E_INVALID, "vae_decode: empty batch");
  Bump bp(ws, wsb);
  VaeWs w = plan_vae(V, bp, B, T);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "vae_decode: workspace too small");
  // z / scale_factor -> post_quant_conv (lcm_audio.py:403, autoencoder1d.py:59-62), z read as NCT
  ALCM_TRY(fill_f32(w.pqs, V.z_ch, inv_scale, s));
  ALCM_TRY(fill_f32(w.pqh, V.z_ch, 0.f, s));
  // (post_quant_conv's rows written at conv_in's padded channel stride, the padding zeroed first: conv_in then reads
  // whole vectors (ALCM_NCT_CL=0: rows of z_ch channels, read element by element))
  const int cpi = V.conv_in.w.cpad;
  const bool padrows = knobs().nct_cl && cpi > V.z_ch && cpi % 4 == 0;
  const int dst = padrows ? cpi : V.z_ch;
  if (padrows) ALCM_TRY(fill_f32(w.d, (int64_t)B * T * cpi, 0.f, s));
  {
    ConvOpts o;
    o.pro = Pro{w.pqs, w.pqh, 0, nullptr, nullptr, 0};
    ALCM_TRY(conv(s, split, B, T, View{z, (int64_t)V.embed * T, 1, T, T, V.embed}, V.pqc,
                  Out{w.d, (int64_t)T * dst, dst, 1, 1, 0}, o));
  }
  int C = V.ch * V.mult.back();
  {
    ConvOpts o;
    o.pad = V.ksz / 2;
    ALCM_TRY(conv(s, split, B, T, View{w.d, (int64_t)T * dst, dst, 1, T, dst}, V.conv_in, ocl(w.a, T, C), o));
  }
  float* h = w.a;
  ALCM_TRY(vae_res(s, split, pk3, B, T, V.mid1, h, w.b, nullptr, h, w));
  ALCM_TRY(vae_attn(s, split, B, T, C, V.attn_n, V.attn_qkv, V.attn_out, h, w.c, w));
  ALCM_TRY(vae_res(s, split, pk3, B, T, V.mid2, h, w.b, nullptr, h, w));
  int Tc = T;
  float* spare = w.c;  // third full buffer for channel-changing blocks
  for (int lvl = (int)V.mult.size() - 1; lvl >= 0; --lvl) {
    for (const ResW& r : V.lv[lvl]) {
      if (r.has_nin) {
        ALCM_TRY(vae_res(s, split, pk3, B, Tc, r, h, w.b, w.d, spare, w));
        std::swap(h, spare);
      } else {
        ALCM_TRY(vae_res(s, split, pk3, B, Tc, r, h, w.b, nullptr, h, w));
      }
      C = r.cout;
    }
    if (V.up[lvl].w.p && vae_planes(pk3)) {
      // Upsample1D: nearest x2 written as a duplicated-row plane, conv k3 on the wide-layer kernel
      ALCM_TRY(affine_plane(h, B, Tc, C, 2, nullptr, nullptr, 0, w.pl, pk3, s));
      ALCM_TRY(plane_conv3(s, pk3, B, 2 * Tc, C, w.pl, V.up[lvl], nullptr, spare));
      std::swap(h, spare);
      Tc *= 2;
    } else if (V.up[lvl].w.p) {
      // Upsample1D: nearest x2 folded into the conv's input index (autoencoder1d.py:291-295)
      ConvOpts o;
      o.pad = 1;
      o.up = 2;
      ALCM_TRY(conv(s, pk3, B, 2 * Tc, cl(h, Tc, C), V.up[lvl], ocl(spare, 2 * Tc, C), o));
      std::swap(h, spare);
      Tc *= 2;
    }
  }
  ALCM_TRY(group_norm_affine(h, B, Tc, C, (int64_t)Tc * C, C, 32, 1e-6f, V.norm_out.g, V.norm_out.b, w.gsc, w.gsh, s));
  ConvOpts o;
  o.pad = V.ksz / 2;
  o.pro = Pro{w.gsc, w.gsh, C, nullptr, nullptr, ACT_SILU};
  return conv(s, split, B, Tc, cl(h, Tc, C), V.conv_out, Out{mel, (int64_t)V.out_ch * Tc, 1, Tc, 1, 0}, o);
}

// AttnBlock1D (autoencoder1d.py:259-278): single head over T, logit scale C^-1/2; h += proj_out(attn(GN(h)));
// o_scratch (B, T, C) holds the attention output and must not alias h
static int vae_attn(hipStream_t s, int split, int B, int T, int C, const NormW& nw, const ConvW& qkvw, const ConvW& ow,
                    float* h, float* o_scratch, VaeWs& w) {
  if (o_scratch == h) return set_error(ALCM_E_INVALID, "vae_attn: scratch aliases the activation");
  {
    ALCM_TRY(group_norm_affine(h, B, T, C, (int64_t)T * C, C, 32, 1e-6f, nw.g, nw.b, w.gsc, w.gsh, s));
    int rc;  // w.b (the ResnetBlock1D scratch) is free here: the split planes go there
    if (!split_1x1(s, split, B, T, h, C, w.gsc, w.gsh, qkvw, nullptr, w.qkv, 3 * C, reinterpret_cast<u16*>(w.b), &rc)) {
      ConvOpts o;
      o.pro = Pro{w.gsc, w.gsh, C, nullptr, nullptr, 0};
      ALCM_TRY(conv(s, split, B, T, cl(h, T, C), qkvw, ocl(w.qkv, T, 3 * C), o));
    }
    ALCM_TRY(rc);
    const int Tp = round_up(T, 8);
    alcm_gemm_args g;
    std::memset(&g, 0, sizeof(g));
    g.M = T; g.N = T; g.Kpad = round_up(C, kBK); g.batch = B; g.zdiv = 1;
    g.a.kind = ALCM_OPND_ACT; g.a.ptr = w.qkv; g.a.st = 3 * C; g.a.sc = 1; g.a.T_in = T; g.a.C_in = C; g.a.Cpad = C;
    g.a.ksize = 1; g.a.dil = 1; g.a.up = 1; g.a.rows_per_batch = T; g.a.zs1 = (int64_t)T * 3 * C;
    g.b = g.a;
    g.b.ptr = w.qkv + C;
    g.acc_scale = 1.0f / sqrtf((float)C);
    g.out_scale = 1.f;
    g.out = w.S; g.o_st = Tp; g.o_sc = 1; g.o_zs1 = (int64_t)T * Tp; g.out_rows_per_batch = T; g.out_step = 1;
    g.prec = split;
    ALCM_TRY(gemm(g, s));
    ALCM_TRY(softmax_rows(w.S, B * T, T, Tp, s));
    alcm_gemm_args p;
    std::memset(&p, 0, sizeof(p));
    p.M = T; p.N = C; p.Kpad = round_up(Tp, kBK); p.batch = B; p.zdiv = 1;
    p.a.kind = ALCM_OPND_ACT; p.a.ptr = w.S; p.a.st = Tp; p.a.sc = 1; p.a.T_in = T; p.a.C_in = Tp; p.a.Cpad = Tp;
    p.a.ksize = 1; p.a.dil = 1; p.a.up = 1; p.a.rows_per_batch = T; p.a.zs1 = (int64_t)T * Tp;
    p.b.kind = ALCM_OPND_ACT_T; p.b.ptr = w.qkv + 2 * C; p.b.st = 3 * C; p.b.sc = 1; p.b.T_in = T; p.b.rows = C;
    p.b.zs1 = (int64_t)T * 3 * C;
    p.acc_scale = 1.f; p.out_scale = 1.f;
    p.out = o_scratch; p.o_st = C; p.o_sc = 1; p.o_zs1 = (int64_t)T * C; p.out_rows_per_batch = T; p.out_step = 1;
    p.prec = split;
    ALCM_TRY(gemm(p, s));
    if (!split_1x1(s, split, B, T, o_scratch, C, nullptr, nullptr, ow, h, h, C, reinterpret_cast<u16*>(w.b), &rc)) {
      ConvOpts oo;
      oo.res = Res{h, (int64_t)T * C, C, 1};
      ALCM_TRY(conv(s, split, B, T, cl(o_scratch, T, C), ow, ocl(h, T, C), oo));
    }
    ALCM_TRY(rc);
  }
  return 0;
}

// Encoder1D + quant_conv (autoencoder1d.py:319-413, AutoencoderKL.encode :54-58): mel (B, in_ch, M) NCT ->
// moments (B, 2 embed, To) NCT, To = M / 2^len(down_layers); DiagonalGaussianDistribution is host-side
static int vae_encode(alcm_model* m, const float* x, float* moments, int B, int M, void* ws, size_t wsb,
                      hipStream_t s) {
  const VaeW& V = m->vae;
  const VaeEncW& E = V.enc;
  if (!E.present) return set_error(ALCM_E_MISSING, "vae_encode: the model was created without encoder.* weights");
  const int split = prec_of(m, false);
  const int pk = prec_of(m, true);
  if (B <= 0 || M <= 1) return set_error(ALCM_E_INVALID, "vae_encode: bad shape");
  Bump bp(ws, wsb);
  VaeWs w = plan_vae(V, bp, B, M);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "vae_encode: workspace too small");
  int C = V.ch, T = M;
  {
    ConvOpts o;
    o.pad = V.ksz / 2;
    ALCM_TRY(conv(s, split, B, T, View{x, (int64_t)E.in_ch * T, 1, T, T, E.in_ch}, E.conv_in, ocl(w.a, T, C), o));
  }
  float* h = w.a;
  float* spare = w.c;
  for (size_t lvl = 0; lvl < E.lv.size(); ++lvl) {
    for (const ResW& r : E.lv[lvl]) {
      if (r.has_nin) {
        ALCM_TRY(vae_res(s, split, pk, B, T, r, h, w.b, w.d, spare, w));
        std::swap(h, spare);
      } else {
        ALCM_TRY(vae_res(s, split, pk, B, T, r, h, w.b, nullptr, h, w));
      }
      C = r.cout;
    }
    if (E.down[lvl].w.p) {
      // Downsample1D (autoencoder1d.py:310-317): zero pad (0, 1), conv k3 stride 2 = the stride-1 conv (pad 0;
      // rows past T read zeros) at even rows
      const int To = (T - 2) / 2 + 1;
      ALCM_TRY(conv(s, split, B, T, cl(h, T, C), E.down[lvl], ocl(w.b, T, C), ConvOpts{}));
      ALCM_TRY(rows_stride2(w.b, B, T, To, C, spare, s));
      std::swap(h, spare);
      T = To;
    }
  }
  ALCM_TRY(vae_res(s, split, pk, B, T, E.mid1, h, w.b, nullptr, h, w));
  ALCM_TRY(vae_attn(s, split, B, T, C, E.attn_n, E.attn_qkv, E.attn_out, h, h == w.c ? w.d : w.c, w));
  ALCM_TRY(vae_res(s, split, pk, B, T, E.mid2, h, w.b, nullptr, h, w));
  ALCM_TRY(group_norm_affine(h, B, T, C, (int64_t)T * C, C, 32, 1e-6f, E.norm_out.g, E.norm_out.b, w.gsc, w.gsh, s));
  {
    ConvOpts o;
    o.pad = V.ksz / 2;
    o.pro = Pro{w.gsc, w.gsh, C, nullptr, nullptr, ACT_SILU};
    ALCM_TRY(conv(s, split, B, T, cl(h, T, C), E.conv_out, ocl(spare, T, 2 * V.z_ch), o));
  }
  return conv(s, split, B, T, cl(spare, T, 2 * V.z_ch), E.quant, Out{moments, (int64_t)2 * V.embed * T, 1, T, 1, 0},
              ConvOpts{});
}

// log-mel spectrogram (MelNet.forward, NAT_mel.py:66-85, center=False): clamp(-1, 1), reflect pad (n_fft - hop)/2,
// |STFT| (hann window, onesided) -> mel_basis @ mag -> log10(clamp(1e-5)); wav (B, L), L % hop == 0 -> (B, n_mels, L/hop)
struct MelWs {
  float *ypad, *spec, *mag, *mel;
};
static MelWs plan_mel(const MelW& Mw, Bump& bp, int B, int L) {
  const size_t Fr = (size_t)L / Mw.hop;
  MelWs w;
  w.ypad = bp.take<float>((size_t)B * (L + Mw.n_fft - Mw.hop) + 64);
  w.spec = bp.take<float>((size_t)B * Fr * 2 * Mw.n_freq);
  w.mag = bp.take<float>((size_t)B * Fr * Mw.n_freq);
  w.mel = bp.take<float>((size_t)B * Fr * Mw.n_mels);
  return w;
}
static int mel_forward(alcm_model* m, const float* wav, float* mel, int B, int L, void* ws, size_t wsb, hipStream_t s) {
  const MelW& Mw = m->mel;
  if (B <= 0 || L <= 0 || L % Mw.hop || L <= (Mw.n_fft - Mw.hop) / 2)
    return set_error(ALCM_E_INVALID, "mel_spectrogram: the waveform length must be a positive multiple of hop");
  Bump bp(ws, wsb);
  MelWs w = plan_mel(Mw, bp, B, L);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "mel_spectrogram: workspace too small");
  const int p = (Mw.n_fft - Mw.hop) / 2, Lp = L + 2 * p, rows = Lp / Mw.hop, Fr = L / Mw.hop, F = Mw.n_freq;
  const int prec = m->policy == ALCM_POLICY_BF16 ? PREC_BF16 : PREC_SPLIT;  // log-magnitudes: keep fp32 accuracy
  ALCM_TRY(reflect_pad_clamp(wav, B, L, p, w.ypad, s));
  // frame f = padded samples [f hop, f hop + n_fft) = hop-rows f .. f + n_fft/hop - 1: a conv over the rows
  ALCM_TRY(conv(s, prec, B, Fr, View{w.ypad, (int64_t)Lp, Mw.hop, 1, rows, Mw.hop}, Mw.dft,
                ocl(w.spec, Fr, 2 * F), ConvOpts{}));
  ALCM_TRY(stft_magnitude(w.spec, F, (int64_t)B * Fr, w.mag, s));
  ALCM_TRY(lin(s, prec, B * Fr, w.mag, F, Mw.basis, w.mel, ConvOpts{}));
  return log10_nct(w.mel, B, Fr, Mw.n_mels, mel, s);
}

// ------------------------------------------------------------------ BigVGAN
struct VocChain {  // per-resblock scratch: running state ping-pong and the two operand-plane buffers
  float *rb, *t;
  u16 *pl, *pl2;  // Activation1d outputs as MFMA operand planes (each 2 planes of B * T * Cp)
};
struct VocWs {
  float *x, *y;
  VocChain ch[3];
  int64_t pl_lo;
  // legacy single-chain names (chain 0)
  float *rb, *t;
  u16 *pl, *pl2;
};
static size_t voc_elems(const VocW& G, int M) {
  size_t big = (size_t)M * G.c0;
  int T = M;
  for (const StageW& S : G.st) {
    T *= S.rate;
    big = std::max(big, (size_t)T * S.cout);
  }
  return big;
}
static VocWs plan_voc(const VocW& G, Bump& bp, int B, int M) {
  const size_t e = (size_t)B * voc_elems(G, M);
  size_t pe = 0;  // largest B * T * Cp over the AMPBlock stages
  int T = M;
  for (const StageW& S : G.st) {
    T *= S.rate;
    pe = std::max(pe, (size_t)B * T * round_up(S.cout, 32));
  }
  VocWs w;
  w.x = bp.take<float>(e);
  w.y = bp.take<float>(e);
  for (VocChain& c : w.ch) {
    c.rb = bp.take<float>(e);
    c.t = bp.take<float>(e);
    c.pl = bp.take<u16>(2 * pe);
    c.pl2 = bp.take<u16>(2 * pe);
  }
  w.rb = w.ch[0].rb;
  w.t = w.ch[0].t;
  w.pl = w.ch[0].pl;
  w.pl2 = w.ch[0].pl2;
  w.pl_lo = (int64_t)pe;
  return w;
}

// MFMA precision of the AMPBlock layers of stage si (scripts/precision_emulate.py):
// mixed policy: fp16 for the three wide stages (~96% of the BigVGAN FLOPs), fp16 activation x fp16 hi+lo
// weight for the narrow tail (the tail is sensitive to weight rounding, not to activation rounding);
// conv_post stays bf16x3 (bigvgan_forward)
static int voc_prec(const alcm_model* m, int si) {
  if (m->policy == ALCM_POLICY_BF16) return PREC_BF16;
  if (m->policy == ALCM_POLICY_SPLIT) return PREC_SPLIT;
  // stage 3 (C = 96, the costliest tail stage) tolerates fp16 weights: +1e-5 waveform rel-L2 emulated,
  // vs +2.5e-4 (stage 4) and +4.3e-4 (stage 5) (scripts/precision_emulate.py 96 tail)
  return si < 4 ? PREC_F16 : PREC_F16W2;
}

static int act_planes(hipStream_t s, const ActW& a, const float* x, const VocWs& w, int B, int T, int C, int prec,
                      u16* planes = nullptr) {
  return activation1d_op(x, planes ? planes : w.pl, B, T, C, round_up(C, 32), a.aexp, a.ibeta, a.fup, a.fdn, prec,
                         s);
}

// the auxiliary resblock streams / events of caller stream s (nullptr: run the chains serially on s)
static const alcm_model::AuxSet* voc_streams(alcm_model* m, hipStream_t s) {
  if (!m->resblock_streams) return nullptr;
  std::lock_guard<std::mutex> lk(m->aux_mu);
  auto it = m->aux.find(s);
  if (it != m->aux.end()) return &it->second;
  alcm_model::AuxSet a;
  bool ok = true;
  for (auto& x : a.s) ok = ok && hipStreamCreateWithFlags(&x, hipStreamNonBlocking) == hipSuccess;
  for (auto& e : a.ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    for (auto x : a.s)
      if (x) (void)hipStreamDestroy(x);
    for (auto e : a.ev)
      if (e) (void)hipEventDestroy(e);
    return nullptr;
  }
  return &(m->aux[s] = a);
}

// conv on the operand planes `in`; with `act` the epilogue also writes Activation1d(conv + bias (+ res)) into
// the planes `act_out` (alcm_actepi.h), and `out` may be null
// the narrow stages' AMPBlock convs on the resident-weight kernel (alcm_tconv.hip): every conv of the stage or none
// (its planes keep stale operand-padding channels, which only that kernel ignores)
static bool stage_tconv(const StageW& S, int prec) {
  if (S.rb.empty() || !S.rb[0].c1[0].dw.p) return false;
  for (const AmpW& A : S.rb)
    for (size_t l = 0; l < A.dil.size(); ++l)
      if (!tconv_supported(prec, S.cout, S.cout, A.k, A.dil[l])) return false;
  return true;
}

// the alcm_opconv arguments of a same-length conv of the planes `in` (default: the workspace planes)
static alcm_opconv_args plane_args(const ConvW& cw, const VocWs& w, int B, int T, int dil, const float* res, float* out,
                                   float out_scale, int accumulate, int out_act, int prec, const u16* in) {
  alcm_opconv_args g;
  std::memset(&g, 0, sizeof(g));
  g.a = in ? in : w.pl; g.a_lo_off = (int64_t)B * T * cw.w.cpad;
  g.B = B; g.T = T; g.C = cw.w.cin; g.Cp = cw.w.cpad;
  g.ksize = cw.w.taps; g.dil = dil; g.pad = (cw.w.taps - 1) * dil / 2;
  g.w = cw.w.p; g.w_lo_off = cw.w.lo; g.kpad = cw.w.kpad; g.N = cw.w.rows;
  g.bias = cw.b; g.res = res; g.out = out; g.out_act = out_act; g.accumulate = accumulate;
  g.out_scale = out_scale; g.prec = prec;
  return g;
}

static int plane_conv(hipStream_t s, const ConvW& cw, const VocWs& w, int B, int T, int dil, const float* res,
                      float* out, float out_scale, int accumulate, int out_act, int prec, const u16* in = nullptr,
                      const ActW* act = nullptr, u16* act_out = nullptr, bool dense = false,
                      void* out_plane = nullptr) {
  alcm_opconv_args g;
  std::memset(&g, 0, sizeof(g));
  if (dense) {
    g.a = in ? in : w.pl;
    g.B = B; g.T = T; g.C = cw.w.cin; g.Cp = cw.w.cpad;
    g.ksize = cw.w.taps; g.dil = dil; g.pad = (cw.w.taps - 1) * dil / 2;
    g.N = cw.w.rows; g.bias = cw.b; g.res = res; g.out = out; g.out_scale = out_scale; g.accumulate = accumulate;
    g.prec = prec;
    ActEpiDev E{};
    if (act) {
      E.plane = act_out;
      E.plane_lo = 0;
      E.Cp = round_up(cw.w.rows, 32);
      E.aexp = act->aexp;
      E.ibeta = act->ibeta;
      for (int k = 0; k < 12; ++k) {
        E.f.up[k] = 2.0f * act->fup[k];
        E.f.dn[k] = act->fdn[k];
      }
    }
    const double M = (double)B * T;
    const double flops = 2.0 * M * g.N * (double)g.ksize * g.C;
    const double bytes = M * g.C * 2.0 + (double)g.N * cw.dw.kpad * 2.0 * (prec == PREC_F16W2 ? 2 : 1) +
                         M * g.N * 4.0 * ((out ? 1 : 0) + (res ? 1 : 0) + (accumulate ? 1 : 0)) +
                         (act ? M * g.N * 2.0 : 0.0);
    return tconv(g, cw.dw.p + 2 * cw.dw.lo, cw.dw.lo, cw.dw.kpad, act ? &E : nullptr, flops, bytes, s);
  }
  g = plane_args(cw, w, B, T, dil, res, out, out_scale, accumulate, out_act, prec, in);
  if (act) {
    g.act_plane = act_out;
    g.act_plane_lo_off = (int64_t)B * T * round_up(cw.w.rows, 32);
    g.act_alpha_exp = act->aexp;
    g.act_inv_beta = act->ibeta;
    g.act_up_filter = act->fup;
    g.act_down_filter = act->fdn;
  }
  g.out_plane = out_plane;
  return opconv(g, s);
}

static int bigvgan_forward(alcm_model* m, const float* mel, float* wav, int B, int M, void* ws, size_t wsb,
                           hipStream_t s) {
  const VocW& G = m->voc;
  const int split = prec_of(m, false);
  if (B <= 0 || M <= 0) return set_error(ALCM_E_INVALID, "bigvgan_forward: empty batch");
  Bump bp(ws, wsb);
  VocWs w = plan_voc(G, bp, B, M);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "bigvgan_forward: workspace too small");
  // conv_pre k7 on the NCT mel (models.py:183)
  {
    ConvOpts o;
    o.pad = 3;
    // the NCT mel as channels-last rows (chain 1's fp32 scratch, free until the first stage's chains), read as whole
    // vectors instead of a stride-M gather per element (ALCM_NCT_CL=0: the gather)
    const int cp = G.pre.w.cpad;
    View mv{mel, (int64_t)G.num_mels * M, 1, M, M, G.num_mels};
    if (knobs().nct_cl && cp % 4 == 0) {
      ALCM_TRY(nct_to_cl(mel, B, G.num_mels, M, cp, w.ch[1].t, s));
      mv = View{w.ch[1].t, (int64_t)M * cp, cp, 1, M, cp};
    }
    ALCM_TRY(conv(s, split, B, M, mv, G.pre, ocl(w.x, M, G.c0), o));
  }
  // buffer roles: x = stage input and (after the upsampler) stage output accumulator,
  // u = upsampler output (resblock input), rb = resblock running state, a / y = scratch
  int T = M;
  float* x = w.x;
  float* u = w.y;
  float* rb = w.rb;
  float* y = w.t;
  // stage si's upsampler runs on operand planes of its input (mixed policy: stages 0-3, +1.9e-4 waveform rel-L2
  // emulated, scripts/precision_emulate.py 96 tail): a plane conv of x with a strided epilogue (the wide-layer kernel
  // for N % 192 == 0, opconv_kernel for N <= 96) — the same eligibility opconv's strided paths check (the wide-layer
  // kernel needs Cp % 64 == 0 and a tap window of at most 64 rows; otherwise the fp32-operand phase conv below)
  auto ups_planes_of = [&](size_t si) {
    const StageW& S = G.st[si];
    const int pamp = voc_prec(m, (int)si);
    const bool wide_ok = S.cout % 192 == 0 && S.cin % 64 == 0 && S.phase[0].w.taps - 1 <= 64;
    return (pamp == PREC_F16 || pamp == PREC_BF16) && S.cin % 32 == 0 &&
           (wide_ok || (S.cout <= 96 && S.cout % 4 == 0)) && S.phase[0].w.cpad == S.cin;
  };
  const u16* xpl = nullptr;  // the stage input's planes when the previous stage's sum-form conv wrote them
  for (size_t si = 0; si < G.st.size(); ++si) {
    const StageW& S = G.st[si];
    const int To = T * S.rate;
    const int pamp = voc_prec(m, (int)si);
    // ConvTranspose1d as S.rate phase convolutions (models.py:160-165, 187-188): on operand planes of x where
    // ups_planes_of(si), the fp32-operand conv at the base precision otherwise
    const bool ups_planes = ups_planes_of(si);
    const u16* upl = xpl ? xpl : w.pl;
    if (ups_planes && !xpl) ALCM_TRY(to_planes(x, w.pl, (int64_t)B * T, S.cin, S.cin, pamp, s));
    xpl = nullptr;
    // the split-precision stride-2 stages with the kernel's widths (stages 4-5): both phases in one pass over x
    const bool ups_two = !ups_planes && split == PREC_SPLIT && S.rate == 2 &&
                         ups2_supported(S.cin, S.cout, S.phase[0].w.cpad, S.rate, S.phase[0].w.taps) &&
                         S.phase[1].w.kpad == S.phase[0].w.kpad && S.phase[1].w.lo == S.phase[0].w.lo;
    if (ups_two)
      ALCM_TRY(ups2(x, u, B, T, S.cin, S.cout, S.phase[0].w.p, S.phase[1].w.p, S.phase[0].w.lo, S.phase[0].w.kpad,
                    S.pad.data(), S.off.data(), S.phase[0].b, s));
    for (int r = 0; r < S.rate && !ups_two; ++r) {
      if (ups_planes) {
        const ConvW& cw = S.phase[r];
        alcm_opconv_args g;
        std::memset(&g, 0, sizeof(g));
        g.a = upl; g.a_lo_off = (int64_t)B * T * S.cin;
        g.B = B; g.T = T; g.C = S.cin; g.Cp = S.cin;
        g.ksize = cw.w.taps; g.dil = 1; g.pad = S.pad[r];
        g.w = cw.w.p; g.w_lo_off = cw.w.lo; g.kpad = cw.w.kpad; g.N = cw.w.rows;
        g.bias = cw.b; g.out = u; g.out_scale = 1.f; g.prec = pamp;
        g.out_stride = S.rate; g.out_offset = S.off[r]; g.out_rows = To;
        ALCM_TRY(opconv(g, s));
        continue;
      }
      ConvOpts o;
      o.pad = S.pad[r];
      ALCM_TRY(conv(s, split, B, T, cl(x, T, S.cin), S.phase[r],
                    Out{u, (int64_t)To * S.cout, S.cout, 1, S.rate, S.off[r]}, o));
    }
    // x = mean over k in (3,7,11) of AMPBlock1(k, (1,3,5))(u)  (models.py:190-199, 72-81); each half-layer
    // is Activation1d -> operand planes -> implicit-GEMM conv on the planes.  Fused form (every stage the
    // kernels support at this precision): the first Activation1d of a resblock runs standalone (act_op); every
    // later one runs in the epilogue of the conv that produces its input (conv1 writes only planes; conv2
    // writes the fp32 running state, ping-ponged between rb and y since its tiles overlap, plus planes)
    const float inv = 1.0f / (float)S.rb.size();
    const bool fuse = opconv_act_supported(pamp, S.cout, round_up(S.cout, 32));
    const bool dense = fuse && stage_tconv(S, pamp);
    const alcm_model::AuxSet* ax = S.rb.size() <= 3 ? voc_streams(m, s) : nullptr;
    const bool conc = ax != nullptr;
    // the wide stages' conv1 -> Activation1d hand-off as an fp16 plane (ALCM_CONV1_H16=0: fp32, the A/B reference).
    // Only from B * To >= 1024 rows, where the fp32 route takes the same wide kernel (below it the fp32 output would
    // go to opconv_kernel, whose K order differs): the A/B stays bit-exact at every size
    const bool h16 = knobs().conv1_h16 && pamp == PREC_F16 && act_mfma_ok(S.cout, round_up(S.cout, 32), pamp) &&
                     (int64_t)B * To >= 1024;
    // the three chains' first Activation1d in one pass over u (their own planes, same taps) — with the chains on
    // their streams and serialised alike (each chain on its own buffers then), so the serialised profile pass runs
    // the same kernels as the concurrent one
    // (the narrow fused stages: the VALU kernel; the wide MFMA-FIR stages: its three-set form, ALCM_ACT_X3_MFMA)
    const bool amok = act_mfma_ok(S.cout, round_up(S.cout, 32), pamp);
    bool act3 = S.rb.size() == 3 && (fuse ? !amok : (amok && knobs().act_x3_mfma));
    for (size_t j = 1; act3 && j < S.rb.size(); ++j)
      act3 = !std::memcmp(S.rb[j].act[0].fup, S.rb[0].act[0].fup, sizeof(S.rb[0].act[0].fup)) &&
             !std::memcmp(S.rb[j].act[0].fdn, S.rb[0].act[0].fdn, sizeof(S.rb[0].act[0].fdn));
    if (act3) {
      void* ys[3] = {w.ch[0].pl, w.ch[1].pl, w.ch[2].pl};
      const float* ae[3] = {S.rb[0].act[0].aexp, S.rb[1].act[0].aexp, S.rb[2].act[0].aexp};
      const float* ib[3] = {S.rb[0].act[0].ibeta, S.rb[1].act[0].ibeta, S.rb[2].act[0].ibeta};
      ALCM_TRY(activation1d_x3(u, ys, B, To, S.cout, round_up(S.cout, 32), ae, ib, S.rb[0].act[0].fup,
                               S.rb[0].act[0].fdn, pamp, s));
    }
    if (conc) {  // chains start after the upsampler wrote u
      ALCM_HIP(hipEventRecord(ax->ev[0], s));
      for (auto a : ax->s) ALCM_HIP(hipStreamWaitEvent(a, ax->ev[0], 0));
    }
    // the wide stages' mean over the three chains in one sum-form launch of their last conv2 + residual
    // (alcm_opconv_sum): x written once, not read and rewritten per chain (ALCM_WCONV_SUM=0: three accumulating
    // launches, the chains' last convs in order)
    const bool sum3 = !fuse && S.rb.size() == 3 && (conc || act3) && knobs().wconv_sum;
    alcm_opconv_args lastc[3];
    for (size_t j = 0; j < S.rb.size(); ++j) {
      const AmpW& A = S.rb[j];
      const VocChain& cb = w.ch[(conc || act3) ? j : 0];
      const hipStream_t sj = (conc && j > 0) ? ax->s[j - 1] : s;
      const float* cur = u;
      float* nxt = cb.rb;
      for (size_t l = 0; l < A.dil.size(); ++l) {
        const bool last = l + 1 == A.dil.size();
        // the mean over resblocks accumulates into x: the chains' last convs run in order (j-1 before j)
        if (last && conc && j > 0 && !sum3) ALCM_HIP(hipStreamWaitEvent(sj, ax->ev[j], 0));
        if (fuse) {
          if (l == 0 && !act3) ALCM_TRY(act_planes(sj, A.act[0], cur, w, B, To, S.cout, pamp, cb.pl));
          ALCM_TRY(plane_conv(sj, A.c1[l], w, B, To, A.dil[l], nullptr, nullptr, 1.f, 0, 0, pamp, cb.pl,
                              &A.act[2 * l + 1], cb.pl2, dense));
          if (last) {
            ALCM_TRY(plane_conv(sj, A.c2[l], w, B, To, 1, cur, x, inv, j > 0, 0, pamp, cb.pl2, nullptr, nullptr,
                                dense));
          } else {
            ALCM_TRY(plane_conv(sj, A.c2[l], w, B, To, 1, cur, nxt, 1.f, 0, 0, pamp, cb.pl2, &A.act[2 * l + 2],
                                cb.pl, dense));
            cur = nxt;
            nxt = nxt == cb.rb ? cb.t : cb.rb;
          }
        } else {
          if (!(l == 0 && act3)) ALCM_TRY(act_planes(sj, A.act[2 * l], cur, w, B, To, S.cout, pamp, cb.pl));
          if (h16) {
            // conv1's only consumer is the next Activation1d, whose MFMA kernel rounds its input to fp16: conv1 writes
            // that fp16 plane (into the fp32 scratch cb.t) and the activation reads it, bit-identical at half the bytes
            ALCM_TRY(plane_conv(sj, A.c1[l], w, B, To, A.dil[l], nullptr, nullptr, 1.f, 0, 0, pamp, cb.pl, nullptr,
                                nullptr, false, cb.t));
            const ActW& a2 = A.act[2 * l + 1];
            ALCM_TRY(activation1d_op_h16(cb.t, cb.pl, B, To, S.cout, round_up(S.cout, 32), a2.aexp, a2.ibeta, a2.fup,
                                         a2.fdn, pamp, sj));
          } else {
            ALCM_TRY(plane_conv(sj, A.c1[l], w, B, To, A.dil[l], nullptr, cb.t, 1.f, 0, 0, pamp, cb.pl));
            ALCM_TRY(act_planes(sj, A.act[2 * l + 1], cb.t, w, B, To, S.cout, pamp, cb.pl));
          }
          if (last && sum3)
            lastc[j] = plane_args(A.c2[l], w, B, To, 1, cur, j == 0 ? x : nullptr, inv, 0, 0, pamp, cb.pl);
          else
            ALCM_TRY(plane_conv(sj, A.c2[l], w, B, To, 1, cur, last ? x : cb.rb, last ? inv : 1.f, last && j > 0, 0,
                                pamp, cb.pl));
          cur = cb.rb;
        }
        if (last && conc) ALCM_HIP(hipEventRecord(ax->ev[j + 1], sj));
      }
    }
    if (sum3) {
      if (conc)
        for (size_t j = 1; j < S.rb.size(); ++j) ALCM_HIP(hipStreamWaitEvent(s, ax->ev[j + 1], 0));
      // the next stage's upsampler reads only the operand planes of this output: the sum-form epilogue writes them
      // (the rounding to_planes applies to the fp32 value, bit for bit) into chain 0's spare plane buffer, free
      // until the next stage's chains start
      if (knobs().wconv_sum == 1 && si + 1 < G.st.size() && ups_planes_of(si + 1) && voc_prec(m, (int)si + 1) == pamp &&
          G.st[si + 1].cin == S.cout) {
        alcm_opconv_args pc[3] = {lastc[0], lastc[1], lastc[2]};
        pc[0].out = nullptr;
        pc[0].out_plane = w.ch[0].pl2;
        if (wconv3_sum_ok(pc, 3)) {
          lastc[0] = pc[0];
          xpl = w.ch[0].pl2;
        }
      }
      ALCM_TRY(opconv_sum(lastc, 3, s));
    } else if (conc) {
      ALCM_HIP(hipStreamWaitEvent(s, ax->ev[S.rb.size()], 0));  // the stage output is complete
    }
    T = To;
  }
  // activation_post -> conv_post k7 -> tanh (models.py:201-203)
  // conv_post maps 24 channels to the waveform: its input rounding shows up 1:1 in the output, so the
  // mixed policy keeps it bf16x3 (one launch, ~5e-4 of the waveform error budget otherwise)
  const int ppost = m->policy == ALCM_POLICY_BF16 ? PREC_BF16 : PREC_SPLIT;
  if (ppost == PREC_SPLIT && G.st.back().cout == 24 && G.post_w32) {
    // one fused fp32 launch (alcm_act.hip post_kernel): exact fp32 where the split path approximates it
    Taps12O f;
    for (int k = 0; k < 12; ++k) {
      f.up[k] = 2.0f * G.post_act.fup[k];
      f.dn[k] = G.post_act.fdn[k];
    }
    void* tok = prof_start(s);
    ALCM_TRY(act_conv_post(x, wav, B, T, 24, G.post_act.aexp, G.post_act.ibeta, f, G.post_w32, G.post_bias, s));
    if (tok) {
      const double n = (double)B * T;
      prof_stop(tok, s, "alcm::post_kernel<24>", n * 24 * (2 * 24 + 2 * 12) + n * 2 * 7 * 24, n * 24 * 4 + n * 4);
    }
    return 0;
  }
  ALCM_TRY(act_planes(s, G.post_act, x, w, B, T, G.st.back().cout, ppost));
  return plane_conv(s, G.post, w, B, T, 1, nullptr, wav, 1.f, 0, ACT_TANH, ppost);
}

// ------------------------------------------------------------------ text conditioning
// FrozenCLAPFLANEmbedder.encode (ldm/modules/encoders/modules.py:567-582) from token ids:
//   z  = Projection(BertModel(clap_ids).last_hidden_state)     CLAP/clap.py:8-20, transformers BertModel
//   z2 = T5EncoderModel(t5_ids).last_hidden_state              transformers T5 (v1.1: gated-gelu, RMSNorm)
//   out = concat([z, z2], dim=1)  -> (B, 2L, 1024)
// Both encoders run without an attention mask (the reference passes input_ids only), so padding tokens attend.
// Weight names are the embedder's state_dict keys: caption_encoder.base.* (BERT), caption_encoder.projection.*,
// t5_transformer.* (Appendix A: cond_stage_model.* of the Lightning checkpoint, prefix stripped).
static void build_text(Ingest& I, const int* ic, int nic) {
  TextW& X = I.m->text;
  if (nic >= 14) {
    X.b_vocab = ic[0]; X.b_hidden = ic[1]; X.b_layers = ic[2]; X.b_heads = ic[3]; X.b_inter = ic[4];
    X.b_maxpos = ic[5]; X.p_out = ic[6]; X.t_vocab = ic[7]; X.t_d = ic[8]; X.t_dkv = ic[9]; X.t_heads = ic[10];
    X.t_ff = ic[11]; X.t_layers = ic[12]; X.max_len = ic[13];
  }
  const int H = X.b_hidden, D = X.t_d, TI = X.t_heads * X.t_dkv;
  if (H % X.b_heads || (H / X.b_heads) % 8 || H % 4 || D % 4 || X.t_dkv % 8 || X.max_len > X.b_maxpos ||
      X.max_len <= 0 || X.p_out % 4)
    throw Error(ALCM_E_INVALID, "unsupported text-encoder geometry");
  const std::string bp = "caption_encoder.base.", pp = "caption_encoder.projection.", tp = "t5_transformer.";
  // BERT embeddings: word + position + token_type[0] (token_type_ids default to zeros), then LayerNorm
  X.b_word = I.upload(I.get(bp + "embeddings.word_embeddings.weight", {X.b_vocab, H}));
  {
    std::vector<float> pos = I.get(bp + "embeddings.position_embeddings.weight", {X.b_maxpos, H});
    const int64_t ntt = I.has(bp + "embeddings.token_type_embeddings.weight") ?
        I.by.at(bp + "embeddings.token_type_embeddings.weight")->shape[0] : 0;
    if (ntt <= 0) throw Error(ALCM_E_MISSING, "missing weight tensor '" + bp + "embeddings.token_type_embeddings.weight'");
    std::vector<float> tt = I.get(bp + "embeddings.token_type_embeddings.weight", {ntt, H});
    for (int t = 0; t < X.b_maxpos; ++t)
      for (int c = 0; c < H; ++c) pos[(size_t)t * H + c] += tt[c];
    X.b_pos_type = I.upload(pos);
  }
  X.b_emb_ln = I.norm(bp + "embeddings.LayerNorm.", H);
  for (int l = 0; l < X.b_layers; ++l) {
    const std::string p = bp + "encoder.layer." + std::to_string(l) + ".";
    BertLayerW L;
    std::vector<float> w, b;
    for (const char* q : {"query", "key", "value"}) {
      auto wq = I.get(p + "attention.self." + q + ".weight", {H, H});
      auto bq = I.get(p + "attention.self." + q + ".bias", {H});
      w.insert(w.end(), wq.begin(), wq.end());
      b.insert(b.end(), bq.begin(), bq.end());
    }
    L.qkv.w = I.pack(w, 3 * H, H, 1);
    L.qkv.b = I.upload(b);
    L.ao = I.linear(p + "attention.output.dense.", H, H);
    L.ln1 = I.norm(p + "attention.output.LayerNorm.", H);
    L.inter = I.linear(p + "intermediate.dense.", X.b_inter, H);
    L.out = I.linear(p + "output.dense.", H, X.b_inter);
    L.ln2 = I.norm(p + "output.LayerNorm.", H);
    X.bl.push_back(L);
  }
  X.p1 = I.linear(pp + "linear1.", X.p_out, H, false);
  X.p2 = I.linear(pp + "linear2.", X.p_out, X.p_out, false);
  X.p_ln = I.norm(pp + "layer_norm.", X.p_out);
  // T5 encoder
  const std::string emb = I.has(tp + "shared.weight") ? tp + "shared.weight" : tp + "encoder.embed_tokens.weight";
  X.t_emb = I.upload(I.get(emb, {X.t_vocab, D}));
  {
    // relative position bias of block 0 (shared by every block): bias[h][i][j] = table[bucket(j - i)][h]; the
    // bucket table (T5Attention._relative_position_bucket, bidirectional) comes from the host as a tensor
    const int ML = X.max_len;
    auto bk = I.get("_alcm.t5_rel_buckets", {ML, ML});
    const std::string rb = tp + "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight";
    const int64_t nb = I.has(rb) ? I.by.at(rb)->shape[0] : 0;
    if (nb <= 0) throw Error(ALCM_E_MISSING, "missing weight tensor '" + rb + "'");
    auto tab = I.get(rb, {nb, X.t_heads});
    std::vector<float> bias((size_t)X.t_heads * ML * ML);
    for (int h = 0; h < X.t_heads; ++h)
      for (int i = 0; i < ML; ++i)
        for (int j = 0; j < ML; ++j) {
          const int64_t k = (int64_t)bk[(size_t)i * ML + j];
          if (k < 0 || k >= nb) throw Error(ALCM_E_INVALID, "relative position bucket out of range");
          bias[((size_t)h * ML + i) * ML + j] = tab[(size_t)k * X.t_heads + h];
        }
    X.t_bias = I.upload(bias);
  }
  for (int l = 0; l < X.t_layers; ++l) {
    const std::string p = tp + "encoder.block." + std::to_string(l) + ".layer.";
    T5BlockW Bk;
    Bk.ln0 = I.upload(I.get(p + "0.layer_norm.weight", {D}));
    std::vector<float> w;
    for (const char* q : {"q", "k", "v"}) {
      auto wq = I.get(p + "0.SelfAttention." + q + ".weight", {TI, D});
      w.insert(w.end(), wq.begin(), wq.end());
    }
    Bk.qkv.w = I.pack(w, 3 * TI, D, 1);
    Bk.o = I.linear(p + "0.SelfAttention.o.", D, TI, false);
    Bk.ln1 = I.upload(I.get(p + "1.layer_norm.weight", {D}));
    // gated-gelu: rows interleaved (wi_1 j, wi_0 j) so the GEMM epilogue pairs value n and gate n^1
    auto w0 = I.get(p + "1.DenseReluDense.wi_0.weight", {X.t_ff, D});
    auto w1 = I.get(p + "1.DenseReluDense.wi_1.weight", {X.t_ff, D});
    std::vector<float> wi((size_t)2 * X.t_ff * D);
    for (int j = 0; j < X.t_ff; ++j) {
      std::memcpy(&wi[(size_t)(2 * j) * D], &w1[(size_t)j * D], (size_t)D * sizeof(float));
      std::memcpy(&wi[(size_t)(2 * j + 1) * D], &w0[(size_t)j * D], (size_t)D * sizeof(float));
    }
    Bk.wi.w = I.pack(wi, 2 * X.t_ff, D, 1);
    Bk.wo = I.linear(p + "1.DenseReluDense.wo.", D, X.t_ff, false);
    X.tb.push_back(Bk);
  }
  X.t_fin = I.upload(I.get(tp + "encoder.final_layer_norm.weight", {D}));
  X.zeros = I.upload(std::vector<float>((size_t)std::max(D, H), 0.f));
}

struct TextWs {
  float *x, *tmp, *qkv, *S, *O, *inter, *e1, *g, *mean, *rstd;
  float* wi;  // T5 wi GEMM output before the gated GELU (plane path)
  u16* pl;    // operand plane of the linears' A (plane path)
  float* kp;  // K-split partial sums of the under-filled linears (alcm_opconv_args.ksplit_ws)
  int64_t kp_floats;
};
static TextWs plan_text(const TextW& X, Bump& bp, int B, int L) {
  const size_t R = (size_t)B * L;
  const int Lp = round_up(L, 8);
  const size_t dmax = (size_t)std::max({X.b_hidden, X.t_d, X.p_out});
  const size_t inner = (size_t)std::max(X.b_hidden, X.t_heads * X.t_dkv);
  TextWs w;
  w.x = bp.take<float>(R * dmax);
  w.tmp = bp.take<float>(R * dmax);
  w.qkv = bp.take<float>(R * 3 * inner);
  w.S = bp.take<float>((size_t)B * std::max(X.b_heads, X.t_heads) * L * Lp);
  w.O = bp.take<float>(R * inner);
  w.inter = bp.take<float>(R * (size_t)std::max(X.b_inter, X.t_ff));
  w.e1 = bp.take<float>(R * X.p_out);
  w.g = bp.take<float>(R * X.p_out);
  w.mean = bp.take<float>(R);
  w.rstd = bp.take<float>(R);
  w.wi = bp.take<float>(R * 2 * (size_t)X.t_ff);
  w.pl = bp.take<u16>(R * (size_t)std::max({X.b_inter, 2 * X.t_ff, (int)dmax, (int)inner}));
  w.kp_floats = (int64_t)8 * R * (int64_t)dmax;  // up to 8 parts of an R x dmax output
  w.kp = bp.take<float>((size_t)w.kp_floats);
  return w;
}

// multi-head self-attention core on a fused qkv buffer (B, L, 3I), I = nh * dh:
// O[b, t, h*dh + d] = softmax_j(scale * q_t . k_j (+ bias[h][t][j])) v_j  (no mask)
static int mha(hipStream_t s, int prec, int B, int L, int nh, int dh, const float* qkv, float scale,
               const float* bias, int bld, float* S, float* O) {
  const int I = nh * dh, Lp = round_up(L, 8);
  alcm_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.M = L; g.N = L; g.Kpad = round_up(dh, kBK); g.batch = B * nh; g.zdiv = nh;
  g.a.kind = ALCM_OPND_ACT; g.a.ptr = qkv; g.a.sb = 0; g.a.st = 3 * I; g.a.sc = 1;
  g.a.T_in = L; g.a.C_in = dh; g.a.Cpad = dh; g.a.ksize = 1; g.a.dil = 1; g.a.up = 1; g.a.rows_per_batch = L;
  g.a.zs1 = (int64_t)L * 3 * I; g.a.zs2 = dh;
  g.b = g.a;
  g.b.ptr = qkv + I;
  g.acc_scale = scale;
  g.out_scale = 1.f;
  g.out = S; g.o_sb = 0; g.o_st = Lp; g.o_sc = 1; g.o_zs1 = (int64_t)nh * L * Lp; g.o_zs2 = (int64_t)L * Lp;
  g.out_rows_per_batch = L; g.out_step = 1;
  g.prec = prec;
  ALCM_TRY(gemm(g, s));
  if (bias) ALCM_TRY(softmax_rows_bias(S, B * nh * L, L, Lp, L, nh, bias, bld, s));
  else ALCM_TRY(softmax_rows(S, B * nh * L, L, Lp, s));
  alcm_gemm_args p;
  std::memset(&p, 0, sizeof(p));
  p.M = L; p.N = dh; p.Kpad = round_up(Lp, kBK); p.batch = B * nh; p.zdiv = nh;
  p.a.kind = ALCM_OPND_ACT; p.a.ptr = S; p.a.sb = 0; p.a.st = Lp; p.a.sc = 1; p.a.T_in = L; p.a.C_in = Lp;
  p.a.Cpad = Lp; p.a.ksize = 1; p.a.dil = 1; p.a.up = 1; p.a.rows_per_batch = L;
  p.a.zs1 = (int64_t)nh * L * Lp; p.a.zs2 = (int64_t)L * Lp;
  p.b.kind = ALCM_OPND_ACT_T; p.b.ptr = qkv + 2 * I; p.b.st = 3 * I; p.b.sc = 1; p.b.T_in = L; p.b.rows = dh;
  p.b.zs1 = (int64_t)L * 3 * I; p.b.zs2 = dh;
  p.acc_scale = 1.f; p.out_scale = 1.f;
  p.out = O; p.o_sb = 0; p.o_st = I; p.o_sc = 1; p.o_zs1 = (int64_t)L * I; p.o_zs2 = dh;
  p.out_rows_per_batch = L; p.out_step = 1;
  p.prec = prec;
  return gemm(p, s);
}

// y (R, N) = x (R, C) W^T (+ bias) with the conv helper (k = 1): rows are one "batch" of R tokens
static int lin(hipStream_t s, int prec, int R, const float* x, int C, const ConvW& w, float* y, const ConvOpts& o) {
  return conv(s, prec, 1, R, View{x, 0, C, 1, R, C}, w, Out{y, 0, w.w.rows, 1, 1, 0}, o);
}

// the same linear on an F16 / BF16 operand plane (alcm_opconv, k = 1: the wide-layer / plane conv kernels): y (R, N) =
// plane (R, C) W^T (+ bias) (+ res) with out_act; the plane is written by the caller
static int plane_lin(hipStream_t s, int prec, int R, const u16* plane, int C, const ConvW& w, float* y,
                     const float* res, int act, int64_t plane_lo = 0, void* out_plane = nullptr,
                     float* kws = nullptr, int64_t kws_floats = 0) {
  if (w.w.cpad != C || w.w.taps != 1) return set_error(ALCM_E_INVALID, "plane_lin: plane width != packed Cin");
  alcm_opconv_args g;
  std::memset(&g, 0, sizeof(g));
  g.a = plane; g.a_lo_off = plane_lo; g.B = 1; g.T = R; g.C = C; g.Cp = C; g.ksize = 1; g.dil = 1; g.pad = 0;
  g.w = w.w.p; g.w_lo_off = w.w.lo; g.kpad = w.w.kpad; g.N = w.w.rows;
  g.bias = w.b; g.res = res; g.out = y; g.out_act = act; g.out_scale = 1.f; g.prec = prec;
  g.out_plane = out_plane;  // (then y == nullptr: the result as a PREC plane)
  g.ksplit_ws = kws; g.ksplit_ws_floats = kws_floats;  // K parts where the grid under-fills the chip (alcm_wconv.hip)
  return opconv(g, s);
}

static int text_encode(alcm_model* m, const int64_t* clap_ids, const int64_t* t5_ids, float* out, int B, int L,
                       void* ws, size_t wsb, hipStream_t s) {
  const TextW& X = m->text;
  if (B <= 0 || L <= 0 || L > X.max_len) return set_error(ALCM_E_INVALID, "text_encode: L must be in [1, max_len]");
  Bump bp(ws, wsb);
  TextWs w = plan_text(X, bp, B, L);
  if (!ws || bp.off > wsb) return set_error(ALCM_E_WORKSPACE, "text_encode: workspace too small");
  const int R = B * L, H = X.b_hidden, D = X.t_d, TI = X.t_heads * X.t_dkv;
  const int ps = prec_of(m, false);  // embeddings / norms / projection head: bf16x3 under every non-bf16 policy
  const int pl = prec_of(m, true);   // the encoders' linears and attention (fp16 under the mixed policy)
  // ---- CLAP text branch: BERT (post-LN), transformers BertModel with input_ids only
  ALCM_TRY(embed_gather(clap_ids, R, X.b_word, X.b_vocab, H, X.b_pos_type, L, w.x, s));
  ALCM_TRY(layer_norm(w.x, R, H, H, X.b_eps, X.b_emb_ln.g, X.b_emb_ln.b, nullptr, 0, w.x, H, s));
  const int bdh = H / X.b_heads;
  // F16 / BF16 linears (mixed / bf16 policies) on operand planes and the plane conv kernels: the fp32-A GEMM with
  // an in-kernel conversion ran the text towers at 0.05 of the MFMA peak (profiles/r3z, bench components)
  const bool planes = (pl == PREC_F16 || pl == PREC_BF16) && H % 64 == 0 && D % 64 == 0 && TI % 64 == 0 &&
                      X.b_inter % 64 == 0 && X.t_ff % 64 == 0;
  // attention of both towers in the fused kernel
  const bool tflash = planes && L <= 512 && H / X.b_heads <= 72 && X.t_dkv <= 72 &&
                      (H / X.b_heads) % 4 == 0 && X.t_dkv % 4 == 0;
  for (const BertLayerW& Ly : X.bl) {
    if (planes) {
      ALCM_TRY(to_planes(w.x, w.pl, R, H, H, pl, s));
      if (tflash) {  // q / k / v as a plane, fused attention writing the out-projection's plane (resident K / V)
        ALCM_TRY(plane_lin(s, pl, R, w.pl, H, Ly.qkv, nullptr, nullptr, 0, 0, w.qkv));
        ALCM_TRY(flash_attention(nullptr, nullptr, B, L, H, X.b_heads, pl, s, w.pl, nullptr, 0, 0.f, w.qkv));
      } else {
        ALCM_TRY(plane_lin(s, pl, R, w.pl, H, Ly.qkv, w.qkv, nullptr, 0));
        ALCM_TRY(mha(s, pl, B, L, X.b_heads, bdh, w.qkv, 1.0f / sqrtf((float)bdh), nullptr, 0, w.S, w.O));
        ALCM_TRY(to_planes(w.O, w.pl, R, H, H, pl, s));
      }
      ALCM_TRY(plane_lin(s, pl, R, w.pl, H, Ly.ao, w.tmp, w.x, 0, 0, nullptr, w.kp, w.kp_floats));
      ALCM_TRY(layer_norm_plane(w.tmp, R, H, H, X.b_eps, Ly.ln1.g, Ly.ln1.b, w.pl, pl, s));
      ALCM_TRY(layer_norm(w.tmp, R, H, H, X.b_eps, Ly.ln1.g, Ly.ln1.b, nullptr, 0, w.x, H, s));
      ALCM_TRY(plane_lin(s, pl, R, w.pl, H, Ly.inter, w.inter, nullptr, ACT_GELU_ERF));
      ALCM_TRY(to_planes(w.inter, w.pl, R, X.b_inter, X.b_inter, pl, s));
      ALCM_TRY(plane_lin(s, pl, R, w.pl, X.b_inter, Ly.out, w.tmp, w.x, 0, 0, nullptr, w.kp, w.kp_floats));
      ALCM_TRY(layer_norm(w.tmp, R, H, H, X.b_eps, Ly.ln2.g, Ly.ln2.b, nullptr, 0, w.x, H, s));
      continue;
    }
    ALCM_TRY(lin(s, pl, R, w.x, H, Ly.qkv, w.qkv, ConvOpts{}));
    ALCM_TRY(mha(s, pl, B, L, X.b_heads, bdh, w.qkv, 1.0f / sqrtf((float)bdh), nullptr, 0, w.S, w.O));
    ConvOpts ra;
    ra.res = Res{w.x, 0, H, 1};
    ALCM_TRY(lin(s, pl, R, w.O, H, Ly.ao, w.tmp, ra));
    ALCM_TRY(layer_norm(w.tmp, R, H, H, X.b_eps, Ly.ln1.g, Ly.ln1.b, nullptr, 0, w.x, H, s));
    ConvOpts gi;
    gi.act = ACT_GELU_ERF;
    ALCM_TRY(lin(s, pl, R, w.x, H, Ly.inter, w.inter, gi));
    ConvOpts ro;
    ro.res = Res{w.x, 0, H, 1};
    ALCM_TRY(lin(s, pl, R, w.inter, X.b_inter, Ly.out, w.tmp, ro));
    ALCM_TRY(layer_norm(w.tmp, R, H, H, X.b_eps, Ly.ln2.g, Ly.ln2.b, nullptr, 0, w.x, H, s));
  }
  // Projection: LayerNorm(e1 + linear2(gelu(e1))), e1 = linear1(h)  (dropout is the identity in eval)
  ALCM_TRY(lin(s, ps, R, w.x, H, X.p1, w.e1, ConvOpts{}));
  {
    ConvOpts ga;
    ga.act = ACT_GELU_ERF;
    ALCM_TRY(lin(s, ps, R, w.x, H, X.p1, w.g, ga));
    ConvOpts r2;
    r2.res = Res{w.e1, 0, X.p_out, 1};
    ALCM_TRY(lin(s, ps, R, w.g, X.p_out, X.p2, w.tmp, r2));
    ALCM_TRY(layer_norm(w.tmp, R, X.p_out, X.p_out, X.p_eps, X.p_ln.g, X.p_ln.b, nullptr, 0, w.e1, X.p_out, s));
    ALCM_HIP(hipMemcpy2DAsync(out, (size_t)2 * L * X.p_out * sizeof(float), w.e1, (size_t)L * X.p_out * sizeof(float),
                              (size_t)L * X.p_out * sizeof(float), B, hipMemcpyDeviceToDevice, s));
  }
  // ---- T5 encoder (v1.1): pre-RMSNorm blocks, unscaled attention + relative position bias, gated-gelu FFN
  ALCM_TRY(embed_gather(t5_ids, R, X.t_emb, X.t_vocab, D, nullptr, L, w.x, s));
  for (const T5BlockW& Bk : X.tb) {
    if (planes) {
      ALCM_TRY(rms_norm_plane(w.x, R, D, X.t_eps, Bk.ln0, w.pl, pl, s));
      if (tflash) {  // unscaled scores + the relative-position bias inside the fused kernel
        ALCM_TRY(plane_lin(s, pl, R, w.pl, D, Bk.qkv, nullptr, nullptr, 0, 0, w.qkv));
        ALCM_TRY(flash_attention(nullptr, nullptr, B, L, TI, X.t_heads, pl, s, w.pl, X.t_bias, X.max_len, 1.0f,
                                 w.qkv));
      } else {
        ALCM_TRY(plane_lin(s, pl, R, w.pl, D, Bk.qkv, w.qkv, nullptr, 0));
        ALCM_TRY(mha(s, pl, B, L, X.t_heads, X.t_dkv, w.qkv, 1.0f, X.t_bias, X.max_len, w.S, w.O));
        ALCM_TRY(to_planes(w.O, w.pl, R, TI, TI, pl, s));
      }
      ALCM_TRY(plane_lin(s, pl, R, w.pl, TI, Bk.o, w.x, w.x, 0, 0, nullptr, w.kp, w.kp_floats));
      ALCM_TRY(rms_norm_plane(w.x, R, D, X.t_eps, Bk.ln1, w.pl, pl, s));
      ALCM_TRY(plane_lin(s, pl, R, w.pl, D, Bk.wi, w.wi, nullptr, 0));
      if (ps == PREC_SPLIT) {
        // wo on bf16 hi / lo planes of the gated-GELU product (fp32 range, bf16x3 products; see below)
        const int64_t lo = (int64_t)R * X.t_ff;
        ALCM_TRY(geglu_split_planes(w.wi, R, X.t_ff, w.pl, lo, s));
        ALCM_TRY(plane_lin(s, PREC_SPLIT, R, w.pl, X.t_ff, Bk.wo, w.x, w.x, 0, lo));
      } else {
        ALCM_TRY(geglu_pairs(w.wi, R, X.t_ff, w.inter, s));
        ConvOpts r2;
        r2.res = Res{w.x, 0, D, 1};
        ALCM_TRY(lin(s, ps, R, w.inter, X.t_ff, Bk.wo, w.x, r2));
      }
      continue;
    }
    ALCM_TRY(rms_stats(w.x, R, D, X.t_eps, w.mean, w.rstd, s));
    ConvOpts oq;
    oq.pro = Pro{Bk.ln0, X.zeros, 0, w.mean, w.rstd, 0};
    ALCM_TRY(lin(s, pl, R, w.x, D, Bk.qkv, w.qkv, oq));
    ALCM_TRY(mha(s, pl, B, L, X.t_heads, X.t_dkv, w.qkv, 1.0f, X.t_bias, X.max_len, w.S, w.O));
    ConvOpts ro;
    ro.res = Res{w.x, 0, D, 1};
    ALCM_TRY(lin(s, pl, R, w.O, TI, Bk.o, w.x, ro));
    ALCM_TRY(rms_stats(w.x, R, D, X.t_eps, w.mean, w.rstd, s));
    ConvOpts of;
    of.pro = Pro{Bk.ln1, X.zeros, 0, w.mean, w.rstd, 0};
    of.geglu = 2;
    ALCM_TRY(conv(s, pl, 1, R, View{w.x, 0, D, 1, R, D}, Bk.wi, Out{w.inter, 0, X.t_ff, 1, 1, 0}, of));
    ConvOpts r2;
    r2.res = Res{w.x, 0, D, 1};
    // wo reads the gated-GELU product, which exceeds the fp16 range on real T5 v1.1 weights (transformers keeps
    // this layer in fp32 for that reason): bf16 hi/lo operands (fp32 range) under every non-bf16 policy
    ALCM_TRY(lin(s, ps, R, w.inter, X.t_ff, Bk.wo, w.x, r2));
  }
  return rms_norm(w.x, R, D, X.t_eps, X.t_fin, L, (int64_t)2 * L * D, out + (int64_t)L * D, s);
}

}  // namespace alcm

// ------------------------------------------------------------------ C-ABI
using namespace alcm;

extern "C" const char* alcm_last_error(void) { return g_err.c_str(); }
extern "C" int alcm_version(void) { return 1; }

extern "C" int alcm_check_device(int dev) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return set_error(ALCM_E_HIP, "hipGetDeviceProperties failed");
  if (std::string(p.gcnArchName).rfind("gfx950", 0) != 0)
    return set_error(ALCM_E_INVALID, std::string("device is ") + p.gcnArchName + ", kernels are built for gfx950");
  return 0;
}

extern "C" int alcm_model_create(int kind, const int* iconfig, int n_iconfig, const alcm_named_tensor* tensors,
                                 int n_tensors, int policy, alcm_model** out) {
  if (!out || (n_tensors > 0 && !tensors)) return set_error(ALCM_E_INVALID, "model_create: null argument");
  *out = nullptr;
  alcm_model* m = new alcm_model();
  m->kind = kind;
  if (policy < ALCM_POLICY_BF16 || policy > ALCM_POLICY_MIXED) {
    delete m;
    return set_error(ALCM_E_INVALID, "model_create: unknown precision policy");
  }
  m->policy = policy;
  m->resblock_streams = !knobs().serial_resblocks;
  try {
    Ingest I(m, tensors, n_tensors);
    if (kind == ALCM_MODEL_DIT) build_dit(I, iconfig, n_iconfig);
    else if (kind == ALCM_MODEL_VAE) build_vae(I, iconfig, n_iconfig);
    else if (kind == ALCM_MODEL_BIGVGAN) build_voc(I, iconfig, n_iconfig);
    else if (kind == ALCM_MODEL_TEXT) build_text(I, iconfig, n_iconfig);
    else if (kind == ALCM_MODEL_MEL) build_mel(I, iconfig, n_iconfig);
    else throw Error(ALCM_E_INVALID, "unknown model kind");
    if (hipDeviceSynchronize() != hipSuccess) throw Error(ALCM_E_HIP, "device sync after weight upload failed");
  } catch (const Error& e) {
    alcm_model_destroy(m);
    return set_error(e.code, e.what());
  } catch (const std::exception& e) {
    alcm_model_destroy(m);
    return set_error(ALCM_E_INVALID, e.what());
  }
  *out = m;
  return 0;
}

extern "C" int alcm_model_destroy(alcm_model* m) {
  if (!m) return 0;
  for (auto& kv : m->aux) {
    for (auto a : kv.second.s)
      if (a) (void)hipStreamDestroy(a);
    for (auto e : kv.second.ev)
      if (e) (void)hipEventDestroy(e);
  }
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
  return 0;
}

extern "C" size_t alcm_model_weight_bytes(const alcm_model* m) { return m ? m->weight_bytes : 0; }

extern "C" int alcm_model_set_split(alcm_model* m, int split) {
  if (!m) return set_error(ALCM_E_INVALID, "null model");
  m->policy = split ? ALCM_POLICY_SPLIT : ALCM_POLICY_BF16;
  return 0;
}

extern "C" int alcm_model_set_precision(alcm_model* m, int policy) {
  if (!m) return set_error(ALCM_E_INVALID, "null model");
  if (policy < ALCM_POLICY_BF16 || policy > ALCM_POLICY_MIXED) return set_error(ALCM_E_INVALID, "unknown policy");
  m->policy = policy;
  return 0;
}

extern "C" int alcm_model_set_resblock_streams(alcm_model* m, int concurrent) {
  if (!m) return set_error(ALCM_E_INVALID, "null model");
  m->resblock_streams = concurrent != 0;
  return 0;
}

extern "C" size_t alcm_dit_workspace_bytes(const alcm_model* m, int B, int T) {
  if (!m || m->kind != ALCM_MODEL_DIT) return 0;
  Bump bp(nullptr, 0);
  plan_dit(m->dit, bp, B, T);
  const size_t ctx = (size_t)2 * B * (m->dit.ctx_tokens / 2) * m->dit.hidden * sizeof(float) + 1024;
  return std::max(bp.off + 256, ctx);
}

extern "C" int alcm_dit_embed_context(alcm_model* m, const float* ctx, int B, float* cemb_cache, void* ws,
                                      size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_DIT || !ctx || !cemb_cache) return set_error(ALCM_E_INVALID, "dit_embed_context: bad args");
  return dit_embed_context(m, ctx, B, cemb_cache, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int alcm_dit_forward(alcm_model* m, const float* x, const int64_t* t, const float* cemb_cache,
                                const float* w_emb, float* eps_out, int B, int T, void* ws, size_t ws_bytes,
                                alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_DIT || !x || !t || !cemb_cache || !eps_out)
    return set_error(ALCM_E_INVALID, "dit_forward: bad args");
  return dit_forward(m, x, t, cemb_cache, w_emb, eps_out, B, T, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t alcm_vae_workspace_bytes(const alcm_model* m, int B, int T) {
  if (!m || m->kind != ALCM_MODEL_VAE) return 0;
  Bump bp(nullptr, 0);
  plan_vae(m->vae, bp, B, T);
  return bp.off + 256;
}

extern "C" int alcm_vae_decode(alcm_model* m, const float* z, float inv_scale_factor, float* mel_out, int B, int T,
                               void* ws, size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_VAE || !z || !mel_out) return set_error(ALCM_E_INVALID, "vae_decode: bad args");
  return vae_decode(m, z, inv_scale_factor, mel_out, B, T, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t alcm_bigvgan_workspace_bytes(const alcm_model* m, int B, int M) {
  if (!m || m->kind != ALCM_MODEL_BIGVGAN) return 0;
  Bump bp(nullptr, 0);
  plan_voc(m->voc, bp, B, M);
  return bp.off + 256;
}

extern "C" int alcm_bigvgan_forward(alcm_model* m, const float* mel, float* wav_out, int B, int M, void* ws,
                                    size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_BIGVGAN || !mel || !wav_out) return set_error(ALCM_E_INVALID, "bigvgan: bad args");
  return bigvgan_forward(m, mel, wav_out, B, M, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t alcm_text_workspace_bytes(const alcm_model* m, int B, int L) {
  if (!m || m->kind != ALCM_MODEL_TEXT) return 0;
  Bump bp(nullptr, 0);
  plan_text(m->text, bp, B, L);
  return bp.off + 256;
}

extern "C" int alcm_text_encode(alcm_model* m, const int64_t* clap_ids, const int64_t* t5_ids, float* out, int B,
                                int L, void* ws, size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_TEXT || !clap_ids || !t5_ids || !out)
    return set_error(ALCM_E_INVALID, "text_encode: bad args");
  if (m->text.p_out != m->text.t_d) return set_error(ALCM_E_INVALID, "text_encode: projection and T5 widths differ");
  return text_encode(m, clap_ids, t5_ids, out, B, L, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t alcm_vae_encode_workspace_bytes(const alcm_model* m, int B, int M) {
  if (!m || m->kind != ALCM_MODEL_VAE) return 0;
  Bump bp(nullptr, 0);
  plan_vae(m->vae, bp, B, M);
  return bp.off + 256;
}

extern "C" int alcm_vae_encode(alcm_model* m, const float* mel, float* moments_out, int B, int M, void* ws,
                               size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_VAE || !mel || !moments_out) return set_error(ALCM_E_INVALID, "vae_encode: bad args");
  return vae_encode(m, mel, moments_out, B, M, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int alcm_vae_encode_len(const alcm_model* m, int M) {
  if (!m || m->kind != ALCM_MODEL_VAE) return -1;
  int T = M;
  for (const auto& d : m->vae.enc.down)
    if (d.w.p) T = (T - 2) / 2 + 1;
  return T;
}

extern "C" size_t alcm_mel_workspace_bytes(const alcm_model* m, int B, int L) {
  if (!m || m->kind != ALCM_MODEL_MEL) return 0;
  Bump bp(nullptr, 0);
  plan_mel(m->mel, bp, B, L);
  return bp.off + 256;
}

extern "C" int alcm_mel_spectrogram(alcm_model* m, const float* wav, float* mel_out, int B, int L, void* ws,
                                    size_t ws_bytes, alcm_stream_t stream) {
  if (!m || m->kind != ALCM_MODEL_MEL || !wav || !mel_out) return set_error(ALCM_E_INVALID, "mel: bad args");
  return mel_forward(m, wav, mel_out, B, L, ws, ws_bytes, (hipStream_t)stream);
}
