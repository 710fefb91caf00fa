// Diagnostic / A-B switches (ALCM_* environment variables), read once when the library is loaded and
// again only on alcm_reload_knobs(): no launch path calls getenv.
#include <cstdlib>

#include "alcm_internal.h"

namespace alcm {

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}
static bool env_set(const char* name) {
  const char* v = std::getenv(name);
  return v && *v;
}

static Knobs read_knobs() {
  Knobs k;
  k.wconv = env_int("ALCM_WCONV", 8);
  k.wconv_order = env_int("ALCM_WCONV_ORDER", -1);
  k.wconv_tile = env_int("ALCM_WCONV_TILE", -1);
  k.wconv3 = env_int("ALCM_WCONV3", -1);
  k.wconv3_grid = env_int("ALCM_WCONV3_GRID", 0);
  k.nconv = env_int("ALCM_NCONV", -1);
  k.nconv_nb = env_int("ALCM_NCONV_NB", 0);
  k.act_rows = env_int("ALCM_ACT_ROWS", 8) == 16 ? 16 : 8;
  k.act_v1 = env_set("ALCM_ACT_V1");
  k.act_np = env_int("ALCM_ACT_NP", 0);
  k.ups_fp32 = env_set("ALCM_UPS_FP32");
  k.opconv_tile = env_int("ALCM_OPCONV_TILE", 0);
  k.no_act_fusion = env_set("ALCM_NO_ACT_FUSION");
  k.no_flash = env_set("ALCM_NO_FLASH");
  k.attn_tiled = env_set("ALCM_ATTN_TILED");
  k.no_attn_planes = env_set("ALCM_NO_ATTN_PLANES");
  k.no_ffn_planes = env_set("ALCM_NO_FFN_PLANES");
  k.no_vae_planes = env_set("ALCM_NO_VAE_PLANES");
  k.tail_f16w2_all = env_set("ALCM_TAIL_F16W2_ALL");
  k.serial_resblocks = env_set("ALCM_SERIAL_RESBLOCKS");
  k.prof_shapes = env_set("ALCM_PROF_SHAPES");
  k.tail_prefetch = env_int("ALCM_TAIL_PREFETCH", 1);
  k.opconv_ablate = env_int("ALCM_OPCONV_ABLATE", 0);
  k.tconv = env_int("ALCM_TCONV", 1);
  k.tconv_wgs = env_int("ALCM_TCONV_WGS", 0);
  k.tconv_bm = env_int("ALCM_TCONV_BM", 256);
  k.tconv_stagger = env_int("ALCM_TCONV_STAGGER", -1);
  k.post_planes = env_set("ALCM_POST_PLANES");
  k.sgemm = env_int("ALCM_SGEMM", 1);
  k.lin1 = env_int("ALCM_LIN1", -1);
  k.ups2 = env_int("ALCM_UPS2", 1);
  k.act3 = env_int("ALCM_ACT3", 1);
  k.text_flash = env_int("ALCM_TEXT_FLASH", 1);
  k.qkv_plane = env_int("ALCM_QKV_PLANE", 1);
  k.tconv_ablate = env_int("ALCM_TCONV_ABLATE", 0);
  k.act_mfma = env_int("ALCM_ACT_MFMA", 1);
  k.act_defer = env_int("ALCM_ACT_DEFER", 1);
  k.xp[0] = env_int("ALCM_XP0", 0);
  k.xp[1] = env_int("ALCM_XP1", 0);
  k.xp[2] = env_int("ALCM_XP2", 0);
  k.xp[3] = env_int("ALCM_XP3", 0);
  k.conv1_h16 = env_int("ALCM_CONV1_H16", 1);
  return k;
}

static Knobs g_knobs = read_knobs();

const Knobs& knobs() { return g_knobs; }

}  // namespace alcm

extern "C" int alcm_reload_knobs(void) {
  alcm::g_knobs = alcm::read_knobs();
  return 0;
}
