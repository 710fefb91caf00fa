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
  k.wconv3 = env_int("ALCM_WCONV3", -1);
  k.wconv3_grid = env_int("ALCM_WCONV3_GRID", 0);
  k.nconv = env_int("ALCM_NCONV", -1);
  k.opconv_tile = env_int("ALCM_OPCONV_TILE", 0);
  k.serial_resblocks = env_set("ALCM_SERIAL_RESBLOCKS");
  k.prof_shapes = env_set("ALCM_PROF_SHAPES");
  k.tconv = env_int("ALCM_TCONV", 1);
  k.lin1 = env_int("ALCM_LIN1", -1);
  k.tconv_ablate = env_int("ALCM_TCONV_ABLATE", 0);
  k.tconv_trace = env_int("ALCM_TCONV_TRACE", 0) != 0;
  k.act_mfma = env_int("ALCM_ACT_MFMA", 1);
  k.act_defer = env_int("ALCM_ACT_DEFER", 1);
  k.xp[0] = env_int("ALCM_XP0", 0);
  k.xp[1] = env_int("ALCM_XP1", 0);
  k.xp[2] = env_int("ALCM_XP2", 0);
  k.xp[3] = env_int("ALCM_XP3", 0);
  k.conv1_h16 = env_int("ALCM_CONV1_H16", 1);
  k.ksplit = env_int("ALCM_KSPLIT", 1);
  k.act_x3_mfma = env_int("ALCM_ACT_X3_MFMA", 1);
  k.wconv_sum = env_int("ALCM_WCONV_SUM", 1);
  k.gemm_skinny = env_int("ALCM_GEMM_SKINNY", 1);
  k.ups_t160 = env_int("ALCM_UPS_T160", 1);
  k.nct_cl = env_int("ALCM_NCT_CL", 1);
  return k;
}

static Knobs g_knobs = read_knobs();

const Knobs& knobs() { return g_knobs; }

}  // namespace alcm

extern "C" int alcm_reload_knobs(void) {
  alcm::g_knobs = alcm::read_knobs();
  return 0;
}
