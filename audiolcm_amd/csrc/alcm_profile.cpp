// Live per-kernel timing with HIP events (bench.py's roofline numbers).
//
// While enabled, every launch site brackets its kernel with two hipEvents on the launch stream
// and records the kernel's ALGORITHMIC flops and bytes; alcm_profile_end synchronises the events
// and returns per-kernel aggregates (launch count, summed event time, summed flops/bytes).  Kernel
// keys use the demangled names rocprofv3 prints, so the two can be compared directly.
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "alcm_internal.h"

namespace alcm {

struct ProfRec {
  std::string name;
  double flops, bytes;
  hipEvent_t e0, e1;
};
static bool g_on = false;
static double g_pf = 2.5e15, g_pb = 8.0e12;
static std::vector<ProfRec> g_recs;
static std::vector<hipEvent_t> g_pool;
static std::mutex g_mu;  // launches may come from several host threads while profiling

static hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

bool prof_enabled() { return g_on; }

void* prof_start(hipStream_t s) {
  if (!g_on) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e = take_event();
  (void)hipEventRecord(e, s);
  return (void*)e;
}

void prof_stop(void* tok, hipStream_t s, const std::string& name, double flops, double bytes) {
  if (!g_on || !tok) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e1 = take_event();
  (void)hipEventRecord(e1, s);
  g_recs.push_back(ProfRec{name, flops, bytes, (hipEvent_t)tok, e1});
}

}  // namespace alcm

using namespace alcm;

extern "C" int alcm_profile_begin(double peak_flops, double peak_bytes_per_s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (peak_flops > 0) g_pf = peak_flops;
  if (peak_bytes_per_s > 0) g_pb = peak_bytes_per_s;
  for (auto& r : g_recs) {
    g_pool.push_back(r.e0);
    g_pool.push_back(r.e1);
  }
  g_recs.clear();
  g_on = true;
  return 0;
}

extern "C" int alcm_profile_end(alcm_prof_entry* out, int max_entries, int* n_entries) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  struct Agg {
    int64_t n = 0;
    double ms = 0, flops = 0, bytes = 0, roof = 0;
    int64_t hn = 0;
    double hms = 0, hbytes = 0;
  };
  std::map<std::string, Agg> agg;
  for (auto& r : g_recs) {
    if (hipEventSynchronize(r.e1) != hipSuccess) return set_error(ALCM_E_HIP, "profile: event sync failed");
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.e0, r.e1) != hipSuccess) return set_error(ALCM_E_HIP, "profile: elapsed failed");
    Agg& a = agg[r.name];
    a.n += 1;
    a.ms += ms;
    a.flops += r.flops;
    a.bytes += r.bytes;
    a.roof += 1e3 * std::max(r.flops / g_pf, r.bytes / g_pb);
    if (r.flops * g_pb < r.bytes * g_pf) {  // HBM-bound by its algorithmic intensity
      a.hn += 1;
      a.hms += ms;
      a.hbytes += r.bytes;
    }
  }
  int i = 0;
  for (auto& kv : agg) {
    if (out && i < max_entries) {
      std::snprintf(out[i].name, sizeof(out[i].name), "%s", kv.first.c_str());
      out[i].launches = kv.second.n;
      out[i].total_ms = kv.second.ms;
      out[i].flops = kv.second.flops;
      out[i].bytes = kv.second.bytes;
      out[i].roof_ms = kv.second.roof;
      out[i].hbm_launches = kv.second.hn;
      out[i].hbm_ms = kv.second.hms;
      out[i].hbm_bytes = kv.second.hbytes;
    }
    ++i;
  }
  if (n_entries) *n_entries = i;
  for (auto& r : g_recs) {
    g_pool.push_back(r.e0);
    g_pool.push_back(r.e1);
  }
  g_recs.clear();
  return 0;
}
