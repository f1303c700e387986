// In-step launch profiler (dn_profile_ops / dn_profile_ops_read): while enabled, every launch
// site of the U-Net executors and the step's elementwise entry points records a pair of HIP
// events on the stream it launches on, with the op, its shape and its algorithmic FLOPs, and the
// executors run single-stream so the event pairs bracket one kernel each.  bench.py reads the
// records of one profiled step to report the step's own per-shape roofline.
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "denoise_hip.h"
#include "dn_internal.h"

namespace dn {

namespace {
struct Rec {
  char op[24];
  char kernel[48];
  int K, NOUT, H, W, N;
  double flops;
  hipEvent_t a, b;
};
std::mutex g_mu;
std::vector<Rec> g_recs;
bool g_on = false;
thread_local char g_kernel[48] = "";  // copied: callers may pass a temporary's c_str()
}  // namespace

bool prof_on() { return g_on; }

void prof_kernel(const char* k) {
  if (g_on) std::snprintf(g_kernel, sizeof g_kernel, "%s", k ? k : "");
}

OpTimer::OpTimer(hipStream_t st, const char* op, double flops, int K, int NOUT, int H, int W,
                 int N) {
  if (!g_on) return;
  Rec r{};
  std::snprintf(r.op, sizeof r.op, "%s", op);
  r.K = K; r.NOUT = NOUT; r.H = H; r.W = W; r.N = N; r.flops = flops;
  if (hipEventCreate(&r.a) != hipSuccess) return;
  if (hipEventCreate(&r.b) != hipSuccess) { (void)hipEventDestroy(r.a); return; }
  if (hipEventRecord(r.a, st) != hipSuccess) {
    (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b);
    return;
  }
  g_kernel[0] = '\0';
  std::lock_guard<std::mutex> lock(g_mu);
  idx = (int)g_recs.size();
  s = st;
  g_recs.push_back(r);
}

OpTimer::~OpTimer() {
  if (idx < 0) return;
  std::lock_guard<std::mutex> lock(g_mu);
  if (idx >= (int)g_recs.size()) return;  // cleared meanwhile
  Rec& r = g_recs[idx];
  std::snprintf(r.kernel, sizeof r.kernel, "%s", g_kernel);
  (void)hipEventRecord(r.b, s);
}

static void clear_locked() {
  for (Rec& r : g_recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_recs.clear();
}

}  // namespace dn

extern "C" {

dn_status dn_profile_ops(int enable) {
  std::lock_guard<std::mutex> lock(dn::g_mu);
  dn::clear_locked();
  dn::g_on = enable != 0;
  return DN_OK;
}

dn_status dn_profile_ops_read(dn_op_record* out, int cap, int* count) {
  if (!count || (cap > 0 && !out)) return DN_ERR_ARG;
  std::lock_guard<std::mutex> lock(dn::g_mu);
  int n = 0;
  dn_status st = DN_OK;
  for (const dn::Rec& r : dn::g_recs) {
    if (hipEventSynchronize(r.b) != hipSuccess) { st = DN_ERR_HIP; break; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) { st = DN_ERR_HIP; break; }
    if (n < cap) {
      dn_op_record& o = out[n];
      std::memset(&o, 0, sizeof o);
      std::snprintf(o.op, sizeof o.op, "%s", r.op);
      std::snprintf(o.kernel, sizeof o.kernel, "%s", r.kernel);
      o.K = r.K; o.NOUT = r.NOUT; o.H = r.H; o.W = r.W; o.N = r.N;
      o.flops = r.flops;
      o.ms = ms;
    }
    ++n;
  }
  *count = n;
  dn::clear_locked();
  return st;
}

}  // extern "C"
