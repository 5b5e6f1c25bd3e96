// Host-side pieces of libtgnx: error state, version, and the native single-pass
// dependency-block assignment (dependencyGraph.py:8-49).
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/tgnx.h"

namespace tgnx {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tgnx

namespace tgnx {
// ------------------------------------------------------------------ kernel probe
// Each probed region records a marker-event pair around it (probe_begin / probe_end: includes the launch's
// dispatch); the region's first launch through launch_k (tgnx_common.h) also binds a second pair to the
// kernel itself (hipExtLaunchKernelGGL start / stop events: the dispatch packet's begin / end timestamps,
// the duration rocprofv3 --kernel-trace reports).  tgnx_probe_read prefers the kernel-bound pair.
struct Probe {
  int id = 0;
  std::vector<hipEvent_t> ev;  // per record: marker start, marker stop, kernel start, kernel stop
  std::vector<char> bound;     // per record: the kernel pair was bound
  size_t used = 0;             // records
  bool open = false;           // a region is open (between probe_begin and probe_end)
  bool armed = false;          // ... and its kernel pair is still unbound
};
static Probe g_probe;

static bool probe_grow() {
  if ((g_probe.used + 1) * 4 <= g_probe.ev.size()) return true;
  const size_t n = std::max<size_t>(2048, g_probe.ev.size() * 2);
  while (g_probe.ev.size() < n) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return false;
    g_probe.ev.push_back(e);
  }
  g_probe.bound.resize(n / 4, 0);
  return true;
}
void probe_begin(int id, hipStream_t s) {
  if (g_probe.id != id || !probe_grow()) return;
  g_probe.open = g_probe.armed = true;
  g_probe.bound[g_probe.used] = 0;
  (void)hipEventRecord(g_probe.ev[4 * g_probe.used], s);
}
bool probe_take(hipEvent_t* k0, hipEvent_t* k1) {
  if (!g_probe.armed) return false;
  g_probe.armed = false;
  g_probe.bound[g_probe.used] = 1;
  *k0 = g_probe.ev[4 * g_probe.used + 2];
  *k1 = g_probe.ev[4 * g_probe.used + 3];
  return true;
}
void probe_end(int id, hipStream_t s) {
  if (g_probe.id != id || !g_probe.open) return;
  (void)hipEventRecord(g_probe.ev[4 * g_probe.used + 1], s);
  g_probe.open = g_probe.armed = false;
  g_probe.used += 1;
}
}  // namespace tgnx

extern "C" {

int tgnx_probe_enable(int32_t kernel_id) {
  tgnx::g_probe.id = kernel_id;
  tgnx::g_probe.used = 0;
  tgnx::g_probe.open = tgnx::g_probe.armed = false;
  return TGNX_OK;
}

int tgnx_probe_read(double* total_ms, int64_t* launches) {
  double ms = 0.0;
  for (size_t i = 0; i < tgnx::g_probe.used; ++i) {
    const bool k = tgnx::g_probe.bound[i] != 0;
    hipEvent_t a = tgnx::g_probe.ev[4 * i + (k ? 2 : 0)], b = tgnx::g_probe.ev[4 * i + (k ? 3 : 1)];
    if (hipEventSynchronize(tgnx::g_probe.ev[4 * i + 1]) != hipSuccess) {
      tgnx::set_error("tgnx_probe_read: event sync failed");
      return TGNX_EHIP;
    }
    float f = 0.f;
    (void)hipEventElapsedTime(&f, a, b);
    ms += f;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = (int64_t)tgnx::g_probe.used;
  tgnx::g_probe.used = 0;
  return TGNX_OK;
}

int tgnx_version(void) { return 1; }

const char* tgnx_last_error(void) { return tgnx::g_err; }

// get_block (dependencyGraph.py:8-28) over consecutive batches (dependecyAwareBatch, :33-49).
// The per-batch dict of the reference becomes a node-indexed array stamped with the batch
// number, so no clearing is needed between batches: O(E) total, ~ns per event.
int tgnx_block_ids_host(const int64_t* src, const int64_t* dst, int64_t num_events, int64_t batch, int64_t* out) {
  if (!src || !dst || !out || num_events < 0 || batch <= 0) {
    tgnx::set_error("tgnx_block_ids_host: bad arguments");
    return TGNX_EINVAL;
  }
  int64_t maxv = -1;
  for (int64_t i = 0; i < num_events; ++i) {
    if (src[i] < 0 || dst[i] < 0) {
      tgnx::set_error("tgnx_block_ids_host: negative node id at %lld", (long long)i);
      return TGNX_EINVAL;
    }
    maxv = std::max(maxv, std::max(src[i], dst[i]));
  }
  std::vector<int64_t> last((size_t)(maxv + 1), -1);
  std::vector<int64_t> stamp((size_t)(maxv + 1), -1);
  for (int64_t b0 = 0, bn = 0; b0 < num_events; b0 += batch, ++bn) {
    int64_t b1 = std::min(num_events, b0 + batch);
    for (int64_t i = b0; i < b1; ++i) {
      int64_t a = src[i], c = dst[i];
      int64_t la = stamp[a] == bn ? last[a] : -1;
      int64_t lc = stamp[c] == bn ? last[c] : -1;
      int64_t blk = std::max(la, lc) + 1;
      last[a] = blk;
      stamp[a] = bn;
      last[c] = blk;
      stamp[c] = bn;
      out[i] = blk;
    }
  }
  return TGNX_OK;
}

}  // extern "C"
