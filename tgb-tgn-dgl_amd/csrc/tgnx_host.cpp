// Host-side pieces of libtgnx: error state, version, and the native single-pass
// dependency-block assignment (dependencyGraph.py:8-49).
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

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

extern "C" {

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
