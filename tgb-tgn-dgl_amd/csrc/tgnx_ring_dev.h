// Device-side ring insert shared by tgnx_ring_insert and the fused TGNN step.
// Reference: neighbor_loader.py:52-104.
#pragma once
#include "tgnx_common.h"

namespace tgnx {

constexpr int KMAX = 32;  // ring width supported by the insert merge (config uses 10)
constexpr int INSERT_MAX_B = 4096;

// ------------------------------------------------------------------ insert
// One workgroup.  Entry i < B: (node dst_i, nbr src_i), entry B+i: (node src_i, nbr dst_i),
// both with e_id = cur + i.  Key = node << 32 | (B-1-i) << 1 | dir sorts node-ascending,
// newest-first; runs of one node are merged with that node's ring row.

// Insert plan of one batch (LastNeighborLoader.insert, neighbor_loader.py:52-104): the 2B entries
// (node << 32 | (B-1-i) << 1 | dir; dir 0 = dst side holding src, 1 = src side holding dst) sorted
// in LDS so each node's run lists its new entries newest first; run_start[r] = first entry of run r.
// Returns the number of runs.  Needs the whole workgroup.
struct NoCheckpoint {
  __device__ void operator()(int) const {}
};
// big_tmp: the LDS past the run starts holds next_pow2(2B) more keys (the scan launch, the standalone
// insert): the register sort then also serves 1024 < 2B <= 4096
template <class AT = NoCheckpoint>
__device__ __forceinline__ int ring_plan_block(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int B,
                                               unsigned char* smem, int* sh, uint64_t** key_out, int** runs_out,
                                               AT at = AT{}, bool big_tmp = false) {
  const int n2 = 2 * B;
  const int n = next_pow2(n2);
  uint64_t* key = reinterpret_cast<uint64_t*>(smem);
  int* run_start = reinterpret_cast<int*>(smem + (size_t)n * 8);
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    uint64_t k = ~0ull;
    if (p < n2) {
      int i = p < B ? p : p - B;
      int dir = p < B ? 0 : 1;
      uint64_t node = (uint64_t)(dir == 0 ? dst[i] : src[i]);
      k = (node << 32) | ((uint64_t)(B - 1 - i) << 1) | (uint64_t)dir;
    }
    key[p] = k;
  }
  __syncthreads();
  at(0);
  sort_u64(key, reinterpret_cast<uint64_t*>(run_start + n2 + (n2 & 1)), n2, n, true, big_tmp);  // keys distinct: (node, i, dir)
  at(1);
  const int T = blockDim.x;
  int pc = (n2 + T - 1) / T;
  int p0 = threadIdx.x * pc, p1 = min(n2, p0 + pc);
  int cnt = 0;
  for (int p = p0; p < p1; ++p) cnt += (p == 0 || (key[p] >> 32) != (key[p - 1] >> 32));
  int U;
  int rid = block_excl_scan(cnt, sh, &U);
  for (int p = p0; p < p1; ++p)
    if (p == 0 || (key[p] >> 32) != (key[p - 1] >> 32)) run_start[rid++] = p;
  __syncthreads();
  *key_out = key;
  *runs_out = run_start;
  return U;
}

// Merge of run r (entries key[a, a+cnt), one node) into the node's ring, by one wave: lanes [0,K)
// hold the old slots, lanes [K, K+m) the m = min(cnt, K) newest new entries; each candidate's slot
// is its rank by e_id (desc) and, separately, by t (desc) — top-K of [old | dense] exactly as
// neighbor_loader.py:91-104.  `key` may live in LDS or global memory.
__device__ __forceinline__ void ring_merge_run(int64_t* __restrict__ nbr, int64_t* __restrict__ eid,
                                               float* __restrict__ rt, int K, const int64_t* __restrict__ src,
                                               const int64_t* __restrict__ dst, const float* __restrict__ ev_t, int B,
                                               int64_t cur, int64_t* __restrict__ assoc, const uint64_t* key, int a,
                                               int cnt, int r, int lane) {
  const int64_t v = (int64_t)(key[a] >> 32);
  if (lane == 0) assoc[v] = r;
  const int m = cnt < K ? cnt : K;
  int64_t* er = eid + v * K;
  int64_t* nr = nbr + v * K;
  float* tr = rt + v * K;
  int64_t ce = INT64_MIN, cn = -1;
  float ct = -INFINITY;
  const bool cand = lane < K + m;
  if (lane < K) {
    ce = er[lane];
    cn = nr[lane];
    ct = tr[lane];
  } else if (cand) {
    const uint64_t kk = key[a + lane - K];
    const int i = B - 1 - (int)((kk & 0xFFFFFFFFull) >> 1);
    ce = cur + i;
    cn = (kk & 1ull) == 0 ? src[i] : dst[i];
    ct = ev_t[i];
  }
  int re = 0, rtk = 0;
  for (int j = 0; j < K + m; ++j) {
    const int64_t oe = (int64_t)(((uint64_t)(uint32_t)lane_i((int)(ce >> 32), j) << 32) |
                                 (uint64_t)(uint32_t)lane_i((int)ce, j));   // j uniform: readlane
    const float ot = lane_f(ct, j);
    re += (oe > ce) || (oe == ce && j < lane);
    rtk += (ot > ct) || (ot == ct && j < lane);
  }
  if (cand && re < K) {
    er[re] = ce;
    nr[re] = ce >= 0 ? cn : -1;
  }
  if (cand && rtk < K) tr[rtk] = ct;
}

// Whole insert in one workgroup (the standalone tgnx_ring_insert): plan, then a wave per run.
__device__ __forceinline__ void ring_insert_block(int64_t* __restrict__ nbr, int64_t* __restrict__ eid,
                                                  float* __restrict__ rt, int K, const int64_t* __restrict__ src,
                                                  const int64_t* __restrict__ dst, const float* __restrict__ ev_t,
                                                  int B, int64_t cur, int64_t* __restrict__ assoc,
                                                  unsigned char* smem, int* sh) {
  uint64_t* key;
  int* run_start;
  const int U = ring_plan_block(src, dst, B, smem, sh, &key, &run_start, NoCheckpoint{}, true);
  const int n2 = 2 * B;
  const int lane = threadIdx.x & 63, nwv = blockDim.x >> 6;
  for (int r = threadIdx.x >> 6; r < U; r += nwv) {
    const int a = run_start[r];
    const int cnt = (r + 1 < U ? run_start[r + 1] : n2) - a;
    ring_merge_run(nbr, eid, rt, K, src, dst, ev_t, B, cur, assoc, key, a, cnt, r, lane);
  }
  __syncthreads();
}

__host__ __device__ __forceinline__ size_t ring_insert_smem_bytes(int B) {
  // keys + run starts (+ register-sort ping-pong buffer for next_pow2(2B) <= 4096)
  const int n = next_pow2(2 * B);
  return (size_t)n * 8 + (size_t)(2 * B + 2) * 4 + (n <= 4096 ? (size_t)n * 8 : 0);
}

}  // namespace tgnx
