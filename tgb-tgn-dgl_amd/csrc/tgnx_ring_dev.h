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

// `smem` must hold next_pow2(2B)*8 + 2B*4 bytes, `sh` >= 20 ints; called by a whole workgroup.
__device__ __forceinline__ void ring_insert_block(int64_t* __restrict__ nbr, int64_t* __restrict__ eid,
                                                  float* __restrict__ rt, int K, const int64_t* __restrict__ src,
                                                  const int64_t* __restrict__ dst, const float* __restrict__ ev_t,
                                                  int B, int64_t cur, int64_t* __restrict__ assoc,
                                                  unsigned char* smem, int* sh) {
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
  bitonic_sort_u64(key, n);
  // run starts -> run ids
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
  for (int r = threadIdx.x; r < U; r += T) {
    int a = run_start[r];
    int c = (r + 1 < U ? run_start[r + 1] : n2) - a;
    int64_t v = (int64_t)(key[a] >> 32);
    assoc[v] = r;
    int m = c < K ? c : K;
    // new entries (newest first), canonical K newest when c > K
    int64_t ne[KMAX], nn[KMAX];
    float nt[KMAX];
    for (int j = 0; j < m; ++j) {
      uint64_t kk = key[a + j];
      int i = B - 1 - (int)((kk & 0xFFFFFFFFull) >> 1);
      int dir = (int)(kk & 1ull);
      ne[j] = cur + i;
      nn[j] = dir == 0 ? src[i] : dst[i];
      nt[j] = ev_t[i];
    }
    // old row
    int64_t oe[KMAX], on[KMAX];
    float ot[KMAX];
    int64_t* er = eid + v * K;
    int64_t* nr = nbr + v * K;
    float* tr = rt + v * K;
    for (int j = 0; j < K; ++j) {
      oe[j] = er[j];
      on[j] = nr[j];
      ot[j] = tr[j];
    }
    // e_id top-K of [old | dense] (dense = m new + (K-m) empty), neighbours follow e_id
    int io = 0, in = 0;
    for (int s = 0; s < K; ++s) {
      int64_t eo = io < K ? oe[io] : -1;
      int64_t en = in < m ? ne[in] : -1;
      if (en > eo) {
        er[s] = en;
        nr[s] = nn[in];
        ++in;
      } else {
        er[s] = eo;
        nr[s] = eo >= 0 ? on[io] : -1;
        ++io;
      }
    }
    // t top-K of [old t | new t + (-1) padding] (neighbor_loader.py:100: independent of e_id)
    for (int x = 1; x < m; ++x) {  // sort new t descending (m <= K)
      float y = nt[x];
      int z = x - 1;
      while (z >= 0 && nt[z] < y) {
        nt[z + 1] = nt[z];
        --z;
      }
      nt[z + 1] = y;
    }
    io = 0;
    in = 0;
    for (int s = 0; s < K; ++s) {
      float to = io < K ? ot[io] : -1.0f;
      float tn = in < m ? nt[in] : -1.0f;
      if (tn > to) {
        tr[s] = tn;
        ++in;
      } else {
        tr[s] = to;
        ++io;
      }
    }
  }
  __syncthreads();
}

__host__ __device__ __forceinline__ size_t ring_insert_smem_bytes(int B) {
  return (size_t)next_pow2(2 * B) * 8 + (size_t)2 * B * 4;
}

}  // namespace tgnx
