// Fused TGNN train / eval step on gfx950 — the running reference path:
//   epoch_utils.py:15-318 (batch assembly, loss, insert), model_utils.py:61-159 (block loop),
//   :201-237 (TimeEncode), :422-455 (TemporalEdgePreprocess), :565-612 (EdgeGATConv),
//   :688-697 (TemporalTransformerConv), :165-195 (EdgePredictor), :709-710 (Adam).
//
// Design:
//  * No DGL graph, no unique/relabel: a "segment" is one predictor row (s / p / n of an
//    event).  Its in-edges in the reference's block-i subgraph are exactly: the root's ring
//    row (sampled before the batch), its self-loop (ones features, t = 0) and one edge per
//    earlier-block event the root took part in as src or dst (model_utils.py:151-157).
//  * time_assoc as of block i (model_utils.py:77-83) is rebuilt per source node from the
//    batch's touch list, sorted by (node, block, kind, event) in one workgroup.
//  * EdgeGATConv collapsed exactly: el/er/ee only enter through head dots, so
//    x_eh = U_e[h]·efeat_e + U_l[h]·nfeat_src + c, U = attn·W (a 372-wide dot per edge
//    per head instead of an 800-wide GEMM row); backward re-expands dU into dW / dattn.
//  * One wave (64 lanes) per segment, lanes over feature dims; online softmax per head.
#include <rocprim/block/block_radix_sort.hpp>
#include "tgnx_math.h"
#include "tgnx_ring_dev.h"

namespace tgnx {

void probe_begin(int id, hipStream_t s);
void probe_end(int id, hipStream_t s);

constexpr int H = 8;          // gnn.att_head
constexpr int DMAX = 128;     // gnn.dim_out (memory/time/embedding dim) capacity
constexpr int FMAX = 320;     // d + D capacity
constexpr int TOUCH_MAX = 8192;
#ifndef TGNX_GBWD
#define TGNX_GBWD 256  // one workgroup per CU; 128 / 192: B = 200 0.0915 / 0.0880 vs 0.0866 ms, B = 2,000 1.263 / 1.045 vs 0.937 (r6au_*)
#endif
#ifndef TGNX_BWD_WAVES
#define TGNX_BWD_WAVES 8  // waves per edge-backward workgroup below TGNX_BIG_BATCH events (12 at and above)
#endif
constexpr int GBWD = TGNX_GBWD;            // workgroups of the edge backward kernel (= partial slabs)
constexpr int BWD_WAVES = TGNX_BWD_WAVES;  // waves per edge backward workgroup (small batches)
#ifndef TGNX_BIG_BATCH
#define TGNX_BIG_BATCH 1000  // batch capacity from which the TGNN step takes its large-batch forms (below)
#endif
// LDS partial rows of the edge backward (16 KB each at the wiki shape): waves past the 8th add theirs into row
// wv - 8 after the first 8 stored (fixed order), so 12 waves (3 per SIMD at 144 VGPRs) fit one CU's LDS.  12 waves:
// TGN.yml's B = 2,000 step 1.117 -> 1.061 ms, B = 200 0.0918 -> 0.0927 (profiles/r6/r6ab_*): 12 from
// TGNX_BIG_BATCH events of capacity up
__host__ __device__ constexpr int bwd_bufs(int nw) { return nw < 8 ? nw : 8; }
constexpr int GSEG = 160;     // workgroups of the segment backward kernel (= segment slabs)
constexpr int GSEG_BIG = 1024;  // ... from TGNX_BIG_BATCH events of capacity (6,000 segments at B = 2,000: 160 took
                                // 132 us, 640 waves each walking ~9 segments)
__host__ __device__ inline int gseg_for(int Bmax) { return Bmax >= TGNX_BIG_BATCH ? GSEG_BIG : GSEG; }
constexpr int MRR_SLOTS = 65536;  // per-batch MRR ring in buffers.mrr
constexpr int BATCH_MAX = 2048;   // max events per batch (touch sort capacity 3 * BATCH_MAX in LDS)
enum { MISC_RUNS = 0, MISC_KMAX = 1, MISC_STAMPS = 16, MISC_WORDS = TGNX_MISC_WORDS };
#ifdef TGNX_TIMING  // phase timestamps of the single-workgroup kernels (measurement builds only)
#define TGNN_PHASE_STAMP(c, i) \
  do { if (threadIdx.x == 0) reinterpret_cast<int64_t*>((c).misc + MISC_STAMPS)[i] = (int64_t)wall_clock64(); } while (0)
#else
#define TGNN_PHASE_STAMP(c, i) do {} while (0)
#endif

// ------------------------------------------------------------------ layouts
struct Lay {
  int64_t te_w, te_b, attn_l, attn_r, attn_e, Wn, bn, We, be, Ws, bs, Wd, bd, Wo, bo, total;
};
__host__ __device__ inline int64_t al4(int64_t x) { return (x + 3) & ~int64_t(3); }
static Lay make_lay(int D, int d) {
  const int64_t F = d + D;
  Lay L;
  int64_t o = 0;
  L.te_w = o; o += al4(D);
  L.te_b = o; o += al4(D);
  L.attn_l = o; o += al4(H * D);
  L.attn_r = o; o += al4(H * D);
  L.attn_e = o; o += al4(H * D);
  L.Wn = o; o += al4((int64_t)H * D * D);
  L.bn = o; o += al4(H * D);
  L.We = o; o += al4((int64_t)H * D * F);
  L.be = o; o += al4(H * D);
  L.Ws = o; o += al4((int64_t)D * D);
  L.bs = o; o += al4(D);
  L.Wd = o; o += al4((int64_t)D * D);
  L.bd = o; o += al4(D);
  L.Wo = o; o += al4(D);
  L.bo = o; o += al4(1);
  L.total = o;
  return L;
}
// derived per step from the params (collapse kernel)
struct ULay {
  int64_t Ue, Ul, Ur, ce, cl, cr, WsT, WdT, Ws1, Wd1, ones, total;
};
static ULay make_ulay(int D, int d) {
  const int64_t F = d + D;
  ULay U;
  int64_t o = 0;
  U.Ue = o; o += al4(H * F);
  U.Ul = o; o += al4(H * D);
  U.Ur = o; o += al4(H * D);
  U.ce = o; o += al4(H);
  U.cl = o; o += al4(H);
  U.cr = o; o += al4(H);
  U.WsT = o; o += al4((int64_t)D * D);
  U.WdT = o; o += al4((int64_t)D * D);
  U.Ws1 = o; o += al4(D);
  U.Wd1 = o; o += al4(D);
  U.ones = o; o += al4(FMAX);  // feature row of self loops (all ones), so gathers need no branch
  U.total = o;
  return U;
}
// backward partial slab: dUe[H*F] dUl[H*D] dUr[H*D] dce[H] dcl[H] dcr[H] dw[D] db[D]
struct PLay {
  int Ue, Ul, Ur, ce, cl, cr, w, b, total;
};
__host__ __device__ inline PLay make_play(int D, int d) {
  const int F = d + D;
  PLay P;
  P.Ue = 0;
  P.Ul = H * F;
  P.Ur = P.Ul + H * D;
  P.ce = P.Ur + H * D;
  P.cl = P.ce + H;
  P.cr = P.cl + H;
  P.w = P.cr + H;
  P.b = P.w + D;
  P.total = P.b + D;
  return P;
}

// per-edge descriptor written by tgnn_edge_meta (48 B)
struct __attribute__((aligned(16))) EdgeMeta {
  int64_t u;     // source node
  int64_t frow;  // >= 0: feature-table row (ring e_id); -1: self loop (ones); <= -2: -(event row) - 2
  float dt;      // edge time - time_assoc[u] as of the segment's block
  int seg, o, blk;
  int64_t root;
  uint32_t eb, nb;  // dropout mask bases: edge features / time encoding, source memory row
};

// ------------------------------------------------------------------ context
struct Ctx {
  int64_t N;
  int K, D, d, F, Kn, drop, quirk, gen_neg;
  // resident train step with the batch cursor folded into its first launch (tgnx_tgnn_train_fwd_bwd_resident):
  // tgnn_assemble derives the step descriptor from the step counter (what tgnn_advance mode 1 computes) and writes
  // it; the counter itself advances in the next launch (tgnn_meta_collapse), after all three workgroups read it
  int adv, adv_rank, adv_world, adv_train;
  // world-1 resident step with a deferred update: tgnn_grad_reduce records the step's update as pending
  // (ctl[TGNX_CTL_APPLY] = its Adam step count) and the next step's tgnn_assemble launch applies it in its extra
  // workgroups (apply_nel of them elementwise), beside the batch assembly
  int defer, apply_nel;
  int seg_in_pred;  // train: the segment forward rides in tgnn_pred_train (batches below TGNX_BIG_BATCH)
  int64_t adv_lo, adv_hi, adv_batch;
  uint64_t adv_seed;
  float pf, pa, inv_kf, inv_ka;
  float lr, b1, b2, eps;
  const int64_t *ev_src, *ev_dst;
  const float* ev_t;
  const int64_t* ev_blk;
  const float* ev_msg;
  int64_t* neg;
  const int64_t* dst_nodes;
  int64_t n_dst;
  const float* feat;
  int64_t *nbr, *eid;
  float* rt;
  int64_t* assoc;
  float* ta;
  const float* mem;
  float *params, *grads, *am, *av;
  int64_t* ctl;
  float *out_pos, *out_neg;
  float* out_ev;  // optional: train logits by event row [nev, 2] (pos, neg), the epoch's log
  double* mrr;
  int4* nodemap;
  // workspace
  uint64_t* touches;
  int* sp_pref;
  uint64_t* sp_keys;
  int* seg_cnt;
  int* seg_eoff;
  float* seg_out;
  float* seg_stats;
  float* seg_g;
  float* X;
  float* DX;
  struct EdgeMeta* meta;
  float* U;
  float* evs;
  float* slabs;
  float* slabs_s;
  float* red;
  float* blkmax;
  int* blk_rank;
  int* blk_order;
  float* HS;
  uint64_t* rkeys;  // ring insert plan: sorted entries (2B)
  int* rruns;       // run starts (U + 1)
  int* misc;        // MISC_* scalars
  int64_t Ecap;
  int Bmax, Ge, Gs;
  Lay L;
  ULay UL;
  PLay PL;
};

// touch key: node << 26 | block << 14 | kind << 12 | event ; kind 0 = neg, 1 = pos dst, 2 = src
__device__ __forceinline__ int64_t knode(uint64_t k) { return (int64_t)(k >> 26); }
__device__ __forceinline__ int kblk(uint64_t k) { return (int)((k >> 14) & 4095u); }
__device__ __forceinline__ int kkind(uint64_t k) { return (int)((k >> 12) & 3u); }
__device__ __forceinline__ int kev(uint64_t k) { return (int)(k & 4095u); }
__device__ __forceinline__ uint64_t mkkey(int64_t node, int blk, int kind, int ev) {
  return ((uint64_t)node << 26) | ((uint64_t)blk << 14) | ((uint64_t)kind << 12) | (uint64_t)ev;
}

__device__ __forceinline__ float keepf(uint64_t h, float p, float inv) { return u01(h) >= p ? inv : 0.0f; }
__device__ __forceinline__ uint64_t seg_key(int blk, int64_t root) { return ((uint64_t)blk << 32) ^ (uint64_t)root; }
__device__ __forceinline__ uint32_t node_base(uint64_t seed, int blk, int64_t u) {
  return drop_base(seed, 1, ((uint64_t)blk << 32) ^ (uint64_t)u, 0);
}
__device__ __forceinline__ float node_keep(const Ctx& c, uint64_t seed, int blk, int64_t u, int dd) {
  return keep32(node_base(seed, blk, u), (uint32_t)dd, c.pf, c.inv_kf);
}
// edge feature mask base (stream 2) and attention mask base (stream 3) of edge o of a segment
__device__ __forceinline__ uint32_t efeat_base(uint64_t seed, uint64_t sk, int o) { return drop_base(seed, 2, sk, (uint64_t)o); }
__device__ __forceinline__ uint32_t attn_base(uint64_t seed, uint64_t sk, int o) { return drop_base(seed, 3, sk, (uint64_t)o); }

// time_assoc[u] as of block `blk` of the current batch (model_utils.py:77-83)
template <bool TRAIN>
__device__ __forceinline__ float ta_at(const Ctx& c, int64_t u, int blk, int gen, const float* evt) {
  const int4 inf = c.nodemap[u];
  if (inf.x == gen) {
    int lo = inf.y, hi = inf.y + inf.z;
    if (TRAIN) {  // last assignment in blocks <= blk: order n, p, s within a block
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (kblk(c.touches[mid]) <= blk) lo = mid + 1; else hi = mid;
      }
      if (lo > inf.y) return evt[kev(c.touches[lo - 1])];
    } else {      // eval: time_assoc[:] = max(t_blk), then p then s of the block, in batch order
      while (lo < hi) {  // last touch with block <= blk (blocks from the val/test swap may repeat a node)
        int mid = (lo + hi) >> 1;
        if (kblk(c.touches[mid]) <= blk) lo = mid + 1; else hi = mid;
      }
      if (lo > inf.y && kblk(c.touches[lo - 1]) == blk) return evt[kev(c.touches[lo - 1])];
      return c.blkmax[blk];
    }
  }
  return TRAIN ? c.ta[u] : c.blkmax[blk];
}

// ------------------------------------------------------------------ small kernels
// the resident step descriptor of batch nb (0-based within the split) of rank / world (tgnn_advance mode 1)
struct StepDesc {
  int64_t start, B, lo, hi, seed;
};
__device__ __forceinline__ StepDesc step_desc(int64_t nb, int64_t split_lo, int64_t split_hi, int64_t batch, int rank,
                                              int world, uint64_t base_seed) {
  StepDesc d;
  d.start = split_lo + nb * batch;
  d.B = d.start >= split_hi ? 0 : (split_hi - d.start < batch ? split_hi - d.start : batch);
  d.lo = d.B * rank / world;
  d.hi = d.B * (rank + 1) / world;
  d.seed = (int64_t)(mix64(base_seed ^ mix64((uint64_t)(nb + 1))) >> 1);   // (the counter after the advance)
  return d;
}
__global__ void tgnn_advance(int64_t* ctl, int mode, int64_t batch_start, int64_t B, int64_t cur, int64_t split_lo,
                             int64_t split_hi, int64_t batch, int rank, int world, uint64_t base_seed, int train) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t bs = batch_start, Bv = B, ce = cur;
  if (mode == 1) {
    const StepDesc sd = step_desc(ctl[TGNX_CTL_NB], split_lo, split_hi, batch, rank, world, base_seed);
    bs = sd.start;
    Bv = sd.B;
    ce = bs;
  }
  ctl[TGNX_CTL_BATCH_START] = bs;
  ctl[TGNX_CTL_B] = Bv;
  ctl[TGNX_CTL_STEP_B] = Bv;
  ctl[TGNX_CTL_CUR_EID] = ce;
  ctl[TGNX_CTL_GEN] += 1;
  ctl[TGNX_CTL_NB] += 1;
  if (train && Bv > 0) ctl[TGNX_CTL_ADAM_T] += 1;
  ctl[TGNX_CTL_LO] = Bv * rank / world;
  ctl[TGNX_CTL_HI] = Bv * (rank + 1) / world;
  ctl[TGNX_CTL_SEED] = (int64_t)(mix64(base_seed ^ mix64((uint64_t)ctl[TGNX_CTL_NB])) >> 1);
}

// U = attn·W per head (exact collapse of EdgeGATConv's el/er/ee), predictor transposes/row sums.
// Blocks [0, nb_dot): 64 outputs of U_e / U_l / U_r x 4 split-d waves (coalesced over outputs);
// then 4 row sums per block (wave each, lanes over the row); then the two predictor transposes.
__host__ __device__ inline int collapse_blocks(const Ctx& c) {
  return (H * c.F + 63) / 64 + 2 * ((H * c.D + 63) / 64) + (3 * H + 2 * c.D + 3) / 4 + 64;
}
__device__ void collapse_body(const Ctx& c, const int bid, const int nblk) {
  __shared__ float part[4][64];
  const int D = c.D, F = c.F;
  const float* P = c.params;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nbe = (H * F + 63) / 64, nbl = (H * D + 63) / 64;
  const int nb_dot = nbe + 2 * nbl;
  const int nrow = 3 * H + 2 * D;
  const int nb_row = (nrow + 3) / 4;
  if (bid == 0)
    for (int i = threadIdx.x; i < FMAX; i += blockDim.x) c.U[c.UL.ones + i] = 1.0f;
  int b = bid;
  if (b < nb_dot) {
    int which, o;
    if (b < nbe) { which = 0; o = b * 64 + lane; }
    else if (b < nbe + nbl) { which = 1; o = (b - nbe) * 64 + lane; }
    else { which = 2; o = (b - nbe - nbl) * 64 + lane; }
    const int n_out = which == 0 ? H * F : H * D;
    const int W = which == 0 ? F : D;
    float s = 0.f;
    if (o < n_out) {
      const int h = o / W, k = o % W;
      const float* a = P + (which == 0 ? c.L.attn_e : which == 1 ? c.L.attn_l : c.L.attn_r) + h * D;
      const float* M = P + (which == 0 ? c.L.We : c.L.Wn);
      for (int dd = wv; dd < D; dd += 4) s += a[dd] * M[(int64_t)(h * D + dd) * W + k];
    }
    part[wv][lane] = s;
    __syncthreads();
    if (wv == 0 && o < n_out) {
      const float v = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
      c.U[(which == 0 ? c.UL.Ue : which == 1 ? c.UL.Ul : c.UL.Ur) + o] = v;
    }
    return;
  }
  b -= nb_dot;
  if (b < nb_row) {
    const int y = b * 4 + wv;
    if (y >= nrow) return;
    float s = 0.f;
    if (y < 3 * H) {
      const int which = y / H, h = y % H;
      const float* a = P + (which == 0 ? c.L.attn_e : which == 1 ? c.L.attn_l : c.L.attn_r) + h * D;
      const float* bb = P + (which == 0 ? c.L.be : c.L.bn) + h * D;
      for (int dd = lane; dd < D; dd += 64) s += a[dd] * bb[dd];
      s = wave_sum(s);
      if (lane == 0) c.U[(which == 0 ? c.UL.ce : which == 1 ? c.UL.cl : c.UL.cr) + h] = s;
    } else {
      const int z = y - 3 * H, which = z / D, o = z % D;
      const float* w = P + (which == 0 ? c.L.Ws : c.L.Wd) + (int64_t)o * D;
      for (int dd = lane; dd < D; dd += 64) s += w[dd];
      s = wave_sum(s);
      if (lane == 0) c.U[(which == 0 ? c.UL.Ws1 : c.UL.Wd1) + o] = s;
    }
    return;
  }
  b -= nb_row;
  const int64_t nP = (int64_t)D * D;
  for (int64_t x = (int64_t)b * blockDim.x + threadIdx.x; x < 2 * nP; x += (int64_t)(nblk - nb_dot - nb_row) * blockDim.x) {
    const int which = (int)(x / nP);
    const int64_t z = x % nP;
    const int dd = (int)(z / D), o = (int)(z % D);
    c.U[(which == 0 ? c.UL.WsT : c.UL.WdT) + z] = P[(which == 0 ? c.L.Ws : c.L.Wd) + (int64_t)o * D + dd];
  }
}

// ------------------------------------------------------------------ segment geometry
// Segment w (this rank's rows): [0, nloc) src rows, [nloc, 2 nloc) dst rows, then neg rows.
struct Seg {
  int kind, i, cc, blk;
  int64_t root;
};
__device__ __forceinline__ bool seg_of(const Ctx& c, int w, int lo, int hi, int64_t start, Seg& s) {
  const int nloc = hi - lo;
  const int Kn = c.Kn;
  if (w < 0 || w >= nloc * (2 + Kn)) return false;
  if (w < nloc) {
    s.kind = 2; s.i = lo + w; s.cc = 0;
  } else if (w < 2 * nloc) {
    s.kind = 1; s.i = lo + w - nloc; s.cc = 0;
  } else {
    const int q = w - 2 * nloc;
    s.kind = 0; s.i = lo + q / Kn; s.cc = q % Kn;
  }
  s.root = s.kind == 2 ? c.ev_src[start + s.i] : s.kind == 1 ? c.ev_dst[start + s.i]
                                                             : c.neg[(start + s.i) * Kn + s.cc];
  s.blk = (int)c.ev_blk[start + s.i];
  return true;
}

// in-edge count of a segment: ring row + self loop + intra-batch edges of earlier blocks
// (returned packed: nring | nintra << 8)
__device__ __forceinline__ int seg_count_one(const Ctx& c, int w, int lo, int hi, int64_t start, int gen) {
  Seg s;
  seg_of(c, w, lo, hi, start, s);
  int nring = 0;
  for (int j = 0; j < c.K; ++j) nring += c.eid[s.root * c.K + j] >= 0;
  int nintra = 0;
  const int4 inf = c.nodemap[s.root];
  if (inf.x == gen) {
    int a = inf.w, z = c.sp_pref[inf.y + inf.z];
    const int base = a;
    while (a < z) {
      const int mid = (a + z) >> 1;
      if (kblk(c.sp_keys[mid]) < s.blk) a = mid + 1; else z = mid;
    }
    nintra = a - base;
  }
  return nring | (nintra << 8);
}

__global__ void tgnn_seg_count(Ctx c) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int S = (int)c.ctl[TGNX_CTL_S];
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (B == 0 || w >= S || c.ctl[TGNX_CTL_ERR] != 0 || c.ctl[TGNX_CTL_E] >= 0) return;  // E >= 0: done in assemble
  c.seg_cnt[w] = seg_count_one(c, w, (int)c.ctl[TGNX_CTL_LO], (int)c.ctl[TGNX_CTL_HI],
                               c.ctl[TGNX_CTL_BATCH_START], (int)c.ctl[TGNX_CTL_GEN]);
}

// ------------------------------------------------------------------ assembly (two workgroups)
// Workgroup 0 sorts the batch's node touches (src / dst / neg rows) by (node, block, kind, event),
// builds the node map {gen, run start, run length, first s/p index}, the compacted s/p touch list
// (the intra-batch edges of model_utils.py:151-152 in block order), per-block max t and block
// order, and (train) each segment's in-edge count + the edge offsets, all from the sorted touches in
// LDS.  Workgroup 1 meanwhile builds the ring insert plan (neighbor_loader.py:52-104) that
// tgnn_finish applies with a wave per node.
// Workgroup 2 computes the per-block max t and the stable block order.
// LDS of workgroup 0: sorted keys [next_pow2(NT)] u64 | run starts [NT] | run id per touch [NT] |
// register-sort ping-pong buffer [1024] u64 | ring fill per unsorted touch [NT]; a touch sort above 1,024 keys
// uses everything past the keys as its ping-pong buffer (next_pow2(NT) keys).
__host__ __device__ inline size_t assemble_smem_bytes(int Bmax) {
  const int NT = 3 * Bmax;
  const size_t tail = (size_t)NT * 8 + 1024 * 8 + (size_t)NT * 4;
  const size_t big = (size_t)next_pow2(NT) * 8;
  return (size_t)next_pow2(NT) * 8 + (tail > big ? tail : big);
}
// Touch sort above 1,024 keys (B > 341; TGN.yml's B = 2,000: 6,000 keys): an LSD radix sort of the block in
// registers (rocprim::block_radix_sort, 8 keys per thread, 8-bit digits over the key's used bits: 26 + log2 N),
// stable, ~5 passes: 37 us at B = 2,000.  An 8-keys-per-thread register bitonic network measured ~100 us for
// 8,192 keys on the one CU (VALU-bound: 63 lane stages x 8 keys; removed), the LDS bitonic network 104 us.  The rocprim storage aliases the LDS from `smem`.
using TouchRadix = rocprim::block_radix_sort<uint64_t, 1024, 8>;
__device__ __forceinline__ bool touch_radix_fits(int Bmax) {
  return sizeof(TouchRadix::storage_type) <= assemble_smem_bytes(Bmax);
}
__device__ __forceinline__ void sort_touches_radix(uint64_t* key, int n_keys, int64_t N, unsigned char* smem) {
  const int t = threadIdx.x;
  uint64_t v[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int p = t * 8 + m;
    v[m] = p < n_keys ? key[p] : ~0ull;
  }
  int nb = 1;
  while (nb < 38 && (int64_t(1) << nb) < N) ++nb;
  __syncthreads();  // (the storage overwrites the keys)
  TouchRadix().sort(v, *reinterpret_cast<TouchRadix::storage_type*>(smem), 0, 26 + nb);
  __syncthreads();
#pragma unroll
  for (int m = 0; m < 8; ++m)
    if (t * 8 + m < n_keys) key[t * 8 + m] = v[m];  // (past n_keys: padding, sorted last)
  __syncthreads();
}

__device__ void expand_adam_body(const Ctx& c, int64_t t, int bid, int nblk, int nel);
template <bool TRAIN>
__global__ void __launch_bounds__(1024) tgnn_assemble(Ctx c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int sh[20];
  const int tid = threadIdx.x, T = blockDim.x;
  if (TRAIN && c.defer && blockIdx.x >= 3) {  // the previous step's pending update, beside this step's assembly
    const int64_t t = c.ctl[TGNX_CTL_APPLY];
    if (t > 0) expand_adam_body(c, t, blockIdx.x - 3, gridDim.x - 3, c.apply_nel);
    return;
  }
  int B;
  int64_t start;
  StepDesc sd{};
  if (c.adv) {  // folded cursor: every workgroup derives the descriptor from the (not yet advanced) step counter
    sd = step_desc(c.ctl[TGNX_CTL_NB], c.adv_lo, c.adv_hi, c.adv_batch, c.adv_rank, c.adv_world, c.adv_seed);
    B = (int)sd.B;
    start = sd.start;
  } else {
    B = (int)c.ctl[TGNX_CTL_B];
    start = c.ctl[TGNX_CTL_BATCH_START];
  }
  if (blockIdx.x == 1) {  // ring insert plan
    if (B == 0 || B > c.Bmax) return;
    TGNN_PHASE_STAMP(c, 8);
    uint64_t* key;
    int* runs;
    // (the LDS holds a full ping-pong buffer past the run starts: register sorts up to 2B = 4,096)
    const int U = ring_plan_block(c.ev_src + start, c.ev_dst + start, B, smem, sh, &key, &runs, NoCheckpoint{}, true);
    TGNN_PHASE_STAMP(c, 9);
    for (int p = tid; p < 2 * B; p += T) c.rkeys[p] = key[p];
    for (int r = tid; r < U; r += T) c.rruns[r] = runs[r];
    if (tid == 0) {
      c.rruns[U] = 2 * B;
      c.misc[MISC_RUNS] = U;
    }
    TGNN_PHASE_STAMP(c, 10);
    return;
  }
  if (blockIdx.x == 2) {  // per-block max t (eval's time_assoc[:] = max, model_utils.py:78), block order
    if (B == 0 || B > c.Bmax) return;
    const int64_t* blk = c.ev_blk + start;
    const float* evt = c.ev_t + start;
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);
    float* bmax = c.blkmax;
    for (int b = tid; b < B; b += T) bmax[b] = -INFINITY;
    __syncthreads();
    for (int e = tid; e < B; e += T) atomicMax(&bmax[(int)blk[e]], evt[e]);
    const int nb = next_pow2(B);
    for (int p = tid; p < nb; p += T) key[p] = p < B ? (((uint64_t)blk[p] << 12) | (uint64_t)p) : ~0ull;
    __syncthreads();
    sort_u64(key, key + nb, B, nb);
    for (int r = tid; r < B; r += T) {
      const int e = (int)(key[r] & 4095u);
      c.blk_rank[e] = r;
      c.blk_order[r] = e;
    }
    if (tid == 0) c.misc[MISC_KMAX] = (int)(key[B - 1] >> 12);
    return;
  }
  // workgroup 0 publishes the descriptor (later launches read it; tgnn_meta_collapse advances the step counter)
  const int gen = (int)c.ctl[TGNX_CTL_GEN] + (c.adv ? 1 : 0);
  if (c.adv) __syncthreads();  // (every thread has read the counter before thread 0 rewrites it)
  if (c.adv && tid == 0) {
    int64_t* ctl = c.ctl;
    ctl[TGNX_CTL_BATCH_START] = sd.start;
    ctl[TGNX_CTL_B] = sd.B;
    ctl[TGNX_CTL_STEP_B] = sd.B;
    ctl[TGNX_CTL_CUR_EID] = sd.start;
    ctl[TGNX_CTL_GEN] = gen;
    if (c.adv_train && sd.B > 0) ctl[TGNX_CTL_ADAM_T] += 1;
    ctl[TGNX_CTL_LO] = sd.lo;
    ctl[TGNX_CTL_HI] = sd.hi;
    ctl[TGNX_CTL_SEED] = sd.seed;
  }
  if (B == 0) {
    if (tid == 0) c.ctl[TGNX_CTL_S] = c.ctl[TGNX_CTL_E] = 0;
    return;
  }
  const int64_t* src = c.ev_src + start;
  const int64_t* dst = c.ev_dst + start;
  const float* evt = c.ev_t + start;
  const int64_t* blk = c.ev_blk + start;
  const int64_t* neg = c.neg + start * c.Kn;
  const int NT = TRAIN ? 3 * B : 2 * B;
  if (B > c.Bmax || B > 4095) {
    if (tid == 0) c.ctl[TGNX_CTL_ERR] |= 1;
    return;
  }
  const int n = next_pow2(NT);
  const int NTc = 3 * c.Bmax;
  uint64_t* key = reinterpret_cast<uint64_t*>(smem);
  int* run_start = reinterpret_cast<int*>(smem + (size_t)next_pow2(NTc) * 8);
  int* run_of = run_start + NTc;
  uint64_t* tmp = reinterpret_cast<uint64_t*>(run_of + NTc);
  int* fill = reinterpret_cast<int*>(tmp + 1024);  // ring fill of touch p's node (one touch per thread)
  TGNN_PHASE_STAMP(c, 0);
  const bool draw = TRAIN && c.gen_neg;
  const uint64_t nseed = !draw ? 0 : c.adv ? (uint64_t)sd.seed : (uint64_t)c.ctl[TGNX_CTL_SEED];
  const uint64_t noff = !draw ? 0 : c.adv ? (uint64_t)sd.start : (uint64_t)c.ctl[TGNX_CTL_CUR_EID];
  // one touch per thread (B <= 341): its node's ring fill is loaded here, beside the key, and parked in LDS after
  // the sort (the segment counts read it there instead of ten dependent-on-the-sort global loads)
  const bool one = TRAIN && NT <= T && c.K <= 16;
  int64_t ring_eid[16];  // consumed after the sort: the loads overlap it
#pragma unroll
  for (int j = 0; j < 16; ++j) ring_eid[j] = -1;
  for (int p = tid; p < n; p += T) {
    uint64_t k = ~0ull;
    if (p < NT) {
      int e = p % B, which = p / B;  // 0 = s, 1 = p, 2 = n
      int64_t node;
      if (which == 2 && draw) {  // NegLinkSamplerDest.sample (neg_sampler.py:8-23), counter-based stream
        const int64_t pd = dst[e];
        node = c.dst_nodes[0];
        for (uint64_t attempt = 0; attempt < 64; ++attempt) {
          const uint64_t h = hash4(nseed, 0x6E656773ull, noff + (uint64_t)e, attempt);
          node = c.dst_nodes[(uint64_t)(((__uint128_t)(h >> 11) * (uint64_t)c.n_dst) >> 53)];
          if (node != pd) break;
        }
        c.neg[start + e] = node;
      } else {
        node = which == 0 ? src[e] : which == 1 ? dst[e] : neg[e];
      }
      k = mkkey(node, (int)blk[e], 2 - which, e);
      if (one)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j < c.K) ring_eid[j] = c.eid[node * c.K + j];
    }
    key[p] = k;
  }
  __syncthreads();
  TGNN_PHASE_STAMP(c, 1);
  // the touch keys are pairwise distinct ((kind, event) is unique): up to 1,024 touches sort in 64-key register
  // chunks + binary-search ranks (sort_u64_chunks) instead of the 55-stage bitonic network (8.7 -> ~3 us at B = 200)
  if (NT <= 1024) sort_u64(key, tmp, NT, n, /*distinct=*/true);
  else if (NT <= 8192 && blockDim.x == 1024 && touch_radix_fits(c.Bmax)) sort_touches_radix(key, n, c.N, smem);
  else sort_u64(key, reinterpret_cast<uint64_t*>(run_start), NT, n, true, /*tmp_full=*/true);
  if (one && tid < NT) {  // (read after the barriers of the scans below)
    int f = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) f += ring_eid[j] >= 0;
    fill[tid] = f;
  }
  TGNN_PHASE_STAMP(c, 2);
  const int pc = (NT + T - 1) / T;
  const int p0 = tid * pc, p1 = min(NT, p0 + pc);
  // compacted s/p list (kind != 0), exclusive prefix over the sorted touches
  {
    int cnt = 0;
    for (int p = p0; p < p1; ++p) cnt += kkind(key[p]) != 0;
    int tot;
    int base = block_excl_scan(cnt, sh, &tot);
    for (int p = p0; p < p1; ++p) {
      c.touches[p] = key[p];
      c.sp_pref[p] = base;
      if (kkind(key[p]) != 0) c.sp_keys[base++] = key[p];
    }
    if (tid == 0) c.sp_pref[NT] = tot;
  }
  TGNN_PHASE_STAMP(c, 3);
  // node runs -> node map; run id of every touch
  {
    int cnt = 0;
    for (int p = p0; p < p1; ++p) cnt += (p == 0 || knode(key[p]) != knode(key[p - 1]));
    int U;
    int rid = block_excl_scan(cnt, sh, &U);
    for (int p = p0; p < p1; ++p) {
      if (p == 0 || knode(key[p]) != knode(key[p - 1])) run_start[rid++] = p;
      run_of[p] = rid - 1;
    }
    __syncthreads();
    for (int r = tid; r < U; r += T) {
      const int a = run_start[r];
      const int e = r + 1 < U ? run_start[r + 1] : NT;
      c.nodemap[knode(key[a])] = make_int4(gen, a, e - a, c.sp_pref[a]);
    }
  }
  TGNN_PHASE_STAMP(c, 4);
  const int lo = c.adv ? (int)sd.lo : (int)c.ctl[TGNX_CTL_LO], hi = c.adv ? (int)sd.hi : (int)c.ctl[TGNX_CTL_HI];
  const int nloc = hi - lo;
  const int S = nloc * (2 + c.Kn);
  if (TRAIN) {  // in-edge count of each segment (= touch p of this rank's rows, Kn == 1):
    // ring fill + self loop + s/p touches of the node in earlier blocks = sp_pref[first touch of
    // (node, block)] - sp_pref[run start]
    for (int p = tid; p < NT; p += T) {
      const uint64_t k = key[p];
      const int ev = kev(k);
      if (ev < lo || ev >= hi) continue;
      const int kind = kkind(k);
      const int w = kind == 2 ? ev - lo : kind == 1 ? nloc + ev - lo : 2 * nloc + (ev - lo);
      int g = p;
      while (g > 0 && (key[g - 1] >> 14) == (k >> 14)) --g;
      const int64_t v = knode(k);
      int nring = 0;
      if (one) nring = fill[(2 - kind) * B + ev];
      else
        for (int j = 0; j < c.K; ++j) nring += c.eid[v * c.K + j] >= 0;
      const int nintra = c.sp_pref[g] - c.sp_pref[run_start[run_of[p]]];
      c.seg_cnt[w] = nring | (nintra << 8);
    }
  }
  __syncthreads();
  TGNN_PHASE_STAMP(c, 5);
  TGNN_PHASE_STAMP(c, 6);
  if (TRAIN) {  // segment edge offsets (seg_cnt written above by this workgroup)
    const int chunk = (S + T - 1) / T;
    const int r0 = tid * chunk, r1 = min(S, r0 + chunk);
    int s = 0;
    for (int r = r0; r < r1; ++r) {
      const int v = c.seg_cnt[r];
      s += (v & 255) + 1 + (v >> 8);
    }
    int tot;
    int base = block_excl_scan(s, sh, &tot);
    for (int r = r0; r < r1; ++r) {
      c.seg_eoff[r] = base;
      const int v = c.seg_cnt[r];
      base += (v & 255) + 1 + (v >> 8);
    }
    if (tid == 0) {
      c.seg_eoff[S] = tot;
      c.ctl[TGNX_CTL_S] = S;
      c.ctl[TGNX_CTL_E] = tot;
      c.ctl[TGNX_CTL_SUM_E] += tot;
      c.ctl[TGNX_CTL_SUM_S] += S;
      if (tot > c.Ecap) c.ctl[TGNX_CTL_ERR] |= 2;
    }
  } else if (tid == 0) {
    c.ctl[TGNX_CTL_S] = S;
    c.ctl[TGNX_CTL_E] = -1;   // counted by tgnn_seg_count / tgnn_seg_scan
  }
  TGNN_PHASE_STAMP(c, 7);
}

// exclusive scan of the edge counts (one workgroup) -> edge offsets
__global__ void __launch_bounds__(1024) tgnn_seg_scan(Ctx c) {
  __shared__ int sh[20];
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0 || c.ctl[TGNX_CTL_E] >= 0) return;
  const int S = (int)c.ctl[TGNX_CTL_S];
  const int T = blockDim.x;
  const int chunk = (S + T - 1) / T;
  const int r0 = threadIdx.x * chunk, r1 = min(S, r0 + chunk);
  int s = 0;
  for (int r = r0; r < r1; ++r) {
    const int v = c.seg_cnt[r];
    s += (v & 255) + 1 + (v >> 8);
  }
  int tot;
  int base = block_excl_scan(s, sh, &tot);
  for (int r = r0; r < r1; ++r) {
    c.seg_eoff[r] = base;
    const int v = c.seg_cnt[r];
    base += (v & 255) + 1 + (v >> 8);
  }
  if (threadIdx.x == 0) {
    c.seg_eoff[S] = tot;
    c.ctl[TGNX_CTL_E] = tot;
    c.ctl[TGNX_CTL_SUM_E] += tot;
    c.ctl[TGNX_CTL_SUM_S] += S;
    if (tot > c.Ecap) c.ctl[TGNX_CTL_ERR] |= 2;
  }
}

// per edge: source node, feature row, dt = t_edge - time_assoc[src] as of the block
template <bool TRAIN>
__device__ void edge_meta_body(const Ctx& c, const int bid, const int nblk) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int S = (int)c.ctl[TGNX_CTL_S];
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  const int lo_ev = (int)c.ctl[TGNX_CTL_LO], hi_ev = (int)c.ctl[TGNX_CTL_HI];
  const int gen = (int)c.ctl[TGNX_CTL_GEN];
  const float* evt = c.ev_t + start;
  const int lane = threadIdx.x & 63;
  // wave per segment, lanes over its edges: the segment's root / block / edge range are loaded once
  // per wave (an edge-parallel layout needed a dependent binary search over the segment offsets)
  for (int w = bid * 4 + (threadIdx.x >> 6); w < S; w += nblk * 4) {
    Seg s;
    seg_of(c, w, lo_ev, hi_ev, start, s);
    const int cntw = c.seg_cnt[w];
    const int nring = cntw & 255;
    const int e0 = c.seg_eoff[w], ne = c.seg_eoff[w + 1] - e0;
    const int spw = c.nodemap[s.root].w;
    for (int o = lane; o < ne; o += 64) {
      EdgeMeta m;
      float bt;
      if (o < nring) {
        const int64_t idx = s.root * c.K + o;
        m.u = c.nbr[idx];
        m.frow = c.eid[idx];
        bt = c.rt[idx];
      } else if (o == nring) {
        m.u = s.root;
        m.frow = -1;
        bt = 0.f;
      } else {
        const uint64_t k = c.sp_keys[spw + (o - nring - 1)];
        const int ev = kev(k);
        m.u = kkind(k) == 2 ? c.ev_dst[start + ev] : c.ev_src[start + ev];
        m.frow = -(start + ev) - 2;
        bt = evt[ev];
      }
      m.dt = bt - ta_at<TRAIN>(c, m.u, s.blk, gen, evt);
      m.seg = w;
      m.o = o;
      m.blk = s.blk;
      m.root = s.root;
      if (c.drop) {
        const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
        m.eb = efeat_base(seed, seg_key(s.blk, s.root), o);
        m.nb = node_base(seed, s.blk, m.u);
      } else {
        m.eb = m.nb = 0u;
      }
      c.meta[e0 + o] = m;
    }
  }
}

// edge metadata and the collapsed weights (independent) in one launch: blocks [0, nmeta) then the
// collapse blocks
template <bool TRAIN>
__global__ void __launch_bounds__(256) tgnn_meta_collapse(Ctx c, int nmeta) {
  // folded cursor: the step counter advances here, after tgnn_assemble's workgroups all read it (nothing in this
  // launch or later reads it within the step)
  if (c.adv && blockIdx.x == 0 && threadIdx.x == 0) c.ctl[TGNX_CTL_NB] += 1;
  if ((int)blockIdx.x < nmeta) edge_meta_body<TRAIN>(c, blockIdx.x, nmeta);
  else collapse_body(c, blockIdx.x - nmeta, gridDim.x - nmeta);
}

__device__ __forceinline__ const float* feat_row(const Ctx& c, int64_t frow) {
  return frow >= 0 ? c.feat + frow * c.d : frow == -1 ? nullptr : c.ev_msg + (-(frow + 2)) * c.d;
}

// Column map shared by the edge kernels (a wave per edge, lanes over columns): CF feature
// columns (dims lane + 64j of the edge feature row, j < CF), CT time-encoding columns (dims
// d + lane + 64j) and CT memory columns (dims lane + 64j of the source memory row).  Gathers use
// clamped indices and the self-loop row points at a row of ones, so no load is predicated;
// lanes past the end read finite values whose weights / outputs are zero / never written.
template <int CF, int CT>
struct EdgeCols {
  int fidx[CF > 0 ? CF : 1], kidx[CT];
  __device__ __forceinline__ EdgeCols(int lane, int d, int D) {
#pragma unroll
    for (int j = 0; j < CF; ++j) fidx[j] = min(lane + 64 * j, d - 1);
#pragma unroll
    for (int j = 0; j < CT; ++j) kidx[j] = min(lane + 64 * j, D - 1);
  }
};
template <int CF, int CT>
struct EdgeVals {
  float dt, vf[CF > 0 ? CF : 1], vm[CT];
  uint32_t eb, nb;
};
template <int CF, int CT>
__device__ __forceinline__ void edge_gather(const Ctx& c, int e, const EdgeCols<CF, CT>& cols, EdgeVals<CF, CT>& S) {
  const EdgeMeta m = c.meta[e];
  const float* fp = m.frow >= 0 ? c.feat + m.frow * c.d
                                : m.frow == -1 ? c.U + c.UL.ones : c.ev_msg + (-(m.frow + 2)) * c.d;
  const float* mu = c.mem + m.u * c.D;
#pragma unroll
  for (int j = 0; j < CF; ++j) S.vf[j] = fp[cols.fidx[j]];
#pragma unroll
  for (int j = 0; j < CT; ++j) S.vm[j] = mu[cols.kidx[j]];
  S.dt = m.dt;
  S.eb = m.eb;
  S.nb = m.nb;
}

// Sum of v[0..7] over the wave by recursive halving (10 exchanges: permlane swaps for lane ^ 32 / ^ 16,
// DPP for the rest — no LDS round trip): on return lane l holds the total of head l / 8 (lanes with
// l % 8 == 0 write).  Full wave.
__device__ __forceinline__ float wave_sum8(const float (&v)[H], int lane) {
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
  float k4[4], k2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float keep = b5 ? v[4 + i] : v[i], send = b5 ? v[i] : v[4 + i];
    k4[i] = keep + xor32_f(send);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float keep = b4 ? k4[2 + i] : k4[i], send = b4 ? k4[i] : k4[2 + i];
    k2[i] = keep + xor16_f(send);
  }
  float s = (b3 ? k2[1] : k2[0]) + dpp_f<0x128>(b3 ? k2[0] : k2[1]);  // row_ror:8 = lane ^ 8 in the row
  s += dpp_f<0xB1>(s);   // lane ^ 1
  s += dpp_f<0x4E>(s);   // lane ^ 2
  s += dpp_f<0x141>(s);  // half-row mirror: the other quad (quads uniform by now)
  return s;
}

// Segment kernels use lane l = 8 j + h: edge slot j (0..7) x head h.  Reductions over the edge
// slots (lanes l ^ 8, l ^ 16, l ^ 32) and over the heads (l ^ 1, l ^ 2, l ^ 4) use DPP / swizzle.
__device__ __forceinline__ float red_j_sum(float v) {
  v += __uint_as_float(xlane_xor<8>(__float_as_uint(v)));
  v += __uint_as_float(xlane_xor<16>(__float_as_uint(v)));
  v += __uint_as_float(xlane_xor<32>(__float_as_uint(v)));
  return v;
}
__device__ __forceinline__ float red_j_max(float v) {
  v = fmaxf(v, __uint_as_float(xlane_xor<8>(__float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(xlane_xor<16>(__float_as_uint(v))));
  v = fmaxf(v, __uint_as_float(xlane_xor<32>(__float_as_uint(v))));
  return v;
}
__device__ __forceinline__ float red_h_sum(float v) {
  v += __uint_as_float(xlane_xor<1>(__float_as_uint(v)));
  v += __uint_as_float(xlane_xor<2>(__float_as_uint(v)));
  v += __uint_as_float(xlane_xor<4>(__float_as_uint(v)));
  return v;
}
// er_h = U_r[h]·drop(mem[root]) + c_r[h] (model_utils.py:588 collapsed) for the lane's head h:
// dims dd = j + 8k, loads issued before the FMAs, then summed over the edge slots
__device__ __forceinline__ float root_er8(const Ctx& c, const Seg& s, uint64_t seed, bool drop, int j, int h) {
  constexpr int KD = DMAX / 8;
  const int D = c.D;
  const uint32_t nb = drop ? node_base(seed, s.blk, s.root) : 0u;
  float mv[KD], uv[KD];
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int dd = min(j + 8 * k, D - 1);
    mv[k] = c.mem[s.root * D + dd];
    uv[k] = c.U[c.UL.Ur + h * D + dd];
  }
  float p = 0.f;
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int dd = j + 8 * k;
    if (dd < D) {
      float v = mv[k];
      if (drop) v *= keep32(nb, (uint32_t)dd, c.pf, c.inv_kf);
      p += uv[k] * v;
    }
  }
  return red_j_sum(p) + c.U[c.UL.cr + h];
}

// x_eh = U_e[h]·[efeat_e, drop(cos(w dt + b))] + U_l[h]·drop(mem[src]) + c_h   (model_utils.py:447-452
// collapsed): a wave per edge, each lane's U columns held in registers across
// edges, two gather sets ping-pong so one edge's loads are in flight during the other's math.
template <bool TRAIN>
__device__ void finish_body(const Ctx& c, const int bid, const int nblk);

#ifndef TGNX_GFWD
// edge workgroups: 150 VGPRs leave room for 3 waves per SIMD, i.e. 768 four-wave workgroups on 256 CUs (512: 2 per
// SIMD; TGN.yml's B = 2,000 step 1.174 -> 1.128 ms, B = 200 +-0, profiles/r6/r6v_*).  1,024 workgroups with the
// registers capped for 4 waves per SIMD measured 1.22 ms (r6w_*)
#define TGNX_GFWD 768
#endif
constexpr int GFWD = TGNX_GFWD;
template <int CF, int CT, bool DROP>
__global__ void __launch_bounds__(256) tgnn_edge_fwd(Ctx c) {
  constexpr int NJ = CF + 2 * CT;
  if ((int)blockIdx.x >= GFWD) {  // train: the batch's ring insert + time_assoc update (nothing after
    // tgnn_edge_meta reads them; epoch_utils.py:304, model_utils.py:81-83) rides in this launch
    finish_body<true>(c, blockIdx.x - GFWD, gridDim.x - GFWD);
    return;
  }
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int F = c.F, D = c.D, d = c.d;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float Ur[NJ][H], tw[CT], tb[CT];
#pragma unroll
  for (int j = 0; j < CF; ++j) {
    const int f = lane + 64 * j;
#pragma unroll
    for (int h = 0; h < H; ++h) Ur[j][h] = f < d ? c.U[c.UL.Ue + h * F + f] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    const int i = lane + 64 * j;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      Ur[CF + j][h] = i < D ? c.U[c.UL.Ue + h * F + d + i] : 0.f;
      Ur[CF + CT + j][h] = i < D ? c.U[c.UL.Ul + h * D + i] : 0.f;
    }
    tw[j] = i < D ? c.params[c.L.te_w + i] : 0.f;
    tb[j] = i < D ? c.params[c.L.te_b + i] : 0.f;
  }
  const float cst = c.U[c.UL.ce + (lane >> 3)] + c.U[c.UL.cl + (lane >> 3)];
  const EdgeCols<CF, CT> cols(lane, d, D);
  const int E = (int)c.ctl[TGNX_CTL_E];
  auto math = [&](int e, const EdgeVals<CF, CT>& S) {
    float acc[H];
#pragma unroll
    for (int h = 0; h < H; ++h) acc[h] = 0.f;
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      float x = S.vf[j];
      if (DROP) x *= keep32(S.eb, (uint32_t)(lane + 64 * j), c.pf, c.inv_kf);
#pragma unroll
      for (int h = 0; h < H; ++h) acc[h] += Ur[j][h] * x;
    }
#pragma unroll
    for (int j = 0; j < CT; ++j) {  // time encoding (model_utils.py:235)
      float x = te_cos(fmaf(tw[j], S.dt, tb[j]));
      if (DROP) x *= keep32(S.eb, (uint32_t)(d + lane + 64 * j), c.pf, c.inv_kf);
#pragma unroll
      for (int h = 0; h < H; ++h) acc[h] += Ur[CF + j][h] * x;
    }
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      float x = S.vm[j];
      if (DROP) x *= keep32(S.nb, (uint32_t)(lane + 64 * j), c.pf, c.inv_kf);
#pragma unroll
      for (int h = 0; h < H; ++h) acc[h] += Ur[CF + CT + j][h] * x;
    }
    const float s = wave_sum8(acc, lane);
    if ((lane & 7) == 0) c.X[(int64_t)e * H + (lane >> 3)] = s + cst;
  };
  const int stride = GFWD * 4;
  int e = blockIdx.x * 4 + wv;
  EdgeVals<CF, CT> A, Bv;
  if (e < E) edge_gather(c, e, cols, A);
  while (e < E) {
    const int e1 = e + stride;
    if (e1 < E) edge_gather(c, e1, cols, Bv);
    math(e, A);
    if (e1 >= E) break;
    const int e2 = e1 + stride;
    if (e2 < E) edge_gather(c, e2, cols, A);
    math(e1, Bv);
    e = e2;
  }
}
template <int CF>
static void launch_edge_fwd_cf(const Ctx& c, int nfin, hipStream_t s) {
  const bool two = c.D > 64;
  const int g = GFWD + nfin;
  if (c.drop) two ? tgnn_edge_fwd<CF, 2, true><<<g, 256, 0, s>>>(c) : tgnn_edge_fwd<CF, 1, true><<<g, 256, 0, s>>>(c);
  else two ? tgnn_edge_fwd<CF, 2, false><<<g, 256, 0, s>>>(c) : tgnn_edge_fwd<CF, 1, false><<<g, 256, 0, s>>>(c);
}
static void launch_edge_fwd(const Ctx& c, int nfin, hipStream_t s) {
  switch ((c.d + 63) / 64) {
    case 0: launch_edge_fwd_cf<0>(c, nfin, s); break;
    case 1: launch_edge_fwd_cf<1>(c, nfin, s); break;
    case 2: launch_edge_fwd_cf<2>(c, nfin, s); break;
    case 3: launch_edge_fwd_cf<3>(c, nfin, s); break;
    case 4: launch_edge_fwd_cf<4>(c, nfin, s); break;
    default: launch_edge_fwd_cf<5>(c, nfin, s); break;
  }
}

__device__ __forceinline__ void load_x8(const float* p, float (&x)[H]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}


// Segments longer than SEG_WIDE edges (a hub node's: up to ~900 at B = 2,000) run with lane = edge slot (64 slots,
// all 8 heads per lane) instead of 8 slots x 8 heads, so their serial chain is 8x shorter (B = 2,000 step 0.997 ->
// 0.967 ms; from 64 edges the B = 200 step lost 2.6 %, from 128 it is unchanged: profiles/r6/r6ak_*, r6al_*)
constexpr int SEG_WIDE = 128;
__device__ __forceinline__ float pick8(const float (&v)[H], int h) {
  float r = v[0];
#pragma unroll
  for (int k = 1; k < H; ++k) r = h == k ? v[k] : r;
  return r;
}
__device__ __forceinline__ void load_row8(const float* p, float (&x)[H]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}

// per segment: LeakyReLU, edge softmax per head (model_utils.py:595-597), ft = Σ a·x, head mean;
// segment w by one wave (lane = 8 edge slots x 8 heads): edge softmax with attention dropout and the head mean
// (model_utils.py:589-605 collapsed), online over chunks of 8 edges; returns the segment's output (every lane)
template <bool TRAIN>
__device__ float seg_fwd_one(const Ctx& c, const int w, const int lane) {
  const int j = lane >> 3, h = lane & 7;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  Seg s;
  seg_of(c, w, (int)c.ctl[TGNX_CTL_LO], (int)c.ctl[TGNX_CTL_HI], start, s);
  const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const bool drop = TRAIN && c.drop;
  const float er = root_er8(c, s, seed, drop, j, h);
  const int e0 = c.seg_eoff[w], ne = c.seg_eoff[w + 1] - e0;
  const uint64_t sk = seg_key(s.blk, s.root);
  const float* __restrict__ X = c.X + (int64_t)e0 * H + h;
  float m = -INFINITY, l = 0.f, acc = 0.f;
  if (ne > SEG_WIDE) {  // (wave-uniform) lane = edge slot, all heads per lane; lanes merged in a fixed order
    float erh[H], mw[H], lw[H], aw[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      erh[k] = __shfl(er, k, WAVE);  // (lane k: slot 0, head k)
      mw[k] = -INFINITY;
      lw[k] = aw[k] = 0.f;
    }
    const float* __restrict__ Xr = c.X + (int64_t)e0 * H;
    for (int o = lane; o < ne; o += WAVE) {
      float xv[H];
      load_row8(Xr + (int64_t)o * H, xv);
      const uint32_t ab = drop ? attn_base(seed, sk, o) : 0u;
#pragma unroll
      for (int k = 0; k < H; ++k) {
        float sc = xv[k] + erh[k];
        sc = sc > 0.f ? sc : 0.2f * sc;
        const float mn = fmaxf(mw[k], sc);
        const float r = mw[k] == -INFINITY ? 0.f : expf(mw[k] - mn);
        const float ex = expf(sc - mn);
        float wgt = ex;
        if (drop) wgt *= keep32(ab, (uint32_t)k, c.pa, c.inv_ka);
        lw[k] = lw[k] * r + ex;
        aw[k] = aw[k] * r + wgt * xv[k];
        mw[k] = mn;
      }
    }
#pragma unroll
    for (int st = 1; st < WAVE; st <<= 1)
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const float mo = __shfl_xor(mw[k], st, WAVE), lo = __shfl_xor(lw[k], st, WAVE),
                    ao = __shfl_xor(aw[k], st, WAVE);
        const float mn = fmaxf(mw[k], mo);
        const float r1 = mw[k] == -INFINITY ? 0.f : expf(mw[k] - mn);
        const float r2 = mo == -INFINITY ? 0.f : expf(mo - mn);
        lw[k] = lw[k] * r1 + lo * r2;
        aw[k] = aw[k] * r1 + ao * r2;
        mw[k] = mn;
      }
    m = pick8(mw, h);
    l = pick8(lw, h);
    acc = pick8(aw, h);
  } else {
  // each lane: online softmax over its edges o = j, j + 8, ... (no cross-lane traffic in the loop)
#pragma unroll 4
  for (int o = j; o < ne; o += 8) {
    const float x = X[(int64_t)o * H];
    float sc = x + er;
    sc = sc > 0.f ? sc : 0.2f * sc;
    const float mn = fmaxf(m, sc);
    const float r = m == -INFINITY ? 0.f : expf(m - mn);
    const float ex = expf(sc - mn);
    float wgt = ex;
    if (drop) wgt *= keep32(attn_base(seed, sk, o), (uint32_t)h, c.pa, c.inv_ka);
    l = l * r + ex;
    acc = acc * r + wgt * x;
    m = mn;
  }
  // merge the 8 edge slots (lanes l ^ 8, ^ 16, ^ 32) in a fixed order
#pragma unroll
  for (int step = 0; step < 3; ++step) {
    float mo, lo, ao;
    if (step == 0) {
      mo = __uint_as_float(xlane_xor<8>(__float_as_uint(m)));
      lo = __uint_as_float(xlane_xor<8>(__float_as_uint(l)));
      ao = __uint_as_float(xlane_xor<8>(__float_as_uint(acc)));
    } else if (step == 1) {
      mo = __uint_as_float(xlane_xor<16>(__float_as_uint(m)));
      lo = __uint_as_float(xlane_xor<16>(__float_as_uint(l)));
      ao = __uint_as_float(xlane_xor<16>(__float_as_uint(acc)));
    } else {
      mo = __uint_as_float(xlane_xor<32>(__float_as_uint(m)));
      lo = __uint_as_float(xlane_xor<32>(__float_as_uint(l)));
      ao = __uint_as_float(xlane_xor<32>(__float_as_uint(acc)));
    }
    const float mn = fmaxf(m, mo);
    const float r1 = m == -INFINITY ? 0.f : expf(m - mn);
    const float r2 = mo == -INFINITY ? 0.f : expf(mo - mn);
    l = l * r1 + lo * r2;  // fp addition commutes: both partners hold the same bits
    acc = acc * r1 + ao * r2;
    m = mn;
  }
  }
  const float ft = acc / l;
  const float out = red_h_sum(ft) * (1.0f / H);
  if (lane == 0) c.seg_out[w] = out;
  if (TRAIN && j == 0) {
    float* sp = c.seg_stats + (int64_t)w * 4 * H;
    sp[h] = m;
    sp[H + h] = l;
    sp[2 * H + h] = ft;
    sp[3 * H + h] = er;
  }
  return out;
}
// eval: a wave per segment (train: the segments ride in tgnn_pred_train, three per event)
template <bool TRAIN>
__global__ void __launch_bounds__(256) tgnn_seg_fwd(Ctx c) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int S = (int)c.ctl[TGNX_CTL_S];
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= S) return;
  seg_fwd_one<TRAIN>(c, w, threadIdx.x & 63);
}

// ------------------------------------------------------------------ backward
// per segment: dx_eh from the saved logits (softmax + LeakyReLU + attn dropout backward),
// d er -> dU_r partials (persistent waves, deterministic workgroup reduction)
// Backward of tgnn_seg_fwd (a wave per segment, lane = 8 edge slots x 8 heads): dx of every edge
// (-> DX), d er_h, and the partials of dU_r (= Σ der_h ⊗ drop(mem[root])) and dc_r, written as a
// compact slab [H*D + H] per workgroup.
__device__ void seg_bwd_body(const Ctx& c, const int bid, const int nblk) {
  constexpr int KD = DMAX / 8;
  __shared__ float part[4][H * DMAX + H];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const bool okb = B > 0 && c.ctl[TGNX_CTL_ERR] == 0;
  const int S = okb ? (int)c.ctl[TGNX_CTL_S] : 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, j = lane >> 3, h = lane & 7;
  const int D = c.D;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const bool drop = c.drop;
  float aUr[KD], acr = 0.f;
#pragma unroll
  for (int k = 0; k < KD; ++k) aUr[k] = 0.f;
  for (int w = bid * 4 + wv; w < S; w += nblk * 4) {
    const float g = c.seg_g[w];
    if (g == 0.f) continue;
    Seg s;
    seg_of(c, w, lo, hi, start, s);
    const float gh = g * (1.0f / H);
    const float* sp = c.seg_stats + (int64_t)w * 4 * H;
    const float m = sp[h], l = sp[H + h], ft = sp[2 * H + h], er = sp[3 * H + h];
    const int e0 = c.seg_eoff[w], ne = c.seg_eoff[w + 1] - e0;
    const uint64_t sk = seg_key(s.blk, s.root);
    float der = 0.f;
    if (ne > SEG_WIDE) {  // (wave-uniform) lane = edge slot, all heads per lane (as tgnn_seg_fwd's long segments)
      float mh[H], lh[H], fh[H], eh[H], dh[H];
#pragma unroll
      for (int k = 0; k < H; ++k) {
        mh[k] = sp[k];
        lh[k] = sp[H + k];
        fh[k] = sp[2 * H + k];
        eh[k] = sp[3 * H + k];
        dh[k] = 0.f;
      }
      const float* __restrict__ Xr = c.X + (int64_t)e0 * H;
      float* __restrict__ DXr = c.DX + (int64_t)e0 * H;
      for (int o = lane; o < ne; o += WAVE) {
        float xv[H], dx[H];
        load_row8(Xr + (int64_t)o * H, xv);
        const uint32_t ab = drop ? attn_base(seed, sk, o) : 0u;
#pragma unroll
        for (int k = 0; k < H; ++k) {
          float sc = xv[k] + eh[k];
          const float lk = sc > 0.f ? 1.f : 0.2f;
          sc = sc > 0.f ? sc : 0.2f * sc;
          const float a = expf(sc - mh[k]) / lh[k];
          const float mk = drop ? keep32(ab, (uint32_t)k, c.pa, c.inv_ka) : 1.f;
          const float ds = a * gh * (xv[k] * mk - fh[k]) * lk;
          dx[k] = gh * a * mk + ds;
          dh[k] += ds;
        }
        float4* dp = reinterpret_cast<float4*>(DXr + (int64_t)o * H);
        dp[0] = make_float4(dx[0], dx[1], dx[2], dx[3]);
        dp[1] = make_float4(dx[4], dx[5], dx[6], dx[7]);
      }
#pragma unroll
      for (int st = 1; st < WAVE; st <<= 1)
#pragma unroll
        for (int k = 0; k < H; ++k) dh[k] += __shfl_xor(dh[k], st, WAVE);
      der = pick8(dh, h);
    } else {
      const float* __restrict__ X = c.X + (int64_t)e0 * H + h;
      float* __restrict__ DXp = c.DX + (int64_t)e0 * H + h;
#pragma unroll 4
      for (int o = j; o < ne; o += 8) {
        const float x = X[(int64_t)o * H];
        float sc = x + er;
        const float lk = sc > 0.f ? 1.f : 0.2f;
        sc = sc > 0.f ? sc : 0.2f * sc;
        const float a = expf(sc - m) / l;
        const float mk = drop ? keep32(attn_base(seed, sk, o), (uint32_t)h, c.pa, c.inv_ka) : 1.f;
        const float ds = a * gh * (x * mk - ft) * lk;
        DXp[(int64_t)o * H] = gh * a * mk + ds;
        der += ds;
      }
      der = red_j_sum(der);
    }
    const uint32_t nb = drop ? node_base(seed, s.blk, s.root) : 0u;
    float mv[KD];
#pragma unroll
    for (int k = 0; k < KD; ++k) mv[k] = c.mem[s.root * D + min(j + 8 * k, D - 1)];
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      float v = mv[k];
      if (drop) v *= keep32(nb, (uint32_t)(j + 8 * k), c.pf, c.inv_kf);
      aUr[k] += der * v;
    }
    acr += der;
  }
  float* pw = part[wv];
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int dd = j + 8 * k;
    if (dd < D) pw[h * D + dd] = aUr[k];
  }
  if (j == 0) pw[H * D + h] = acr;
  __syncthreads();
  const int n = H * D + H;
  float* slab = c.slabs_s + (int64_t)bid * n;
  for (int p = threadIdx.x; p < n; p += blockDim.x) slab[p] = (part[0][p] + part[1][p]) + (part[2][p] + part[3][p]);
}

// dU_e, dU_l, dw, db, dc_e, dc_l partials of the edge terms (backward of tgnn_edge_fwd).
// Lanes own feature columns and waves stride over edges, so every reduction over edges stays in
// registers.  Column classes are compile-time (CF feature columns, CT time-encoding columns, CT
// memory columns); gathers use clamped indices (values of lanes past the end are never written
// out), the self-loop row points at a row of ones: the loop body has no divergent control flow.
// Two register sets ping-pong so one edge's gathers are in flight during the other's math.  Each
// wave leaves its partial in LDS and the workgroup sums them in a fixed order into its slab.
template <int CF, int CT, bool DROP, int NW>
__global__ void __launch_bounds__(64 * NW) tgnn_edge_bwd(Ctx c) {
  constexpr int BWD_BUFS = bwd_bufs(NW);
  static_assert(NW <= 2 * BWD_BUFS, "edge backward: at most two waves per LDS partial row");
  constexpr int NJ = CF + 2 * CT;
  extern __shared__ __attribute__((aligned(16))) float part[];   // [BWD_BUFS][PL.total]
  __shared__ __attribute__((aligned(16))) float Uenc[DMAX * H];   // U_e[h][d + i] as [i][h], zero for i >= D
  const PLay PL = c.PL;
  const int F = c.F, D = c.D, d = c.d;
  for (int x = threadIdx.x; x < DMAX * H; x += blockDim.x) {
    const int i = x / H, h = x % H;
    Uenc[x] = i < D ? c.U[c.UL.Ue + h * F + d + i] : 0.f;
  }
  const int B = (int)c.ctl[TGNX_CTL_B];
  const bool okb = B > 0 && c.ctl[TGNX_CTL_ERR] == 0;
  const int E = okb ? (int)c.ctl[TGNX_CTL_E] : 0;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const EdgeCols<CF, CT> cols(lane, d, D);
  float aU[NJ][H], tw[CT], tb[CT], aw[CT], ab[CT], ac[H];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int h = 0; h < H; ++h) aU[j][h] = 0.f;
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    const int i = lane + 64 * j;
    tw[j] = i < D ? c.params[c.L.te_w + i] : 0.f;
    tb[j] = i < D ? c.params[c.L.te_b + i] : 0.f;
    aw[j] = ab[j] = 0.f;
  }
#pragma unroll
  for (int h = 0; h < H; ++h) ac[h] = 0.f;
  __syncthreads();

  struct Slot {
    EdgeVals<CF, CT> g;
    float dx[H];
  };
  auto load = [&](int e, Slot& S) {
    edge_gather(c, e, cols, S.g);
    load_x8(c.DX + (int64_t)e * H, S.dx);
  };
  auto math = [&](const Slot& S) {
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      float x = S.g.vf[j];
      if (DROP) x *= keep32(S.g.eb, (uint32_t)(lane + 64 * j), c.pf, c.inv_kf);
#pragma unroll
      for (int h = 0; h < H; ++h) aU[j][h] += S.dx[h] * x;
    }
#pragma unroll
    for (int j = 0; j < CT; ++j) {  // time encoding dim i: x = cos(w_i dt + b_i)  (model_utils.py:235)
      const int i = lane + 64 * j;
      float sn, cs;
      te_sincos(fmaf(tw[j], S.g.dt, tb[j]), sn, cs);
      const float km = DROP ? keep32(S.g.eb, (uint32_t)(d + i), c.pf, c.inv_kf) : 1.f;
      const float x = cs * km;
#pragma unroll
      for (int h = 0; h < H; ++h) aU[CF + j][h] += S.dx[h] * x;
      const float4 u0 = *reinterpret_cast<const float4*>(&Uenc[(i & (DMAX - 1)) * H]);
      const float4 u1 = *reinterpret_cast<const float4*>(&Uenc[(i & (DMAX - 1)) * H + 4]);
      const float denc = S.dx[0] * u0.x + S.dx[1] * u0.y + S.dx[2] * u0.z + S.dx[3] * u0.w +
                         S.dx[4] * u1.x + S.dx[5] * u1.y + S.dx[6] * u1.z + S.dx[7] * u1.w;
      const float gz = -denc * km * sn;
      aw[j] += gz * S.g.dt;
      ab[j] += gz;
    }
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      float x = S.g.vm[j];
      if (DROP) x *= keep32(S.g.nb, (uint32_t)(lane + 64 * j), c.pf, c.inv_kf);
#pragma unroll
      for (int h = 0; h < H; ++h) aU[CF + CT + j][h] += S.dx[h] * x;
    }
#pragma unroll
    for (int h = 0; h < H; ++h) ac[h] += S.dx[h];
  };

  const int stride = gridDim.x * NW;
  int e = blockIdx.x * NW + wv;
  Slot A, Bs;
  if (e < E) load(e, A);
  while (e < E) {
    const int e1 = e + stride;
    if (e1 < E) load(e1, Bs);
    math(A);
    if (e1 >= E) break;
    const int e2 = e1 + stride;
    if (e2 < E) load(e2, A);
    math(Bs);
    e = e2;
  }
  // this wave's partial -> LDS row wv (entries owned by nobody are zeroed in the sum below); waves past BWD_BUFS
  // add theirs into row wv - BWD_BUFS once the first BWD_BUFS have stored (each lane owns the same entries)
  auto put = [&](float* pw, auto st) {
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      const int f = lane + 64 * j;
      if (f < d)
#pragma unroll
        for (int h = 0; h < H; ++h) st(pw + PL.Ue + h * F + f, aU[j][h]);
    }
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      const int i = lane + 64 * j;
      if (i < D) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          st(pw + PL.Ue + h * F + d + i, aU[CF + j][h]);
          st(pw + PL.Ul + h * D + i, aU[CF + CT + j][h]);
        }
        st(pw + PL.w + i, aw[j]);
        st(pw + PL.b + i, ab[j]);
      }
    }
    if (lane == 0)
#pragma unroll
      for (int h = 0; h < H; ++h) {
        st(pw + PL.ce + h, ac[h]);
        st(pw + PL.cl + h, ac[h]);
      }
  };
  if (wv < BWD_BUFS) put(part + wv * PL.total, [](float* q, float v) { *q = v; });
  if constexpr (NW > BWD_BUFS) {
    __syncthreads();
    if (wv >= BWD_BUFS) put(part + (wv - BWD_BUFS) * PL.total, [](float* q, float v) { *q += v; });
  }
  __syncthreads();
  float* slab = c.slabs + (int64_t)blockIdx.x * PL.total;
  for (int p = threadIdx.x; p < PL.total; p += blockDim.x) {
    float s = 0.f;
    const bool owned = (p < PL.Ur) || (p >= PL.ce && p < PL.cr) || p >= PL.w;
    if (owned)
#pragma unroll
      for (int w = 0; w < BWD_BUFS; ++w) s += part[w * PL.total + p];
    slab[p] = s;
  }
}

template <int CF, int CT, bool DROP, int NW>
static void launch_edge_bwd_nw(const Ctx& c, hipStream_t s) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)tgnn_edge_bwd<CF, CT, DROP, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              150 * 1024);
    return true;
  }();
  (void)attr;
  const size_t shp = (size_t)bwd_bufs(NW) * c.PL.total * 4;
  tgnn_edge_bwd<CF, CT, DROP, NW><<<GBWD, 64 * NW, shp, s>>>(c);
}
template <int CF, int CT, bool DROP>
static void launch_edge_bwd_t(const Ctx& c, size_t, hipStream_t s) {
  if (c.Bmax >= TGNX_BIG_BATCH) launch_edge_bwd_nw<CF, CT, DROP, 12>(c, s);
  else launch_edge_bwd_nw<CF, CT, DROP, BWD_WAVES>(c, s);
}
template <int CF>
static void launch_edge_bwd_cf(const Ctx& c, size_t shp, hipStream_t s) {
  const bool two = c.D > 64;
  if (c.drop) two ? launch_edge_bwd_t<CF, 2, true>(c, shp, s) : launch_edge_bwd_t<CF, 1, true>(c, shp, s);
  else two ? launch_edge_bwd_t<CF, 2, false>(c, shp, s) : launch_edge_bwd_t<CF, 1, false>(c, shp, s);
}
static void launch_edge_bwd(const Ctx& c, hipStream_t s) {
  const size_t shp = 0;  // (per wave count: launch_edge_bwd_nw)
  switch ((c.d + 63) / 64) {
    case 0: launch_edge_bwd_cf<0>(c, shp, s); break;
    case 1: launch_edge_bwd_cf<1>(c, shp, s); break;
    case 2: launch_edge_bwd_cf<2>(c, shp, s); break;
    case 3: launch_edge_bwd_cf<3>(c, shp, s); break;
    case 4: launch_edge_bwd_cf<4>(c, shp, s); break;
    default: launch_edge_bwd_cf<5>(c, shp, s); break;
  }
}

// Sum the partial slabs in a fixed order (deterministic): a workgroup owns 64 consecutive outputs
// (one per lane, coalesced rows), its 16 waves take every 16th slab, LDS combines the waves.
constexpr int RED_WAVES = 16;
__global__ void __launch_bounds__(64 * RED_WAVES) tgnn_grad_reduce(Ctx c, int Ge, int Gs) {
  __shared__ float acc[RED_WAVES][64];
  const PLay PL = c.PL;
  const int P = PL.total;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + lane;
  // segment slabs are compact [dU_r (H*D) | dc_r (H)]
  const int HD = H * c.D, ns = HD + H;
  const int q = (p >= PL.Ur && p < PL.Ur + HD) ? p - PL.Ur : (p >= PL.cr && p < PL.cr + H) ? HD + (p - PL.cr) : -1;
  float s = 0.f;
  if (p < P) {
#pragma unroll 4
    for (int g = wv; g < Ge; g += RED_WAVES) s += c.slabs[(int64_t)g * P + p];
    if (q >= 0)
#pragma unroll 4
      for (int g = wv; g < Gs; g += RED_WAVES) s += c.slabs_s[(int64_t)g * ns + q];
  }
  acc[wv][lane] = s;
  if (c.defer && blockIdx.x == 0 && threadIdx.x == 64 * RED_WAVES - 1) {
    // deferred update: the loss sum, and the step's update recorded as pending for the next tgnn_assemble launch
    // (or tgnx_tgnn_apply_pending); an empty or failed step records none
    const int64_t B = c.ctl[TGNX_CTL_B];
    const bool ok = B > 0 && c.ctl[TGNX_CTL_ERR] == 0;
    if (ok) {
      double* loss = reinterpret_cast<double*>(c.ctl + TGNX_CTL_LOSS);
      *loss += (double)c.grads[c.L.total] * (double)B;
    }
    c.ctl[TGNX_CTL_APPLY] = ok ? c.ctl[TGNX_CTL_ADAM_T] : 0;
  }
  __syncthreads();
  if (wv == 0 && p < P) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < RED_WAVES; ++w) t += acc[w][lane];
    c.red[p] = t;
  }
}

// ------------------------------------------------------------------ predictor (train): one wave per event
__device__ __forceinline__ float softplus(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }

__global__ void __launch_bounds__(256) tgnn_pred_train(Ctx c) {
  // one workgroup per event; its 4 waves split the D-long contractions, LDS combines them in a
  // fixed order, wave 0 finishes the event
  __shared__ float se[3][DMAX];
  __shared__ float part[4][3][DMAX];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const int i = lo + blockIdx.x;
  if (B == 0 || i >= hi || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nloc = hi - lo;
  const int D = c.D;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const int blk = (int)c.ev_blk[start + i];
  // batches below TGNX_BIG_BATCH: the event's three segments (src, pos, neg: segments i, nloc + i, 2 nloc + i of
  // the rank's slice) by waves 0-2 — tgnn_seg_fwd's work, one launch fewer (B = 200 step 0.0918 -> 0.0884 ms; at
  // B = 2,000 the separate launch is faster, 1.061 vs 1.087: profiles/r6/r6ae_*)
  __shared__ float sv_l[3];
  if (c.seg_in_pred) {
    if (wv < 3) {
      const float o = seg_fwd_one<true>(c, wv * nloc + (i - lo), lane);
      if (lane == 0) sv_l[wv] = o;
    }
  } else if (tid < 3) {
    sv_l[tid] = c.seg_out[tid * nloc + (i - lo)];
  }
  __syncthreads();
  {
    const int64_t roots[3] = {c.ev_src[start + i], c.ev_dst[start + i], c.neg[start + i]};
    const float sv[3] = {sv_l[0], sv_l[1], sv_l[2]};
    for (int x = tid; x < 3 * D; x += blockDim.x) {
      const int r = x / D, dd = x % D;
      float v = c.mem[roots[r] * D + dd];
      if (c.drop) v *= node_keep(c, seed, blk, roots[r], dd);
      se[r][dd] = v + sv[r];
    }
  }
  __syncthreads();
  const float* P = c.params;
  {
    // wave wv owns rows [d0, d0 + kc) of the contraction (kc <= DMAX / 4): all its weight loads are
    // issued before any FMA, so one memory latency covers the chunk
    constexpr int KC = DMAX / 4;
    const int kc = (D + 3) / 4, d0 = wv * kc, n = min(D - d0, kc);
    const float* WsT = c.U + c.UL.WsT;
    const float* WdT = c.U + c.UL.WdT;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      const int oc = o < D ? o : D - 1;
      float ws[KC], wd[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const int dd = d0 + (j < n ? j : 0);
        ws[j] = WsT[dd * D + oc];
        wd[j] = WdT[dd * D + oc];
      }
      float a = 0.f, b = 0.f, d2 = 0.f;
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        if (j < n) {
          a += ws[j] * se[0][d0 + j];
          b += wd[j] * se[1][d0 + j];
          d2 += wd[j] * se[2][d0 + j];
        }
      }
      if (o < D) {
        part[wv][0][o] = a;
        part[wv][1][o] = b;
        part[wv][2][o] = d2;
      }
    }
  }
  __syncthreads();
  if (wv != 0) return;
  float hs[2], hp[2], hn[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int o = lane + 64 * q;
    float a = 0.f, b = 0.f, d2 = 0.f;
    if (o < D) {
      a = P[c.L.bs + o] + ((part[0][0][o] + part[1][0][o]) + (part[2][0][o] + part[3][0][o]));
      b = P[c.L.bd + o] + ((part[0][1][o] + part[1][1][o]) + (part[2][1][o] + part[3][1][o]));
      d2 = P[c.L.bd + o] + ((part[0][2][o] + part[1][2][o]) + (part[2][2][o] + part[3][2][o]));
    }
    hs[q] = a; hp[q] = b; hn[q] = d2;
  }
  float hpos[2], hneg[2], zp = 0.f, zn = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int o = lane + 64 * q;
    hpos[q] = fmaxf(hs[q] + hp[q], 0.f);
    hneg[q] = fmaxf(hs[q] + hn[q], 0.f);
    if (o < D) {
      zp += P[c.L.Wo + o] * hpos[q];
      zn += P[c.L.Wo + o] * hneg[q];
    }
  }
  zp = wave_sum(zp) + P[c.L.bo];
  zn = wave_sum(zn) + P[c.L.bo];
  const float invB = 1.0f / (float)B;
  const float dzp = (1.0f / (1.0f + expf(-zp)) - 1.0f) * invB;
  const float dzn = (1.0f / (1.0f + expf(-zn))) * invB;
  const float li = (softplus(-zp) + softplus(zn)) * invB;
  float* ev = c.evs + (int64_t)i * (8 * D + 4);
  float gs = 0.f, gp = 0.f, gn = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int o = lane + 64 * q;
    if (o < D) {
      const float wo = P[c.L.Wo + o];
      const float dhp = hpos[q] > 0.f ? dzp * wo : 0.f;
      const float dhn = hneg[q] > 0.f ? dzn * wo : 0.f;
      const float A = dhp + dhn;
      gs += A * c.U[c.UL.Ws1 + o];
      gp += dhp * c.U[c.UL.Wd1 + o];
      gn += dhn * c.U[c.UL.Wd1 + o];
      ev[0 * D + o] = A;
      ev[1 * D + o] = se[0][o];
      ev[2 * D + o] = dhp;
      ev[3 * D + o] = se[1][o];
      ev[4 * D + o] = dhn;
      ev[5 * D + o] = se[2][o];
      ev[6 * D + o] = hpos[q];
      ev[7 * D + o] = hneg[q];
    }
  }
  gs = wave_sum(gs);
  gp = wave_sum(gp);
  gn = wave_sum(gn);
  if (lane == 0) {
    c.seg_g[i - lo] = gs;
    c.seg_g[nloc + i - lo] = gp;
    c.seg_g[2 * nloc + i - lo] = gn;
    c.out_pos[i] = zp;
    c.out_neg[i] = zn;
    if (c.out_ev) {
      const int64_t e = c.ctl[TGNX_CTL_BATCH_START] + i;
      c.out_ev[2 * e] = zp;
      c.out_ev[2 * e + 1] = zn;
    }
    ev[8 * D + 0] = dzp;
    ev[8 * D + 1] = dzn;
    ev[8 * D + 2] = li;
  }
}

// predictor weight gradients dWs = Σ_i A_i ⊗ e_s,i and dWd = Σ_i dhp_i ⊗ e_p,i + dhn_i ⊗ e_n,i:
// AᵀB products over the events, one 16x16 output tile per wave on v_mfma_f32_16x16x4_f32
// (exact fp32, k-ordered fmaf chain).  Grid: 2 * ceil(D/16)^2 waves.
__device__ void pred_reduce_vec_body(const Ctx& c, int y, int lane);

__device__ void pred_reduce_body(const Ctx& c, const int bid) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __shared__ f32x4 part[4][64];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int D = c.D;
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const bool ok = B > 0 && c.ctl[TGNX_CTL_ERR] == 0;
  const int nt = (D + 15) / 16;
  if (bid >= 2 * nt * nt) {  // trailing blocks: bias / output-layer / loss sums
    pred_reduce_vec_body(c, (bid - 2 * nt * nt) * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
    return;
  }
  const int which = bid / (nt * nt);
  const int t = bid % (nt * nt), tm = t / nt, tn = t % nt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int S = 8 * D + 4;
  const int m = tm * 16 + (lane & 15), n = tn * 16 + (lane & 15), kk = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int npass = which == 0 ? 1 : 2;
  for (int pass = 0; pass < npass && ok; ++pass) {
    // which 0: A = cols [0,D) (dhp+dhn), B = cols [D,2D) (e_s)
    // which 1: pass 0: A = [2D,3D) dhp, B = [3D,4D) e_p ; pass 1: A = [4D,5D) dhn, B = [5D,6D) e_n
    const int ca = which == 0 ? 0 : (pass == 0 ? 2 * D : 4 * D);
    const int cb = which == 0 ? D : (pass == 0 ? 3 * D : 5 * D);
    // k-steps of 4 events; wave wv takes steps wv, wv+4, ...; 8 steps' loads in flight
    for (int s0 = lo + 4 * wv; s0 < hi; s0 += 4 * 4 * 8) {
      float a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = s0 + 16 * u + kk;
        const bool in = i < hi;
        a[u] = (in && m < D) ? c.evs[(int64_t)i * S + ca + m] : 0.f;
        b[u] = (in && n < D) ? c.evs[(int64_t)i * S + cb + n] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc, 0, 0, 0);
    }
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv != 0) return;
  acc = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
  float* out = c.grads + (which == 0 ? c.L.Ws : c.L.Wd);
  const int col = tn * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = tm * 16 + (lane >> 4) * 4 + r;
    if (row < D && col < D) out[(int64_t)row * D + col] = acc[r];
  }
}

// segment backward (blocks [0, GSEG)) and the predictor weight reductions (the rest) in one launch:
// both only need tgnn_pred_train's per-event rows
__global__ void __launch_bounds__(256) tgnn_seg_bwd_pred(Ctx c, int nseg) {
  if ((int)blockIdx.x < nseg) seg_bwd_body(c, blockIdx.x, nseg);
  else pred_reduce_body(c, blockIdx.x - nseg);
}
__host__ __device__ inline int pred_reduce_blocks(int D) {
  const int nt = (D + 15) / 16;
  return 2 * nt * nt + (3 * D + 2 + 3) / 4;
}

// predictor bias / output-layer gradients and the batch loss: one wave per output, lanes over events
__device__ void pred_reduce_vec_body(const Ctx& c, int y, int lane) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int D = c.D;
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const bool ok = B > 0 && c.ctl[TGNX_CTL_ERR] == 0;
  if (y >= 3 * D + 2) return;
  const int S = 8 * D + 4;
  float acc = 0.f;
  for (int i = lo + lane; ok && i < hi; i += 64) {
    const float* e = c.evs + (int64_t)i * S;
    if (y < D) acc += e[y];                                                  // dbs = Σ (dhp + dhn)
    else if (y < 2 * D) acc += e[2 * D + y - D] + e[4 * D + y - D];          // dbd
    else if (y < 3 * D) acc += e[8 * D] * e[6 * D + y - 2 * D] + e[8 * D + 1] * e[7 * D + y - 2 * D];  // dWo
    else if (y == 3 * D) acc += e[8 * D] + e[8 * D + 1];                     // dbo
    else acc += e[8 * D + 2];                                                // batch loss
  }
  acc = wave_sum(acc);
  if (lane != 0) return;
  if (y < D) c.grads[c.L.bs + y] = acc;
  else if (y < 2 * D) c.grads[c.L.bd + y - D] = acc;
  else if (y < 3 * D) c.grads[c.L.Wo + y - 2 * D] = acc;
  else if (y == 3 * D) c.grads[c.L.bo] = acc;
  else c.grads[c.L.total] = acc;
}

// re-expand the collapsed gradients into the reference's parameters
// a*x + b*y with one fixed rounding order, so the folded-Adam expansion (tgnn_expand_adam) is bit-identical to it
__device__ __forceinline__ float dot2(float a, float x, float b, float y) { return __fmaf_rn(b, y, __fmul_rn(a, x)); }
__device__ void grad_attn_body(const Ctx& c, int y, int lane);

// blocks [0, nexp): elementwise dU -> dW / db re-expansion; trailing blocks: d attn (wave per output)
__global__ void __launch_bounds__(256) tgnn_grad_expand(Ctx c, int nexp) {
  if ((int)blockIdx.x >= nexp) {
    grad_attn_body(c, ((int)blockIdx.x - nexp) * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
    return;
  }
  const Lay L = c.L;
  const PLay PL = c.PL;
  const int D = c.D, F = c.F;
  const float* P = c.params;
  const float* r = c.red;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < L.Ws; x += (int64_t)nexp * blockDim.x) {
    float g = 0.f;
    if (x >= L.te_w && x < L.te_w + D) {
      g = r[PL.w + (x - L.te_w)];
    } else if (x >= L.te_b && x < L.te_b + D) {
      g = r[PL.b + (x - L.te_b)];
    } else if (x >= L.attn_l && x < L.Wn) {
      continue;  // tgnn_grad_attn
    } else if (x >= L.Wn && x < L.Wn + (int64_t)H * D * D) {
      const int64_t y = x - L.Wn;
      const int j = (int)(y / D), k = (int)(y % D), h = j / D;
      g = dot2(P[L.attn_l + j], r[PL.Ul + h * D + k], P[L.attn_r + j], r[PL.Ur + h * D + k]);
    } else if (x >= L.bn && x < L.bn + H * D) {
      const int j = (int)(x - L.bn), h = j / D;
      g = dot2(P[L.attn_l + j], r[PL.cl + h], P[L.attn_r + j], r[PL.cr + h]);
    } else if (x >= L.We && x < L.We + (int64_t)H * D * F) {
      const int64_t y = x - L.We;
      const int j = (int)(y / F), f = (int)(y % F), h = j / D;
      g = P[L.attn_e + j] * r[PL.Ue + h * F + f];
    } else if (x >= L.be && x < L.be + H * D) {
      const int j = (int)(x - L.be), h = j / D;
      g = P[L.attn_e + j] * r[PL.ce + h];
    }
    c.grads[x] = g;
  }
}

// d attn_{l,r}[h,d] = W_n[hD+d,:]·dU_{l,r}[h,:] + b_n[hD+d]·dc ; d attn_e likewise with W_e:
// one wave per output, lanes over the contraction
__device__ void grad_attn_body(const Ctx& c, int y, int lane) {
  const Lay L = c.L;
  const PLay PL = c.PL;
  const int D = c.D, F = c.F;
  if (y >= 3 * H * D) return;
  const int which = y / (H * D), j = y % (H * D), h = j / D;
  const float* P = c.params;
  const float* r = c.red;
  float g = 0.f;
  if (which < 2) {
    const float* dU = r + (which == 0 ? PL.Ul : PL.Ur) + h * D;
    const float* w = P + L.Wn + (int64_t)j * D;
    for (int k = lane; k < D; k += 64) g = __fmaf_rn(w[k], dU[k], g);
  } else {
    const float* dU = r + PL.Ue + h * F;
    const float* w = P + L.We + (int64_t)j * F;
    for (int f = lane; f < F; f += 64) g = __fmaf_rn(w[f], dU[f], g);
  }
  g = wave_sum(g);
  if (lane == 0) {
    if (which == 0) c.grads[L.attn_l + j] = __fmaf_rn(P[L.bn + j], r[PL.cl + h], g);
    else if (which == 1) c.grads[L.attn_r + j] = __fmaf_rn(P[L.bn + j], r[PL.cr + h], g);
    else c.grads[L.attn_e + j] = __fmaf_rn(P[L.be + j], r[PL.ce + h], g);
  }
}

// torch.optim.Adam (single-tensor form, same per-element operation order), bias corrections from
// the device step count, computed once per workgroup; 4 parameters per thread.
__device__ __forceinline__ void adam1(float g, float& m, float& v, float& p, float b1, float b2, float eps, float step,
                                      float bc2s) {
  // every operation rounded on its own (no contraction: the build's -ffp-contract=fast would otherwise fuse
  // differently per call site), in torch's order: lerp, mul + addcmul, sqrt / bc2 + eps, addcdiv — so the
  // separate Adam launch and the one folded into the expansion compute the same bits
#pragma clang fp contract(off)
  m = m + (1.0f - b1) * (g - m);
  v = v * b2 + ((1.0f - b2) * g) * g;
  const float den = __fsqrt_rn(v) / bc2s + eps;
  p = p - step * (m / den);
}
__global__ void __launch_bounds__(256) tgnn_adam(Ctx c) {
  __shared__ float sc[2];
  const int64_t B = c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  if (threadIdx.x == 0) {
    const int64_t t = c.ctl[TGNX_CTL_ADAM_T];
    const double bc1 = 1.0 - pow((double)c.b1, (double)t);
    const double bc2 = 1.0 - pow((double)c.b2, (double)t);
    sc[0] = (float)(c.lr / bc1);
    sc[1] = (float)sqrt(bc2);
    if (blockIdx.x == 0) {  // loss sum (slot after the parameters, all-reduced with them)
      double* loss = reinterpret_cast<double*>(c.ctl + TGNX_CTL_LOSS);
      *loss += (double)c.grads[c.L.total] * (double)B;
    }
  }
  __syncthreads();
  const float step = sc[0], bc2s = sc[1], b1 = c.b1, b2 = c.b2, eps = c.eps;
  const int64_t n4 = c.L.total / 4;  // layout is padded to multiples of 4
  float4* P4 = reinterpret_cast<float4*>(c.params);
  float4* M4 = reinterpret_cast<float4*>(c.am);
  float4* V4 = reinterpret_cast<float4*>(c.av);
  const float4* G4 = reinterpret_cast<const float4*>(c.grads);
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n4; x += (int64_t)gridDim.x * blockDim.x) {
    const float4 g = G4[x];
    float4 m = M4[x], v = V4[x], p = P4[x];
    adam1(g.x, m.x, v.x, p.x, b1, b2, eps, step, bc2s);
    adam1(g.y, m.y, v.y, p.y, b1, b2, eps, step, bc2s);
    adam1(g.z, m.z, v.z, p.z, b1, b2, eps, step, bc2s);
    adam1(g.w, m.w, v.w, p.w, b1, b2, eps, step, bc2s);
    M4[x] = m;
    V4[x] = v;
    P4[x] = p;
  }
}

// World 1: the gradient expansion with Adam folded in (tgnn_grad_expand + tgnn_attn grads + tgnn_adam in one launch).
// A wave owns W_n row j = (h, d) together with b_n[j], attn_l[j], attn_r[j] — the only elements whose old values its
// gradients read (d W_n[j, k] = attn_l[j] dU_l[h, k] + attn_r[j] dU_r[h, k]; d attn_l[j] = W_n[j, :]·dU_l[h, :] + b_n[j]
// dc_l[h]; d b_n[j] = attn_l[j] dc_l[h] + attn_r[j] dc_r[h]) — or W_e row j with b_e[j], attn_e[j]; so every old value
// is loaded before the same wave updates it and no other wave reads it.  The rest (te_w, te_b from the reduced
// partials; the predictor's gradients, final since tgnn_seg_bwd_pred) elementwise.  Same per-element gradient and
// Adam arithmetic as the three kernels (the gradient buffer is written as well).
__device__ __forceinline__ void adam_store(const Ctx& c, int64_t x, float g, float m, float v, float p, float step,
                                           float bc2s) {
  adam1(g, m, v, p, c.b1, c.b2, c.eps, step, bc2s);
  c.grads[x] = g;
  c.am[x] = m;
  c.av[x] = v;
  c.params[x] = p;
}
__device__ __forceinline__ void adam_at(const Ctx& c, int64_t x, float g, float step, float bc2s) {
  adam_store(c, x, g, c.am[x], c.av[x], c.params[x], step, bc2s);
}
// Adam's step scalars from the device step count (every wave computes them itself: no barrier, and the double-
// precision pow runs while the wave's loads are in flight)
__device__ __forceinline__ void adam_scalars(const Ctx& c, int64_t t, float& step, float& bc2s) {
  const double bc1 = 1.0 - pow((double)c.b1, (double)t);
  const double bc2 = 1.0 - pow((double)c.b2, (double)t);
  step = (float)(c.lr / bc1);
  bc2s = (float)sqrt(bc2);
}
template <int NR>
__device__ __forceinline__ void expand_row_adam(const Ctx& c, int j, int lane, bool edge, int64_t t) {
  const Lay L = c.L;
  const PLay PL = c.PL;
  const int D = c.D, F = c.F, h = j / D;
  const int W = edge ? F : D;
  float* P = c.params;
  const float* r = c.red;
  const int64_t row = (edge ? L.We : L.Wn) + (int64_t)j * W;
  // every old value first — the row, its bias, its attention element(s), the row's reduced dU, and the Adam moments
  // of all of them — in one load round
  float w[NR], ua[NR], ub[NR], mm[NR], vv[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int k = min(lane + 64 * i, W - 1);
    w[i] = P[row + k];
    mm[i] = c.am[row + k];
    vv[i] = c.av[row + k];
    ua[i] = edge ? r[PL.Ue + h * F + k] : r[PL.Ul + h * D + k];
    ub[i] = edge ? 0.f : r[PL.Ur + h * D + k];
  }
  const int64_t xa = (edge ? L.attn_e : L.attn_l) + j, xr = L.attn_r + j, xb = (edge ? L.be : L.bn) + j;
  const float a0 = P[xa], a1 = edge ? 0.f : P[xr];
  const float bj = P[xb];
  const float c0 = r[(edge ? PL.ce : PL.cl) + h], c1 = edge ? 0.f : r[PL.cr + h];
  const float ma = c.am[xa], va = c.av[xa], mb = c.am[xb], vb = c.av[xb];
  const float mr = edge ? 0.f : c.am[xr], vr = edge ? 0.f : c.av[xr];
  float step, bc2s;
  adam_scalars(c, t, step, bc2s);
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < NR; ++i)
    if (lane + 64 * i < W) {
      s0 = __fmaf_rn(w[i], ua[i], s0);
      s1 = __fmaf_rn(w[i], ub[i], s1);
    }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int k = lane + 64 * i;
    if (k < W)
      adam_store(c, row + k, edge ? a0 * ua[i] : dot2(a0, ua[i], a1, ub[i]), mm[i], vv[i], w[i], step, bc2s);
  }
  if (lane == 0) {
    adam_store(c, xa, __fmaf_rn(bj, c0, s0), ma, va, a0, step, bc2s);
    if (!edge) adam_store(c, xr, __fmaf_rn(bj, c1, s1), mr, vr, a1, step, bc2s);
    adam_store(c, xb, edge ? a0 * c0 : dot2(a0, c0, a1, c1), mb, vb, bj, step, bc2s);
  }
}
// The expansion + Adam of update step t over `nblk` workgroups of any size: the first `nel` elementwise (te_w, te_b,
// the predictor block [Ws, total)), the rest a wave per W_n / W_e row.
__device__ void expand_adam_body(const Ctx& c, int64_t t, int bid, int nblk, int nel) {
  const Lay L = c.L;
  const PLay PL = c.PL;
  const int D = c.D, lane = threadIdx.x & 63, T = blockDim.x;
  if (bid < nel) {
    float step, bc2s;
    adam_scalars(c, t, step, bc2s);
    const int64_t n = 2 * D + (L.total - L.Ws);
    for (int64_t y = bid * (int64_t)T + threadIdx.x; y < n; y += (int64_t)nel * T) {
      if (y < D) adam_at(c, L.te_w + y, c.red[PL.w + y], step, bc2s);
      else if (y < 2 * D) adam_at(c, L.te_b + y - D, c.red[PL.b + y - D], step, bc2s);
      else {
        const int64_t x = L.Ws + y - 2 * D;
        adam_at(c, x, c.grads[x], step, bc2s);
      }
    }
    return;
  }
  const int wpb = T >> 6, nw = (nblk - nel) * wpb;
  for (int wv = (bid - nel) * wpb + (threadIdx.x >> 6); wv < 2 * H * D; wv += nw) {  // (wave-uniform)
    if (wv < H * D) expand_row_adam<(DMAX + 63) / 64>(c, wv, lane, false, t);
    else expand_row_adam<(FMAX + 63) / 64>(c, wv - H * D, lane, true, t);
  }
}
__host__ __device__ inline int expand_rows_blocks(int D, int threads) { return (2 * H * D + threads / 64 - 1) / (threads / 64); }

__global__ void __launch_bounds__(256) tgnn_expand_adam(Ctx c, int nelem_blocks) {
  const int64_t B = c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;   // (as tgnn_adam: no update for an empty batch)
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // loss sum (the slot after the parameters)
    double* loss = reinterpret_cast<double*>(c.ctl + TGNX_CTL_LOSS);
    *loss += (double)c.grads[c.L.total] * (double)B;
  }
  expand_adam_body(c, c.ctl[TGNX_CTL_ADAM_T], blockIdx.x, gridDim.x, nelem_blocks);
}
// the pending (deferred) update, if any: tgnx_tgnn_apply_pending and tgnx_tgnn_eval_step's first launch
__global__ void __launch_bounds__(256) tgnn_apply_pending(Ctx c, int nelem_blocks) {
  const int64_t t = c.ctl[TGNX_CTL_APPLY];
  if (t <= 0) return;
  expand_adam_body(c, t, blockIdx.x, gridDim.x, nelem_blocks);
}
__global__ void tgnn_clear_pending(int64_t* ctl) {
  if (threadIdx.x == 0) ctl[TGNX_CTL_APPLY] = 0;
}

// Ring/time state update of a batch (many workgroups): time_assoc of the touched nodes
// (model_utils.py:77-83) and the ring insert of the whole batch with a wave per node run of
// tgnn_assemble's plan.
template <bool TRAIN>
__device__ void finish_body(const Ctx& c, const int bid, const int nblk) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  const float* evt = c.ev_t + start;
  const int NT = TRAIN ? 3 * B : 2 * B;
  const int gt = bid * blockDim.x + threadIdx.x, gs = nblk * blockDim.x;
  if (TRAIN) {  // final time_assoc = last assignment of each touched node
    for (int j = gt; j < NT; j += gs) {
      const uint64_t k = c.touches[j];
      if (j == NT - 1 || knode(c.touches[j + 1]) != knode(k)) c.ta[knode(k)] = evt[kev(k)];
    }
  } else {      // after tgnn_ta_fill: s/p of the last block keep their own t, the later assignment
    const int kmax = c.misc[MISC_KMAX];  // (s after p, batch order) wins = last of its (node, block) group
    for (int j = gt; j < NT; j += gs) {
      const uint64_t k = c.touches[j];
      if (kblk(k) == kmax && (j == NT - 1 || (c.touches[j + 1] >> 14) != (k >> 14))) c.ta[knode(k)] = evt[kev(k)];
    }
  }
  const int U = c.misc[MISC_RUNS];
  const int r = bid * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r < U) {
    const int a = c.rruns[r];
    ring_merge_run(c.nbr, c.eid, c.rt, c.K, c.ev_src + start, c.ev_dst + start, evt, B, c.ctl[TGNX_CTL_CUR_EID],
                   c.assoc, c.rkeys, a, c.rruns[r + 1] - a, r, threadIdx.x & 63);
  }
}
template <bool TRAIN>
__global__ void __launch_bounds__(256) tgnn_finish(Ctx c) {
  finish_body<TRAIN>(c, blockIdx.x, gridDim.x);
}
__host__ __device__ inline int finish_blocks(int Bmax) { return (2 * Bmax + 3) / 4; }

__global__ void tgnn_ta_fill(Ctx c) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const float v = c.blkmax[c.misc[MISC_KMAX]];
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < c.N; x += (int64_t)gridDim.x * blockDim.x)
    c.ta[x] = v;
}

// ------------------------------------------------------------------ eval predictor + MRR
// phase 1: one wave per event: source projection (kept in block order) and the positive logit
__global__ void __launch_bounds__(256) tgnn_pred_eval_src(Ctx c) {
  __shared__ float se[4][2][DMAX];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + wv;
  const bool active = B > 0 && i < B && c.ctl[TGNX_CTL_ERR] == 0;
  const int D = c.D;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  if (active) {
    const int64_t roots[2] = {c.ev_src[start + i], c.ev_dst[start + i]};
    const int segs[2] = {i, B + i};
    for (int r = 0; r < 2; ++r) {
      const float sv = c.seg_out[segs[r]];
      for (int dd = lane; dd < D; dd += 64) se[wv][r][dd] = c.mem[roots[r] * D + dd] + sv;
    }
  }
  __syncthreads();
  if (!active) return;
  const float* P = c.params;
  const int rho = c.blk_rank[i];
  float z = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int o = lane + 64 * q;
    if (o < D) {
      float a = P[c.L.bs + o], b = P[c.L.bd + o];
      for (int dd = 0; dd < D; ++dd) {
        a += c.U[c.UL.WsT + dd * D + o] * se[wv][0][dd];
        b += c.U[c.UL.WdT + dd * D + o] * se[wv][1][dd];
      }
      c.HS[(int64_t)rho * D + o] = a;
      z += P[c.L.Wo + o] * fmaxf(a + b, 0.f);
    }
  }
  z = wave_sum(z) + P[c.L.bo];
  if (lane == 0) c.out_pos[rho] = z;
}

// phase 2: one wave per negative row, rows in block order (model_utils.py:135-137, 159)
__global__ void __launch_bounds__(256) tgnn_pred_eval_neg(Ctx c) {
  __shared__ float se[4][DMAX];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int Kn = c.Kn;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + wv;
  const bool active = B > 0 && r < (int64_t)B * Kn && c.ctl[TGNX_CTL_ERR] == 0;
  const int D = c.D;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  int rho = 0;
  if (active) {
    rho = (int)(r / Kn);
    const int cc = (int)(r % Kn);
    const int i = c.blk_order[rho];
    const int64_t root = c.neg[(start + i) * Kn + cc];
    const float sv = c.seg_out[2 * B + i * Kn + cc];
    for (int dd = lane; dd < D; dd += 64) se[wv][dd] = c.mem[root * D + dd] + sv;
  }
  __syncthreads();
  if (!active) return;
  const float* P = c.params;
  const int srow = c.quirk ? (int)(r % B) : rho;   // h_src.tile(neg_samples, 1) (model_utils.py:192)
  float z = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int o = lane + 64 * q;
    if (o < D) {
      float b = P[c.L.bd + o];
      for (int dd = 0; dd < D; ++dd) b += c.U[c.UL.WdT + dd * D + o] * se[wv][dd];
      z += P[c.L.Wo + o] * fmaxf(c.HS[(int64_t)srow * D + o] + b, 0.f);
    }
  }
  z = wave_sum(z) + P[c.L.bo];
  if (lane == 0) c.out_neg[r] = z;
}

// TGB rank rule: rank = 0.5 (#neg > pos + #neg >= pos) + 1; batch MRR = mean 1/rank
__global__ void __launch_bounds__(1024) tgnn_mrr(Ctx c) {
  __shared__ double red[1024];
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int Kn = c.Kn;
  double s = 0.0;
  for (int rho = threadIdx.x; rho < B; rho += blockDim.x) {
    const float p = c.out_pos[rho];
    int gt = 0, ge = 0;
    const float* ng = c.out_neg + (int64_t)rho * Kn;
    for (int k = 0; k < Kn; ++k) {
      gt += ng[k] > p;
      ge += ng[k] >= p;
    }
    s += 1.0 / (0.5 * (gt + ge) + 1.0);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) c.mrr[(c.ctl[TGNX_CTL_NB] - 1) & (MRR_SLOTS - 1)] = red[0] / (double)B;
}

// ------------------------------------------------------------------ host glue
static size_t carve(size_t& off, size_t bytes) {
  size_t o = off;
  off += (bytes + 255) & ~size_t(255);
  return o;
}

struct WsLay {
  size_t touches, sp_pref, sp_keys, seg_cnt, seg_eoff, seg_out, seg_stats, seg_g, X, DX, meta, U, evs, slabs,
      slabs_s, red, blkmax, blk_rank, blk_order, HS, rkeys, rruns, misc, total;
  int64_t Ecap, Scap;
};
static WsLay make_ws(const tgnx_tgnn_config* cfg) {
  WsLay W;
  const int64_t B = cfg->max_batch, Kn = cfg->max_neg < 1 ? 1 : cfg->max_neg;
  const int D = cfg->mem_dim, d = cfg->msg_dim;
  W.Scap = B * (2 + (Kn > 1 ? Kn : 1));
  if (W.Scap < 3 * B) W.Scap = 3 * B;
  W.Ecap = W.Scap * (cfg->ring + 1) + 2 * B * B + 64;
  const int P = make_play(D, d).total;
  size_t off = 0;
  W.touches = carve(off, (size_t)TOUCH_MAX * 8);
  W.sp_pref = carve(off, (size_t)(TOUCH_MAX + 1) * 4);
  W.sp_keys = carve(off, (size_t)TOUCH_MAX * 8);
  W.seg_cnt = carve(off, (size_t)W.Scap * 4);
  W.seg_eoff = carve(off, (size_t)(W.Scap + 1) * 4);
  W.seg_out = carve(off, (size_t)W.Scap * 4);
  W.seg_stats = carve(off, (size_t)3 * B * 4 * H * 4);
  W.seg_g = carve(off, (size_t)3 * B * 4);
  W.X = carve(off, (size_t)W.Ecap * H * 4);
  W.DX = carve(off, (size_t)(3 * B * (cfg->ring + 1) + 2 * B * B + 64) * H * 4);
  W.meta = carve(off, (size_t)W.Ecap * sizeof(EdgeMeta));
  W.U = carve(off, (size_t)make_ulay(D, d).total * 4);
  W.evs = carve(off, (size_t)B * (8 * D + 4) * 4);
  W.slabs = carve(off, (size_t)GBWD * P * 4);
  W.slabs_s = carve(off, (size_t)gseg_for(cfg->max_batch) * (H * D + H) * 4);
  W.red = carve(off, (size_t)P * 4);
  W.blkmax = carve(off, (size_t)B * 4);
  W.blk_rank = carve(off, (size_t)B * 4);
  W.blk_order = carve(off, (size_t)B * 4);
  W.HS = carve(off, (size_t)B * D * 4);
  W.rkeys = carve(off, (size_t)2 * B * 8);
  W.rruns = carve(off, (size_t)(2 * B + 2) * 4);
  W.misc = carve(off, (size_t)MISC_WORDS * 4);
  W.total = off;
  return W;
}

static int check_cfg(const tgnx_tgnn_config* cfg) {
  TGNX_CHECK_ARG(cfg, "tgnn: null config");
  TGNX_CHECK_ARG(cfg->heads == H, "tgnn: heads must be %d (gnn.att_head), got %d", H, cfg->heads);
  TGNX_CHECK_ARG(cfg->mem_dim > 0 && cfg->mem_dim <= DMAX, "tgnn: mem_dim must be in [1, %d]", DMAX);
  TGNX_CHECK_ARG(cfg->msg_dim >= 0 && cfg->msg_dim + cfg->mem_dim <= FMAX, "tgnn: msg_dim + mem_dim must be <= %d",
                 FMAX);
  TGNX_CHECK_ARG(cfg->ring > 0 && cfg->ring <= KMAX && cfg->ring <= 64, "tgnn: ring size must be in [1, %d]", KMAX);
  TGNX_CHECK_ARG(cfg->max_batch > 0 && cfg->max_batch <= BATCH_MAX, "tgnn: max_batch must be in [1, %d]",
                 BATCH_MAX);
  TGNX_CHECK_ARG(cfg->num_nodes > 0 && cfg->num_nodes < (1ll << 37), "tgnn: bad num_nodes");
  return TGNX_OK;
}

static int make_ctx(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* b, int Kn, Ctx& c) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(b && b->ctl && b->ws && b->node_map && b->params && b->ev_src && b->ev_dst && b->ev_t && b->ev_blk,
                 "tgnn: null buffer");
  memset(&c, 0, sizeof(c));
  c.N = cfg->num_nodes;
  c.K = cfg->ring;
  c.D = cfg->mem_dim;
  c.d = cfg->msg_dim;
  c.F = c.d + c.D;
  c.Kn = Kn;
  c.pf = cfg->feat_drop;
  c.pa = cfg->attn_drop;
  c.inv_kf = cfg->feat_drop < 1.f ? 1.0f / (1.0f - cfg->feat_drop) : 0.f;
  c.inv_ka = cfg->attn_drop < 1.f ? 1.0f / (1.0f - cfg->attn_drop) : 0.f;
  c.lr = cfg->lr;
  c.b1 = cfg->beta1;
  c.b2 = cfg->beta2;
  c.eps = cfg->eps;
  c.ev_src = b->ev_src;
  c.ev_dst = b->ev_dst;
  c.ev_t = b->ev_t;
  c.ev_blk = b->ev_blk;
  c.ev_msg = b->ev_msg;
  c.neg = b->neg;
  c.dst_nodes = b->dst_nodes;
  c.n_dst = b->n_dst;
  c.feat = b->feat;
  c.nbr = b->nbr;
  c.eid = b->eid;
  c.rt = b->rt;
  c.assoc = b->assoc;
  c.ta = b->time_assoc;
  c.mem = b->memory;
  c.params = b->params;
  c.grads = b->grads;
  c.am = b->adam_m;
  c.av = b->adam_v;
  c.ctl = b->ctl;
  c.out_pos = b->out_pos;
  c.out_ev = b->out_ev;
  c.out_neg = b->out_neg;
  c.mrr = b->mrr;
  c.nodemap = reinterpret_cast<int4*>(b->node_map);
  WsLay W = make_ws(cfg);
  char* ws = reinterpret_cast<char*>(b->ws);
  c.touches = reinterpret_cast<uint64_t*>(ws + W.touches);
  c.sp_pref = reinterpret_cast<int*>(ws + W.sp_pref);
  c.sp_keys = reinterpret_cast<uint64_t*>(ws + W.sp_keys);
  c.seg_cnt = reinterpret_cast<int*>(ws + W.seg_cnt);
  c.seg_eoff = reinterpret_cast<int*>(ws + W.seg_eoff);
  c.seg_out = reinterpret_cast<float*>(ws + W.seg_out);
  c.seg_stats = reinterpret_cast<float*>(ws + W.seg_stats);
  c.seg_g = reinterpret_cast<float*>(ws + W.seg_g);
  c.X = reinterpret_cast<float*>(ws + W.X);
  c.DX = reinterpret_cast<float*>(ws + W.DX);
  c.meta = reinterpret_cast<EdgeMeta*>(ws + W.meta);
  c.U = reinterpret_cast<float*>(ws + W.U);
  c.evs = reinterpret_cast<float*>(ws + W.evs);
  c.slabs = reinterpret_cast<float*>(ws + W.slabs);
  c.slabs_s = reinterpret_cast<float*>(ws + W.slabs_s);
  c.red = reinterpret_cast<float*>(ws + W.red);
  c.blkmax = reinterpret_cast<float*>(ws + W.blkmax);
  c.blk_rank = reinterpret_cast<int*>(ws + W.blk_rank);
  c.blk_order = reinterpret_cast<int*>(ws + W.blk_order);
  c.HS = reinterpret_cast<float*>(ws + W.HS);
  c.rkeys = reinterpret_cast<uint64_t*>(ws + W.rkeys);
  c.rruns = reinterpret_cast<int*>(ws + W.rruns);
  c.misc = reinterpret_cast<int*>(ws + W.misc);
  c.Ecap = W.Ecap;
  c.Bmax = cfg->max_batch;
  c.Ge = GBWD;
  c.Gs = gseg_for(cfg->max_batch);
  c.L = make_lay(c.D, c.d);
  c.UL = make_ulay(c.D, c.d);
  c.PL = make_play(c.D, c.d);
  return TGNX_OK;
}

static inline int grid_for(int64_t n, int per) { return (int)((n + per - 1) / per); }


static int edge_grid(int64_t Ecap) {
  const int64_t g = (Ecap * 16 + 255) / 256;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

// assembly -> counts -> offsets -> edge metadata -> collapsed weights -> edge logits -> segment softmax
template <bool TRAIN>
static int launch_forward(const Ctx& c, int64_t Scap, hipStream_t s) {
  probe_begin(TGNX_K_ASSEMBLE, s);
  const int napply = TRAIN && c.defer ? c.apply_nel + expand_rows_blocks(c.D, 1024) : 0;
  tgnn_assemble<TRAIN><<<3 + napply, 1024, assemble_smem_bytes(c.Bmax), s>>>(c);
  probe_end(TGNX_K_ASSEMBLE, s);
  TGNX_LAUNCH_CHECK("tgnn_assemble");
  if (!TRAIN) {
    tgnn_seg_count<<<grid_for(Scap, 256), 256, 0, s>>>(c);
    TGNX_LAUNCH_CHECK("tgnn_seg_count");
    tgnn_seg_scan<<<1, 1024, 0, s>>>(c);
    TGNX_LAUNCH_CHECK("tgnn_seg_scan");
  }
  {  // edge metadata + collapsed weights (depends on the parameters only) in one launch
    const int nmeta = (int)std::min<int64_t>(4096, (Scap + 3) / 4);  // wave per segment
    probe_begin(TGNX_K_EDGE_META, s);
    tgnn_meta_collapse<TRAIN><<<nmeta + collapse_blocks(c), 256, 0, s>>>(c, nmeta);
    probe_end(TGNX_K_EDGE_META, s);
    TGNX_LAUNCH_CHECK("tgnn_meta_collapse");
  }
  probe_begin(TGNX_K_EDGE_FWD, s);
  launch_edge_fwd(c, TRAIN ? finish_blocks(c.Bmax) : 0, s);
  probe_end(TGNX_K_EDGE_FWD, s);
  TGNX_LAUNCH_CHECK("tgnn_edge_fwd");
  if (!TRAIN || !c.seg_in_pred) {  // (train below TGNX_BIG_BATCH: the segments ride in tgnn_pred_train)
    probe_begin(TGNX_K_SEG_FWD, s);
    tgnn_seg_fwd<TRAIN><<<grid_for(Scap, 4), 256, 0, s>>>(c);
    probe_end(TGNX_K_SEG_FWD, s);
    TGNX_LAUNCH_CHECK("tgnn_seg_fwd");
  }
  return TGNX_OK;
}

static int launch_backward(const Ctx& c, hipStream_t s) {
  probe_begin(TGNX_K_SEG_BWD, s);
  tgnn_seg_bwd_pred<<<c.Gs + pred_reduce_blocks(c.D), 256, 0, s>>>(c, c.Gs);
  probe_end(TGNX_K_SEG_BWD, s);
  TGNX_LAUNCH_CHECK("tgnn_seg_bwd_pred");
  probe_begin(TGNX_K_EDGE_BWD, s);
  launch_edge_bwd(c, s);
  probe_end(TGNX_K_EDGE_BWD, s);
  TGNX_LAUNCH_CHECK("tgnn_edge_bwd");
  tgnn_grad_reduce<<<(c.PL.total + 63) / 64, 64 * RED_WAVES, 0, s>>>(c, GBWD, c.Gs);
  TGNX_LAUNCH_CHECK("tgnn_grad_reduce");
  return TGNX_OK;
}


}  // namespace tgnx

using namespace tgnx;

extern "C" {

int tgnx_tgnn_param_layout(const tgnx_tgnn_config* cfg, int64_t* off) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(off, "tgnx_tgnn_param_layout: null output");
  Lay L = make_lay(cfg->mem_dim, cfg->msg_dim);
  const int64_t v[TGNX_TGNN_NPARAM + 1] = {L.te_w, L.te_b, L.attn_l, L.attn_r, L.attn_e, L.Wn, L.bn, L.We,
                                           L.be,   L.Ws,   L.bs,     L.Wd,     L.bd,     L.Wo, L.bo, L.total};
  for (int k = 0; k <= TGNX_TGNN_NPARAM; ++k) off[k] = v[k];
  return TGNX_OK;
}

size_t tgnx_tgnn_ws_bytes(const tgnx_tgnn_config* cfg) {
  if (check_cfg(cfg)) return 0;
  return make_ws(cfg).total;
}

size_t tgnx_tgnn_ws_misc_offset(const tgnx_tgnn_config* cfg) {
  if (check_cfg(cfg)) return 0;
  return make_ws(cfg).misc;
}

int tgnx_tgnn_advance(int64_t* ctl, int32_t mode, int64_t batch_start, int64_t B, int64_t cur_e_id, int64_t split_lo,
                      int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed, int32_t train,
                      void* stream) {
  TGNX_CHECK_ARG(ctl && (mode == 0 || mode == 1) && world >= 1 && rank >= 0 && rank < world,
                 "tgnx_tgnn_advance: bad arguments");
  TGNX_CHECK_ARG(mode == 0 ? (B >= 0 && B < 4096) : (batch > 0 && batch < 4096), "tgnx_tgnn_advance: batch too large");
  tgnn_advance<<<1, 64, 0, as_stream(stream)>>>(ctl, mode, batch_start, B, cur_e_id, split_lo, split_hi, batch, rank,
                                                world, base_seed, train);
  TGNX_LAUNCH_CHECK("tgnn_advance");
  return TGNX_OK;
}

static int train_fwd_bwd_impl(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t gen_neg,
                              int32_t dropout, void* stream, const Ctx* adv, bool fuse_adam = false);

int tgnx_tgnn_train_fwd_bwd(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t gen_neg,
                            int32_t dropout, void* stream) {
  return train_fwd_bwd_impl(cfg, buf, gen_neg, dropout, stream, nullptr);
}

int tgnx_tgnn_train_fwd_bwd_resident(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int64_t split_lo,
                                     int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                     int32_t dropout, void* stream) {
  TGNX_CHECK_ARG(batch > 0 && batch < 4096 && world >= 1 && rank >= 0 && rank < world && split_lo >= 0 &&
                     split_hi >= split_lo,
                 "tgnx_tgnn_train_fwd_bwd_resident: bad cursor arguments");
  Ctx a;
  memset(&a, 0, sizeof(a));
  a.adv = 1;
  a.adv_lo = split_lo;
  a.adv_hi = split_hi;
  a.adv_batch = batch;
  a.adv_rank = rank;
  a.adv_world = world;
  a.adv_seed = base_seed;
  a.adv_train = 1;
  return train_fwd_bwd_impl(cfg, buf, 1, dropout, stream, &a);
}

int tgnx_tgnn_train_step_resident(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int64_t split_lo,
                                  int64_t split_hi, int64_t batch, uint64_t base_seed, int32_t dropout, void* stream) {
  TGNX_CHECK_ARG(batch > 0 && batch < 4096 && split_lo >= 0 && split_hi >= split_lo,
                 "tgnx_tgnn_train_step_resident: bad cursor arguments");
  TGNX_CHECK_ARG(buf && buf->adam_m && buf->adam_v, "tgnx_tgnn_train_step_resident: null optimizer buffer");
  Ctx a;
  memset(&a, 0, sizeof(a));
  a.adv = 1;
  a.adv_lo = split_lo;
  a.adv_hi = split_hi;
  a.adv_batch = batch;
  a.adv_rank = 0;
  a.adv_world = 1;
  a.adv_seed = base_seed;
  a.adv_train = 1;
  a.defer = 1;
  return train_fwd_bwd_impl(cfg, buf, 1, dropout, stream, &a, true);
}

int tgnx_tgnn_apply_pending(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, void* stream) {
  Ctx c;
  int rc = make_ctx(cfg, buf, 1, c);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->grads && buf->adam_m && buf->adam_v, "tgnx_tgnn_apply_pending: null optimizer buffer");
  hipStream_t s = as_stream(stream);
  const int nel = grid_for(2 * c.D + (c.L.total - c.L.Ws), 256);
  tgnn_apply_pending<<<nel + expand_rows_blocks(c.D, 256), 256, 0, s>>>(c, nel);
  TGNX_LAUNCH_CHECK("tgnn_apply_pending");
  tgnn_clear_pending<<<1, 64, 0, s>>>(c.ctl);
  TGNX_LAUNCH_CHECK("tgnn_clear_pending");
  return TGNX_OK;
}

static int train_fwd_bwd_impl(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t gen_neg,
                              int32_t dropout, void* stream, const Ctx* adv, bool fuse_adam) {
  Ctx c;
  int rc = make_ctx(cfg, buf, 1, c);
  if (rc) return rc;
  if (adv) {
    c.adv = 1;
    c.adv_lo = adv->adv_lo;
    c.adv_hi = adv->adv_hi;
    c.adv_batch = adv->adv_batch;
    c.adv_rank = adv->adv_rank;
    c.adv_world = adv->adv_world;
    c.adv_seed = adv->adv_seed;
    c.adv_train = adv->adv_train;
    c.defer = adv->defer;
    c.apply_nel = grid_for(2 * c.D + (c.L.total - c.L.Ws), 1024);
  }
  TGNX_CHECK_ARG(buf->neg && buf->grads && buf->out_pos && buf->out_neg && buf->feat && buf->ev_msg && buf->memory &&
                     buf->time_assoc && buf->nbr && buf->eid && buf->rt,
                 "tgnx_tgnn_train_fwd_bwd: null buffer");
  TGNX_CHECK_ARG(!gen_neg || (buf->dst_nodes && buf->n_dst > 0), "tgnx_tgnn_train_fwd_bwd: no destination set");
  c.drop = dropout && (c.pf > 0.f || c.pa > 0.f);
  hipStream_t s = as_stream(stream);
  const int Bmax = cfg->max_batch;
  c.gen_neg = gen_neg ? 1 : 0;
  c.seg_in_pred = Bmax < TGNX_BIG_BATCH ? 1 : 0;
  rc = launch_forward<true>(c, 3 * (int64_t)Bmax, s);
  if (rc) return rc;
  probe_begin(TGNX_K_PRED, s);
  tgnn_pred_train<<<Bmax, 256, 0, s>>>(c);
  probe_end(TGNX_K_PRED, s);
  TGNX_LAUNCH_CHECK("tgnn_pred_train");
  rc = launch_backward(c, s);
  if (rc) return rc;
  if (fuse_adam && c.defer) {
    // (the expansion + Adam runs in the next step's first launch, or tgnx_tgnn_apply_pending)
  } else if (fuse_adam) {  // world 1: the expansion with Adam folded in (no tgnx_tgnn_train_update launch)
    const int nel = grid_for(2 * c.D + (c.L.total - c.L.Ws), 256);
    probe_begin(TGNX_K_ADAM, s);
    tgnn_expand_adam<<<nel + grid_for(2 * H * c.D, 4), 256, 0, s>>>(c, nel);
    probe_end(TGNX_K_ADAM, s);
    TGNX_LAUNCH_CHECK("tgnn_expand_adam");
  } else {
    const int nexp = grid_for(c.L.Ws, 256) < 1024 ? grid_for(c.L.Ws, 256) : 1024;
    tgnn_grad_expand<<<nexp + grid_for(3 * H * c.D, 4), 256, 0, s>>>(c, nexp);
    TGNX_LAUNCH_CHECK("tgnn_grad_expand");
  }
  return TGNX_OK;
}

int tgnx_tgnn_train_update(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, void* stream) {
  Ctx c;
  int rc = make_ctx(cfg, buf, 1, c);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->grads && buf->adam_m && buf->adam_v, "tgnx_tgnn_train_update: null optimizer buffer");
  hipStream_t s = as_stream(stream);
  probe_begin(TGNX_K_ADAM, s);
  tgnn_adam<<<grid_for(c.L.total / 4, 256), 256, 0, s>>>(c);
  probe_end(TGNX_K_ADAM, s);
  TGNX_LAUNCH_CHECK("tgnn_adam");
  return TGNX_OK;
}

int tgnx_tgnn_eval_step(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t Kn, int32_t tile_quirk,
                        void* stream) {
  Ctx c;
  TGNX_CHECK_ARG(Kn >= 1 && Kn <= cfg->max_neg, "tgnx_tgnn_eval_step: Kn must be in [1, max_neg]");
  int rc = make_ctx(cfg, buf, Kn, c);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->neg && buf->out_pos && buf->out_neg && buf->mrr && buf->feat && buf->ev_msg && buf->memory,
                 "tgnx_tgnn_eval_step: null buffer");
  c.quirk = tile_quirk ? 1 : 0;
  c.drop = 0;
  hipStream_t s = as_stream(stream);
  const int Bmax = cfg->max_batch;
  if (buf->grads && buf->adam_m && buf->adam_v) {  // a deferred train update still pending is applied first
    rc = tgnx_tgnn_apply_pending(cfg, buf, stream);
    if (rc) return rc;
  }
  rc = launch_forward<false>(c, (int64_t)Bmax * (2 + Kn), s);
  if (rc) return rc;
  tgnn_pred_eval_src<<<grid_for(Bmax, 4), 256, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgnn_pred_eval_src");
  tgnn_pred_eval_neg<<<grid_for((int64_t)Bmax * Kn, 4), 256, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgnn_pred_eval_neg");
  tgnn_mrr<<<1, 1024, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgnn_mrr");
  tgnn_ta_fill<<<grid_for(cfg->num_nodes, 256) < 4096 ? grid_for(cfg->num_nodes, 256) : 4096, 256, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgnn_ta_fill");
  tgnn_finish<false><<<finish_blocks(cfg->max_batch), 256, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgnn_finish");
  return TGNX_OK;
}

}  // extern "C"
