// TGN memory path on gfx950 (SURVEY §8 a14–a16): the PyG TGN of the reference's modules/ directory,
// wired as pyg_model_utils.py:10-36, trained by the canonical loop pyg_epoch_utils.py:106-137 carries
// commented out.  Reference semantics restated in oracle/tgn_ref.py (the checker).
//
// One train step at world 1 (tgnx_tgn_train_step_pp, the bench's step): 8 launches, no host sync, graph-replayed
// (one graph per scan-output parity).  The previous step already marked and scanned this batch into its set.
//   1 tgn_agg_emit   sampled edges (neighbor_loader.py:26-50 order) + Δt cos/sin into dense [enc | msg] rows ‖
//                    per sampled node its stored messages -> IdentityMessage -> Last/Mean aggregate
//                    (memory_module.py:152-207) ‖ per-root / per-centre records for the predictor's attention
//   2 gemmN          ring insert of the batch ‖ GRUCell / RNNCell over [msg | memory] (gate math in the
//                    epilogue) ‖ lin_edge over [cos(w Δt + b) | msg] (the per-neighbour contraction)
//   3 gemmN          lin_query / key / value / skip of every sampled node
//   4 tgn_pred_train per event: TransformerConv forward of its 3 roots (waves 1-3) ‖ predictor weight
//                    staging (wave 0); LinkPredictor + BCE + backward rows ‖ the sampled edges sorted by
//                    neighbour (one block) ‖ the NEXT batch's marking into the other set
//                    (DyRep embedding messages: + one update-list aggregation / updater launch here)
//   5 tgn_attn_bwd   attention backward: dq per centre ‖ per edge (dk, dv, dE) summed into the neighbours' k / v
//                    rows ‖ predictor bias / output-layer / loss reductions (+ fused Adam)
//   6 gemmN          dz0 = dP W with the cell backward in the epilogue ‖ dW_proj, dW_src/dst (split-K)
//   7 gemmN          the NEXT batch's scan into the other set (sorted node sets, insert / store plans) ‖ dX_enc ‖
//                    dW_cell, dW_edge (split-K) ‖ dEnc·W_e ‖ step-descriptor snapshot ‖ message stores
//   8 gemm_fixup     split-K sums with fused Adam ‖ Δt reduction ‖ memory / last_update of src ∪ dst ‖ counters
//                    advance + the next batch's descriptor
// 2 hops: the outer level's attention backward sums its edges' (dk, dv, dE) as launch 5 does; the inner
// (conv2) level keeps its k / v reduction launch (tgn_kv_reduce2 beside its dE2-only GEMMs).
// Data parallel (world > 1): the same launches without fused Adam; the exchange (one all-reduce of
// [gradients | memory-row slots]) and tgnx_tgn_apply_rows_update follow.
#include <mutex>
#include <unordered_map>

#include "tgnx_gemm.h"
#include "tgnx_math.h"
#include "tgnx_ring_dev.h"

namespace tgnx {

void probe_begin(int id, hipStream_t s);
void probe_end(int id, hipStream_t s);

namespace tgn {

constexpr int TH = 2;        // TransformerConv heads (emb_module.py:66)
constexpr int TDMAX = 128;   // memory / time / embedding dim capacity (C = D / 2 <= 64 lanes)
constexpr int TB_MAX = 4095; // events per batch (12-bit event index in the touch keys)
#ifndef TGNX_GRU_CAP
#define TGNX_GRU_CAP TGNX_GEMM_GRID_CAP  // grid cap of the GRU GEMM (its workgroups loop past it; 512: +0.3 %)
#endif
#ifndef TGNX_EDGE_CAP200
#define TGNX_EDGE_CAP200 768  // grid cap of the lin_edge GEMM per 200 events of the rank's batch (env TGNX_EDGE_CAP200; same-box
                              // A/Bs at wiki: 1024 0.0953 / 0.0952 / 0.0949 / 0.0948 ms, 768 0.0947 / 0.0946 / 0.0943 / 0.0942)
#endif
#ifndef TGNX_GRU_WAVES
#define TGNX_GRU_WAVES 6  // waves-per-SIMD floor of the ring ‖ GRU ‖ lin_edge launch (1 hop; round 5 with the graphs
                          // replayed without packet capture: 6 0.0867 / 0.0867 vs 0 0.0874 / 0.0872 ms, the launch 13.1-13.4 vs
                          // 13.8-13.9 us; tgn_agg_emit floors 6 / 8: 0.0879 / 0.0901 — profiles/r5/r5_agg_gru_waves_ab.txt)
#endif
#ifndef TGNX_W3_WAVES
#define TGNX_W3_WAVES 7  // waves-per-SIMD floor of the dW_cell launch (0: the compiler's register count, 84 + 8 -> 5 waves;
                         // same-box A/B: 0.0966 / 0.0961 ms, 6 waves 0.0961 / 0.0955, 7 (72 VGPRs, 12 B spilled) 0.0951 / 0.0951;
                         // round 5, 7 vs 0: wiki B = 200 0.0917 / 0.0914 vs 0.0927 / 0.0928 ms, B = 2,000 launch 32.6 vs
                         // 34.2 us with the step +-0, comment 2-hop B = 600 +-0 — profiles/r5/r5_w3waves_ab.txt; round 6,
                         // 8 waves: 0.0856 / 0.0854 vs 0.0847 / 0.0848 ms, and a 6 / 8-wave floor on the dz0 launch 0.0851 /
                         // 0.0858 — profiles/r6/r6as_tgn_waves_ab.txt)
#endif
#ifndef TGNX_DXE_DR
#define TGNX_DXE_DR TGNX_G32L_DR  // direct-operand slabs per round of the dX_enc GEMM (the 7-wave dW_cell launch)
#endif
using GXE = GemmCfg<TGNX_G32L_T, TGNX_G32L_T, TGNX_G32L_KC, TGNX_G32L_PF, TGNX_G32L_WS, TGNX_DXE_DR>;
enum { CNT_R = 0, CNT_M = 1, CNT_E = 2, CNT_U = 3, CNT_LIST = 6, CNT_NB = 9, CNT_WORDS = 16 };  // (4, 5: unused)
// ctl[ERR] bit of a step that found its scan-output set holding another batch (tgnx_tgn_train_step_pp)
constexpr int64_t ERR_STALE_SET = 16;
constexpr int64_t ERR_SORT_CAP = 32;  // edge_sort_body: more sampled rows than its LDS counters (host-checked; never expected)

__host__ __device__ inline int64_t al4(int64_t x) { return (x + 3) & ~int64_t(3); }

// Flat parameter buffer.  The four node projections of TransformerConv (query, key, value, skip) sit
// at a fixed stride (pw weights, pb biases) so kernels address projection g as base + g * stride:
// a 4-way pointer select was lowered to a scratch-memory lookup table inside the GEMM loaders.
struct Lay {
  int64_t te_w, te_b, w_ih, w_hh, b_ih, b_hh, wk, bk, wq, bq, wv, bv, we, wsk, bsk, lsw, lsb, ldw, ldb, lfw, lfb, total;
  int64_t pw, pb;  // projection strides: wq + g pw, bq + g pb for g = query, key, value, skip
  // layers = 2: gnn.conv2 (same shapes, same fixed-stride projection block), after lin_final.bias
  int64_t wk2, bk2, wq2, bq2, wv2, bv2, we2, wsk2, bsk2;
};
// cell: the memory updater, 0 = GRUCell (weights [3D, .]), 1 = RNNCell (DyRepMemory 'rnn', weights [D, .])
static Lay make_lay(int D, int d, int layers, int cell = 0) {
  const int64_t Qm = 3 * (int64_t)D + d, HC = D, G3 = cell ? 1 : 3;
  Lay L;
  int64_t o = 0;
  L.te_w = o; o += al4(D);
  L.te_b = o; o += al4(D);
  L.w_ih = o; o += al4(G3 * D * Qm);
  L.w_hh = o; o += al4(G3 * (int64_t)D * D);
  L.b_ih = o; o += al4(G3 * D);
  L.b_hh = o; o += al4(G3 * D);
  L.pw = al4(HC * D);
  L.pb = al4(HC);
  auto proj = [&](int64_t& wq, int64_t& wk, int64_t& wv, int64_t& wsk, int64_t& bq, int64_t& bk, int64_t& bv,
                  int64_t& bsk, int64_t& we) {
    wq = o; o += L.pw;
    wk = o; o += L.pw;
    wv = o; o += L.pw;
    wsk = o; o += L.pw;
    bq = o; o += L.pb;
    bk = o; o += L.pb;
    bv = o; o += L.pb;
    bsk = o; o += L.pb;
    we = o; o += al4(HC * (D + d));
  };
  proj(L.wq, L.wk, L.wv, L.wsk, L.bq, L.bk, L.bv, L.bsk, L.we);
  L.lsw = o; o += al4((int64_t)D * D);
  L.lsb = o; o += al4(D);
  L.ldw = o; o += al4((int64_t)D * D);
  L.ldb = o; o += al4(D);
  L.lfw = o; o += al4(D);
  L.lfb = o; o += al4(1);
  if (layers == 2) proj(L.wq2, L.wk2, L.wv2, L.wsk2, L.bq2, L.bk2, L.bv2, L.bsk2, L.we2);
  else L.wq2 = L.wk2 = L.wv2 = L.wsk2 = L.bq2 = L.bk2 = L.bv2 = L.bsk2 = L.we2 = 0;
  L.total = o;
  return L;
}

__device__ __forceinline__ void adam1(float g, float& m, float& v, float& p, float b1, float b2, float eps, float step,
                                      float bc2s) {
  m = m + (1.0f - b1) * (g - m);
  v = v * b2 + (1.0f - b2) * g * g;
  const float den = sqrtf(v) / bc2s + eps;
  p -= step * (m / den);
}

// Adam folded into the gradient writers (tgnx_tgn_train_step, world 1): the writer of a gradient
// element also applies the update to its parameter, so no separate optimizer pass re-reads the
// 4 buffers.  p == nullptr: plain gradient store (tgnx_tgn_train_fwd_bwd; data parallel).  The step
// scalars (lr / (1 - b1^t), sqrt(1 - b2^t)) are written to ctl[TGNX_CTL_ADAM_SC] by tgn_pred_train.
constexpr int TGNX_CTL_ADAM_SC = 15;
struct AdamFuse {
  float *p = nullptr, *m = nullptr, *v = nullptr;
  const int64_t* ctl = nullptr;
  float b1 = 0.f, b2 = 0.f, eps = 0.f;
  int keep_g = 1;  // fused: also store the gradient (0: TGNX_TGN_NO_GRAD_STORE, nothing reads it; 1.1 MB less per step)
  // n gradient elements (idx < 0: none) of one thread: every load issued before any store (the
  // buffers may alias as far as the compiler knows, so interleaving would serialise the elements)
  template <int N>
  __device__ __forceinline__ void put_n(float* g, const int64_t (&idx)[N], const float (&val)[N]) const {
    // no update for an empty batch (a resident cursor past the split): the split-K fixup still finishes
    // the previous step's partials, as tgn_adam skips B = 0
    if (!p || ctl[TGNX_CTL_B] == 0 || ctl[TGNX_CTL_ERR] != 0) {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (idx[i] >= 0) g[idx[i]] = val[i];
      return;
    }
    float mm[N], vv[N], pp[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int64_t j = idx[i] >= 0 ? idx[i] : 0;
      mm[i] = m[j];
      vv[i] = v[j];
      pp[i] = p[j];
    }
    const float* sc = reinterpret_cast<const float*>(ctl + TGNX_CTL_ADAM_SC);
    const float s0 = sc[0], s1 = sc[1];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (idx[i] < 0) continue;
      adam1(val[i], mm[i], vv[i], pp[i], b1, b2, eps, s0, s1);
      if (keep_g) st_wt(g + idx[i], val[i]);
      st_wt(m + idx[i], mm[i]);
      st_wt(v + idx[i], vv[i]);
      st_wt(p + idx[i], pp[i]);
    }
  }
  __device__ __forceinline__ void put(float* g, int64_t i, float val) const {
    const int64_t ix[1] = {i};
    const float vx[1] = {val};
    put_n<1>(g, ix, vx);
  }
};
struct Ctx {
  int64_t N, nev, words;
  int K, D, d, Qm, HC, C, aggr, Kn, drop, gen_neg;
  float p, inv_keep, lr, b1, b2, eps;
  const int64_t *ev_src, *ev_dst;
  const float *ev_t, *ev_msg;
  int64_t* neg;
  const int64_t* dst_nodes;
  int64_t n_dst;
  int64_t *nbr, *eid;
  float* rt;
  int64_t* assoc;
  float* mem;
  int64_t* lu_buf;
  int64_t* st;     // [4N] {s_off, s_cnt, d_off, d_cnt}
  int64_t* arena;  // [2 * nev] event ids, batch at event start s occupies [2s, 2s + 2B)
  int32_t* node_gen;
  float *params, *grads, *am, *av;
  int64_t* ctl;
  float *out_pos, *out_neg;
  float* out_ev;   // optional: train outputs by event row [nev, 2] (sigmoid pos, neg), the epoch's log
  double* mrr;
  float* xrows;  // data parallel: this rank's updated memory rows (TGNX_TGN_ROW layout), or nullptr
  int xcap;
  // workspace
  uint32_t *cb, *nb;       // centre / sampled-node bitmaps over N
  uint32_t *cbs, *nbs, *rbs;  // their summaries (bit per word)
  int *cl, *nl, *rl;       // tgn_scan: nonzero word lists
  int* kval;  // [N] valid ring slots of a centre (written by tgn_mark for this batch's centres)
  int* cnt;
  int64_t *cent, *nid, *upd;
  int *cent_loc, *ceoff, *crank, *upd_loc;
  int *e_j, *e_c;
  int64_t* e_id;
  float* e_t;
  float *X, *trel, *lu;
  int* evr;  // [3 B] centre row of each root (src, dst, neg) of this rank's events (tgn_agg_emit)
  int4* evq;  // [3 B] 1 hop: per root {centre row, P row, edge range} (tgn_pred_train<ATT>); nullptr at 2 hops
  int* evj;   // [3 B][16] 1 hop, ring K <= 16: per root the P rows of its edges' neighbours (e_j of its range)
  int4* cevq;  // [Rcap] with evj: per centre {P row, edge range} (tgn_attn_bwd's first round)
  int* cevj;   // [Rcap][16] with evj: per centre its edges' neighbour rows (every root of the centre writes
               // the same values)
  int64_t* xw;
  float *gates, *Z0, *P, *Ep, *alpha, *Zc, *evs, *Hs, *Hd;
  float* Hp;  // (GRU train step) row m's pre-update memory mem[nid[m]] [M][D], written by the GRU forward
  float *dZc, *dP, *dE, *dG, *tgp;
  // 1-hop train: the predictor accumulates the centres' output gradient into dzrep copies of dZc (dzstride floats
  // apart; workgroup b adds into copy b % dzrep), which the attention backward sums: a hub centre's row takes the
  // float atomics of ~40 % of the batch's workgroups (one row: ~14x slower, MI355X_MICROARCH.md 'Global float
  // atomics'); 2 hops: 1
  int dzrep;
  int64_t dzstride;
  int dzrep1;           // 2 hops: the same for the root level's dZr (the predictor's rows there; root_view)
  int64_t dzstride1;
  // resident batch cursor folded into tgn_mark (tgnx_tgn_train_step_resident): mark derives the batch
  // descriptor from the step counters, the step's last launch advances them
  int adv = 0;
  int64_t adv_lo = 0, adv_hi = 0, adv_batch = 0;
  int adv_rank = 0, adv_world = 1;
  uint64_t adv_seed = 0;
  AdamFuse adf;  // fused optimizer (tgnx_tgn_train_step) or plain gradient stores
  float* dKV;  // per edge [dk | dv] of the attention backward [E][2 HC] (tgn_kv_reduce sums them into dP)
  // kvf (1-hop train step, attention backward fused with the k / v sums, tgn_attn_bwd's edge blocks): the
  // forward also writes alk = alpha * keep per edge [E][2] and Qo = [q | Σ alpha~ v] per centre [R][2 HC]
  float *alk, *Qo;
  int kvf = 0;
  int *kj, *kx, *ke;  // kvf: the sampled edges sorted by neighbour row (tgn_pred_train's sort block): row, centre, edge
  int kvs = 0;        // kvf: those arrays are this step's (else the edge blocks read the edges in sampling order)
  int ktr = 1;        // rows of kj / kx / ke (the train edge capacity)
  float* encE;  // per sampled edge: the dense train edge row [cos of the Δt encoding argument | msg] [E][D + d]
  float *s0m, *s1m;    // per GRU row: (mean over its messages of) sin(arg), sin(arg) Δt  [M][D]
  float *pA, *pB, *pC, *pD;  // split-K partials of the deferred weight-gradient GEMMs
  uint64_t *rkeys, *skeys;
  int *rruns, *sruns;
  // plans split by node range over pplan workgroups each (tgn_scan): partition q's keys at [poff[q], +n_q) of
  // the key array (node order across partitions), its runs at runs[poff[q] + q ...] (+ terminator); pcnt[q]
  // = its run count.  pplan = 1: one workgroup per plan, runs at [0, U].
  int pplan;
  int *rpc, *rpo, *spc, *spo;
  // the fixup's copy of what the next batch's scan rewrites (it runs beside the fixup, SnapJob below):
  // ctl words, counts, update list; errw = the live error word (the fixup's view reads ctl from the copy)
  int64_t* snap_ctl;
  int* snap_cnt;
  int64_t* snap_upd;
  int* snap_upd_loc;
  int64_t* errw;
  int Bmax, Qcap, Rcap, Mcap, Ecap, Ucap, tgp_rows;
  int Bplan;  // the global max_batch (plan sizes)
  Lay L;
  // ---- 2-hop (layers = 2).  The arrays above then describe the OUTER sample: centres = the 1-hop node
  // set (roots ∪ their ring neighbours, sorted), nodes = the 2-hop set; gnn.conv runs over it and
  // writes Zc = h1 per centre.  The ROOT level (gnn.conv2 over the roots' own ring rows, whose
  // neighbours are all outer centres) has its own lists; `root_view` swaps them into a Ctx so the
  // attention kernels run unchanged on either level.
  int layers;
  int rsel;        // cnt word holding this view's centre count (CNT_R; root view: CNT_R1)
  int ccap;        // rows of this view's centre arrays (cent_loc; ceoff has ccap + 1): Rcap, root view R1cap
  int att_salt;    // attention-dropout stream (conv: 7, conv2: 9)
  uint32_t* rb;    // roots bitmap
  int* x2r;        // [outer centre] -> root index or -1 (nullptr at layers = 1)
  int64_t* cent1;  // roots (sorted)
  int *r_x2, *ceoff1;                // root -> its outer-centre index (row of P2 / h1); root edge offsets
  int *e1_j, *e1_e2;                 // root edge -> neighbour's outer-centre index; -> outer edge index
  int64_t* e1_id;                    // root edge -> event id
  float *P2, *Ep2, *alpha1, *Zr, *dZr, *dP2, *dE2, *pE, *pF;
  int R1cap, E1cap, tgp_e1;          // tgp rows of the root edges start at tgp_e1
  // DyRepMemory use_src_emb_in_msg (bit 0) / use_dst_emb_in_msg (bit 1) (memory_module.py:387-408; 0 =
  // TGNMemory messages): the memory update of src ∪ dst builds its messages with the embedding rows zemb
  // (per centre) in place of memory rows; Zupd: the memory updater's output rows of the update list
  // (train: computed beside the step's own GRU rows, read by the fixup's memory write)
  int emb;
  const float* zemb;
  float* Zupd;
  // tgnx_tgn_train_step_pp: tgn_agg_emit checks that the scan-output set holds this step's batch (cnt[CNT_NB])
  int tagchk;
  // resident steps over a split whose plans were built once (tgnx_tgn_plan_table): the ring-insert / store
  // plans of batch b at ptab + 64 + b * ptab_stride (plan_view), instead of the scan's per-step set
  const char* ptab;
  int64_t ptab_stride;
};
constexpr int CNT_R1 = 7, CNT_E1 = 8;
// the level's sampled-edge count (= ceoff[cnt[rsel]], written beside it by the scan): one load instead of two
// dependent ones at the head of the edge blocks
__device__ __forceinline__ int level_edges(const Ctx& c) {
  return c.cnt[c.rsel == CNT_R1 ? CNT_E1 : CNT_E];
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
// e / d for 0 <= e < 2^22, 0 < d (inv = 1.0f / d): float estimate, corrected to the exact quotient
__device__ __forceinline__ int div_small(int e, int d, float inv) {
  int q = (int)((float)e * inv);
  q -= q * d > e;
  q += (q + 1) * d <= e;
  return q;
}
__device__ __forceinline__ float softplusf(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }
// softplus of an argument in [-1, 1] (BCE-with-logits on a sigmoid output): 1 + e^-|x| lies in [1.37, 2], so the
// hardware log / exp (1-2 ulp) carry no cancellation; log1pf + expf took ~130 instructions each on the predictor's
// epilogue path
__device__ __forceinline__ float softplus_unit(float x) { return fmaxf(x, 0.f) + __logf(1.0f + __expf(-fabsf(x))); }

// ------------------------------------------------------------------ sampling (neighbor_loader.py:26-50)
// Node sets are bitmaps over N with a summary level (bit per bitmap word, set by the lane whose atomicOr
// found the word empty), so tgn_scan visits only the words that hold nodes: O(sampled + N / 1024)
// instead of O(N / 32) per batch (a single-workgroup walk of a 1M-node bitmap took ~40 us per pass).
// Plain read first: hub words are hit by many lanes, most find the bit set.
// tgn_scan walks every bitmap word of a small graph directly (<= 2 words per thread of its 1024) and
// the nonzero words of a large one from the summary bitmaps; mark sets summary bits only for the latter
constexpr int TGN_SCAN_THREADS = 1024;
constexpr int SCAN_LW = 2 * TGN_SCAN_THREADS;  // LDS word list of the listed walk (tgn_scan)
constexpr int SCAN_SWR = 4;                     // node-summary words per thread held in registers there
// plan partitions per plan (tgn_scan): one per TGNX_PLAN_KEYS keys of the (global) batch, up to TGNX_PLAN_PMAX
#ifndef TGNX_PLAN_KEYS
#define TGNX_PLAN_KEYS 512
#endif
#define TGNX_PLAN_PMAX 16
__host__ __device__ inline int plan_parts(int B) {
  const int p = (2 * B + TGNX_PLAN_KEYS - 1) / TGNX_PLAN_KEYS;
  return p < 1 ? 1 : (p > TGNX_PLAN_PMAX ? TGNX_PLAN_PMAX : p);
}
__host__ __device__ __forceinline__ bool scan_direct(int64_t words) { return words <= 2 * (int64_t)TGN_SCAN_THREADS; }
__device__ __forceinline__ void mark_node(uint32_t* bm, uint32_t* sum, int64_t v) {
  const int64_t w = v >> 5;
  const uint32_t bit = 1u << (v & 31);
  if (!(bm[w] & bit)) {
    if (atomicOr(&bm[w], bit) == 0u) atomicOr(&sum[w >> 5], 1u << (w & 31));
  }
}

// K1: every query entry marks its node as a centre and its node + valid ring neighbours as sampled;
// train negatives are drawn here (NegLinkSamplerDest, counter-based stream as in tgnx_tgnn);
// src / pos nodes are stamped for the update list (memory_module.py:129).  16 lanes per entry, one
// ring slot each (all slot loads in flight at once); the entry's valid-slot count goes to kval[v].
template <class AT = NoCheckpoint>
__device__ __forceinline__ void plan_blocks(const Ctx& c, int which, int B, int64_t start, unsigned char* smem, int* sh, AT at = AT{});
// The resident step's batch descriptor, from the step counters (tgnn_advance mode 1 restated): the
// batch `ahead` batches past the counters' one.  Every block derives it itself; the scan launch writes it
// into ctl for the later launches (TGNX_CTL_BATCH_START .. SEED).  The pipelined step marks the next
// batch (ahead = 1) before this step's last launch advances the counters.
struct ResDesc {
  int64_t start, seed;
  int B, lo, hi, gen;
};
__device__ __forceinline__ ResDesc res_desc(const Ctx& c, int ahead) {
  ResDesc d;
  const int64_t nb = c.ctl[TGNX_CTL_NB] + ahead;
  d.start = c.adv_lo + nb * c.adv_batch;
  d.B = d.start >= c.adv_hi ? 0 : (int)min(c.adv_hi - d.start, c.adv_batch);
  d.lo = (int)((int64_t)d.B * c.adv_rank / c.adv_world);
  d.hi = (int)((int64_t)d.B * (c.adv_rank + 1) / c.adv_world);
  d.seed = (int64_t)(mix64(c.adv_seed ^ mix64((uint64_t)(nb + 1))) >> 1);
  d.gen = (int)c.ctl[TGNX_CTL_GEN] + 1 + ahead;
  return d;
}
// the descriptor words of batch d into ctl, for the launches after this one
__device__ __forceinline__ void write_desc(const Ctx& c, const ResDesc& d) {
  c.ctl[TGNX_CTL_BATCH_START] = d.start;
  c.ctl[TGNX_CTL_B] = d.B;
  c.ctl[TGNX_CTL_CUR_EID] = d.start;
  c.ctl[TGNX_CTL_LO] = d.lo;
  c.ctl[TGNX_CTL_HI] = d.hi;
  c.ctl[TGNX_CTL_SEED] = d.seed;
}
// K1 body over `nmark` 256-thread blocks (bid = this block's index among them).  Resident train steps
// (c.adv) take the batch from the counters (ahead: see res_desc), every other step from ctl.
// lbm (LDS, MARK_LDS_WORDS x 3, or null): for a graph the scan walks directly (<= 2 words per scan thread),
// the block sets its bits in LDS bitmaps and ORs the nonzero words into the global ones at the end: a
// wiki-shaped hub neighbour sits in ~40 % of the page rings, and ~240 global atomics on its word queued at
// the memory side (~11-13 ns each, MI355X_MICROARCH.md 'fanin'); now each word takes one per block.
constexpr int MARK_LDS_WORDS = 2 * TGN_SCAN_THREADS;
template <bool TRAIN>
__device__ void mark_body(const Ctx& c, int bid, int nmark, int ahead, uint32_t* lbm) {
  int B, lo, nl, gen;
  int64_t start;
  uint64_t nseed, noff;
  const bool adv = TRAIN && c.adv;
  if (adv) {
    const ResDesc d = res_desc(c, ahead);
    B = d.B;
    start = d.start;
    lo = d.lo;
    nl = d.hi - d.lo;
    gen = d.gen;
    nseed = (uint64_t)d.seed;
    noff = (uint64_t)d.start;
  } else {
    B = (int)c.ctl[TGNX_CTL_B];
    start = c.ctl[TGNX_CTL_BATCH_START];
    // train: this rank's event slice [lo, lo + nl) (data parallel; the whole batch at world 1)
    lo = TRAIN ? (int)c.ctl[TGNX_CTL_LO] : 0;
    nl = TRAIN ? (int)(c.ctl[TGNX_CTL_HI] - c.ctl[TGNX_CTL_LO]) : B;
    gen = (int)c.ctl[TGNX_CTL_GEN];
    nseed = (uint64_t)c.ctl[TGNX_CTL_SEED];
    noff = (uint64_t)c.ctl[TGNX_CTL_CUR_EID];
  }
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const bool local = lbm && scan_direct(c.words);  // block-uniform
  const int W = (int)c.words;
  uint32_t *Lc = lbm, *Ln = lbm + MARK_LDS_WORDS, *Lr = lbm + 2 * MARK_LDS_WORDS;
  if (local) {
    for (int x = threadIdx.x; x < W; x += blockDim.x) Lc[x] = Ln[x] = Lr[x] = 0u;
    __syncthreads();
  }
  const int Kn = TRAIN ? 1 : c.Kn;
  const int nq = nl * (2 + Kn);
  const int sl = threadIdx.x & 15, grp = (threadIdx.x & 63) >> 4;
  const int gstride = (nmark * 256) >> 4;
  // (the entries are dealt to 256 threads per block; a wider block's other threads only share the LDS bitmaps' clear
  // and flush — the 8-wave predictor launch that hosts these blocks)
  for (int q = threadIdx.x < 256 ? (bid * 256 + (int)threadIdx.x) >> 4 : nq; q < nq; q += gstride) {
    int64_t v;
    if (q < nl) {
      v = c.ev_src[start + lo + q];
    } else if (q < 2 * nl) {
      v = c.ev_dst[start + lo + q - nl];
    } else if (TRAIN) {
      const int i = lo + q - 2 * nl;
      if (c.gen_neg) {
        const uint64_t seed = nseed, off = noff;
        const int64_t pd = c.ev_dst[start + i];
        v = c.dst_nodes[0];
        for (uint64_t attempt = 0; attempt < 64; ++attempt) {
          const uint64_t h = hash4(seed, 0x6E656773ull, off + (uint64_t)i, attempt);
          v = c.dst_nodes[(uint64_t)(((__uint128_t)(h >> 11) * (uint64_t)c.n_dst) >> 53)];
          if (v != pd) break;
        }
        if (sl == 0) c.neg[start + i] = v;
      } else {
        v = c.neg[start + i];
      }
    } else {
      const int x = q - 2 * nl;
      v = c.neg[(start + x / Kn) * Kn + x % Kn];
    }
    // every load of the entry before any atomic (vmcnt retires in issue order: a load issued after an
    // atomic waits for it), atomics without return: a lane sets a bit its plain read found clear, and the
    // word's summary bit only when that read found the whole word zero (a nonzero word was seen after an
    // atomic of a lane that found it zero, which set the summary; the bitmaps start the batch cleared).
    // The chain is entry -> ring slot -> neighbour word -> atomics.
    const int64_t vw = v >> 5;
    const uint32_t vbit = 1u << (v & 31);
    const bool summ = !scan_direct(c.words);
    uint32_t wcv = 0u, wnv = 0u, wrv = 0u;
    if (sl == 0 && !local) {
      wcv = c.cb[vw];
      wnv = c.nb[vw];
      if (c.layers == 2) wrv = c.rb[vw];
    }
    int k = 0;
    for (int j0 = 0; j0 < c.K; j0 += 16) {
      const int j = j0 + sl, jc = min(j, c.K - 1);
      const int64_t ej = c.eid[v * c.K + jc], u = c.nbr[v * c.K + jc];
      const bool ok = j < c.K && ej >= 0;
      const int64_t uw = ok ? (u >> 5) : vw;
      const uint32_t ubit = 1u << (u & 31);
      uint32_t wu = 0u, wcu = 0u;
      if (!local) {
        wu = c.nb[uw];
        if (c.layers == 2) wcu = c.cb[uw];
      }
      if (ok && local) {
        atomicOr(&Ln[uw], ubit);
        if (c.layers == 2) atomicOr(&Lc[uw], ubit);
      } else if (ok) {
        if (!(wu & ubit)) atomicOr(&c.nb[uw], ubit);
        if (summ && !wu) atomicOr(&c.nbs[uw >> 5], 1u << (uw & 31));
        if (c.layers == 2) {
          if (!(wcu & ubit)) atomicOr(&c.cb[uw], ubit);
          if (summ && !wcu) atomicOr(&c.cbs[uw >> 5], 1u << (uw & 31));
        }
      }
      if (ok && c.layers == 2) {
        // 2 hops: the neighbour is an outer centre; its own ring neighbours are sampled nodes
        // (the lane walks u's ring row, all K slot loads issued before the marking)
        int ku = 0;
        for (int i0 = 0; i0 < c.K; i0 += 8) {
          int64_t ev[8], w[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int ii = min(i0 + i, c.K - 1);
            ev[i] = c.eid[u * c.K + ii];
            w[i] = c.nbr[u * c.K + ii];
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if (i0 + i >= c.K || ev[i] < 0) continue;
            ++ku;
            if (local) atomicOr(&Ln[w[i] >> 5], 1u << (w[i] & 31));
            else mark_node(c.nb, c.nbs, w[i]);
          }
        }
        c.kval[u] = ku;
      }
      k += __popcll((__ballot(ok) >> (16 * grp)) & 0xFFFFull);
    }
    if (sl == 0) {
      if (q < 2 * nl) c.node_gen[v] = gen;
      c.kval[v] = k;
      if (local) {
        atomicOr(&Lc[vw], vbit);
        atomicOr(&Ln[vw], vbit);
        if (c.layers == 2) atomicOr(&Lr[vw], vbit);
      } else {
        if (!(wcv & vbit)) atomicOr(&c.cb[vw], vbit);
        if (summ && !wcv) atomicOr(&c.cbs[vw >> 5], 1u << (vw & 31));
        if (!(wnv & vbit)) atomicOr(&c.nb[vw], vbit);
        if (summ && !wnv) atomicOr(&c.nbs[vw >> 5], 1u << (vw & 31));
        if (c.layers == 2) {
          if (!(wrv & vbit)) atomicOr(&c.rb[vw], vbit);
          if (summ && !wrv) atomicOr(&c.rbs[vw >> 5], 1u << (vw & 31));
        }
      }
    }
  }
  if (local) {  // direct-scan graph: no summaries
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
      const uint32_t a = Lc[x], b = Ln[x], r = Lr[x];
      if (a) atomicOr(&c.cb[x], a);
      if (b) atomicOr(&c.nb[x], b);
      if (r) atomicOr(&c.rb[x], r);
    }
  }
}
template <bool TRAIN>
__global__ void __launch_bounds__(256) tgn_mark(Ctx c, int nmark) {
  TGNX_STAMP(1);
  __shared__ uint32_t lbm[3 * MARK_LDS_WORDS];
  mark_body<TRAIN>(c, blockIdx.x, nmark, 0, lbm);
}

// message-store plan of a batch: (node << 33 | dir << 32 | i), dir 0 = as source (msg_s_store),
// 1 = as destination (msg_d_store); sorted, each (node, dir) run lists its events in batch order
// (memory_module.py:188-191 with a stable sort): plan_part(which = 1) below.

template <class AT>
__device__ __forceinline__ void store_plan_block(const Ctx& c, int B, int64_t start, unsigned char* smem, int* sh, AT at) {
  const int n2 = 2 * B, n = next_pow2(n2);
  uint64_t* key = reinterpret_cast<uint64_t*>(smem);
  int* runs = reinterpret_cast<int*>(smem + (size_t)n * 8);
  uint64_t* tmp = reinterpret_cast<uint64_t*>(smem + (size_t)n * 8 + (size_t)(n2 + 2) * 4 + 8);
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    uint64_t k = ~0ull;
    if (p < n2) {
      const int i = p < B ? p : p - B, dir = p < B ? 0 : 1;
      const uint64_t node = (uint64_t)(dir == 0 ? c.ev_src[start + i] : c.ev_dst[start + i]);
      k = (node << 33) | ((uint64_t)dir << 32) | (uint64_t)i;
    }
    key[p] = k;
  }
  __syncthreads();
  at(0);
  sort_u64(key, tmp, n2, n, true, true);  // keys distinct: (node, dir, i); tmp holds n keys (tgn_scan_smem)
  at(1);
  const int T = blockDim.x, pc = (n2 + T - 1) / T;
  const int p0 = threadIdx.x * pc, p1 = min(n2, p0 + pc);
  int cntr = 0;
  for (int p = p0; p < p1; ++p) cntr += (p == 0 || (key[p] >> 32) != (key[p - 1] >> 32));
  int U;
  int rid = block_excl_scan(cntr, sh, &U);
  for (int p = p0; p < p1; ++p)
    if (p == 0 || (key[p] >> 32) != (key[p - 1] >> 32)) runs[rid++] = p;
  __syncthreads();
  for (int p = threadIdx.x; p < n2; p += T) c.skeys[p] = key[p];
  for (int r = threadIdx.x; r < U; r += T) c.sruns[r] = runs[r];
  if (threadIdx.x == 0) {
    c.sruns[U] = n2;
    c.spc[0] = U;
    c.spo[0] = 0;
  }
}

// the indices of the nonzero words of two bitmaps, ascending, from their summaries (cleared); whole block
__device__ void occupied_words2(uint32_t* sa, uint32_t* sb, int64_t words, int* la, int* lb, int* sh, int* na,
                                int* nb) {
  const int T = blockDim.x;
  const int64_t SW = (words + 31) >> 5, sc = (SW + T - 1) / T, s0 = min(SW, threadIdx.x * sc), s1 = min(SW, s0 + sc);
  int ca = 0, cb = 0;
  for (int64_t i = s0; i < s1; ++i) {
    ca += __popc(sa[i]);
    cb += sb ? __popc(sb[i]) : 0;
  }
  int oa, ob;
  block_excl_scan2(ca, cb, sh, &oa, &ob, na, nb);
  auto emit = [&](uint32_t* sum, int* list, int o) {
    for (int64_t i = s0; i < s1; ++i) {
      uint32_t m = sum[i];
      if (!m) continue;
      sum[i] = 0u;
      while (m) {
        const int b = __ffs(m) - 1;
        m &= m - 1;
        list[o++] = (int)((i << 5) + b);
      }
    }
  };
  emit(sa, la, oa);
  if (sb) emit(sb, lb, ob);
}

// dynamic LDS of the scan launch (the plan workgroups' keys, runs and sort buffer)
__host__ __device__ inline size_t tgn_scan_smem(int Bmax) {
  const int n = next_pow2(2 * Bmax);
  return (size_t)n * 16 + (size_t)(2 * Bmax + 4) * 4 + 64;
}

// the batch's ring-insert plan (which = 0) and message-store plan (which = 1); they read only the batch's
// events and run as two extra 1024-thread workgroups of the scan launch
// One partition (node range) of a batch's plan: which = 0 ring-insert plan (keys node << 32 | (B-1-i) << 1 | dir,
// runs per node), 1 message-store plan (node << 33 | dir << 32 | i, runs per (node, dir)).  With P > 1 the
// P workgroups of a plan derive the same node splitters from a 64-entry sample (sorted by wave 0), count
// every partition's entries (so each knows its key offset), compact their own entries in entry order and
// sort only those: P sorts of ~2B / P keys in parallel instead of one of 2B (a data-parallel step plans
// the whole global batch; sorting 3,200 keys took one workgroup 49 us).
// where a partitioned plan writes (one parity set's keys, runs and per-partition counts / offsets)
struct PlanOut {
  uint64_t *rkeys, *skeys;
  int *rruns, *sruns, *pc;  // pc: rpc | rpo | spc | spo, TGNX_PLAN_PMAX each
};
__host__ __device__ inline PlanOut plan_out(const Ctx& c) { return PlanOut{c.rkeys, c.skeys, c.rruns, c.sruns, c.rpc}; }
// MAXE: entries per thread (2B <= MAXE x the workgroup size)
template <int MAXE = 8, class AT>
__device__ __forceinline__ void plan_part(const Ctx& c, int which, int part, int P, int B, int64_t start, unsigned char* smem, int* sh,
                          AT at, const PlanOut& po) {
  const int tid = threadIdx.x, T = blockDim.x, n2 = 2 * B;
  const int64_t* src = c.ev_src + start;
  const int64_t* dst = c.ev_dst + start;
  __shared__ int64_t split[17];
  __shared__ int pn[17];
  auto node_of = [&](int p) -> int64_t {
    const int i = p < B ? p : p - B;
    return which == 0 ? (p < B ? dst[i] : src[i]) : (p < B ? src[i] : dst[i]);
  };
  auto key_of = [&](int p, int64_t v) -> uint64_t {
    const int i = p < B ? p : p - B, dir = p < B ? 0 : 1;
    const uint64_t node = (uint64_t)v;
    return which == 0 ? (node << 32) | ((uint64_t)(B - 1 - i) << 1) | (uint64_t)dir
                      : (node << 33) | ((uint64_t)dir << 32) | (uint64_t)i;
  };
  auto part_of = [&](int64_t v) {
    int q = 0;
    for (int x = 1; x < P; ++x) q += v >= split[x];
    return q;
  };
  uint64_t* key = reinterpret_cast<uint64_t*>(smem);
  int* runs = reinterpret_cast<int*>(smem + (size_t)next_pow2(n2) * 8);
  uint64_t* tmp = reinterpret_cast<uint64_t*>(smem + (size_t)next_pow2(n2) * 8 + (size_t)(n2 + 2) * 4 + 8);
  // entries p = tid + j T (all loads of a thread in flight at once); a partition's keys are compacted in
  // any order (wave-aggregated LDS slots): the keys are distinct, so the sort fixes their order
  int64_t v[MAXE];
#pragma unroll
  for (int j = 0; j < MAXE; ++j) v[j] = node_of(min(tid + j * T, n2 - 1));  // unconditional (clamped) loads
  __shared__ int lpos;
  int off = 0;
  if (P > 1) {
    if (tid < WAVE) {  // 64 sampled nodes, sorted in registers; splitters at the P-quantiles
      uint64_t sv = (uint64_t)node_of((int)(((int64_t)tid * n2) >> 6));
      for (int k = 2; k <= WAVE; k <<= 1) switch (k >> 1) {
          case 32: sv = bitonic_lane_stage<32>(sv, tid, k); [[fallthrough]];
          case 16: sv = bitonic_lane_stage<16>(sv, tid, k); [[fallthrough]];
          case 8: sv = bitonic_lane_stage<8>(sv, tid, k); [[fallthrough]];
          case 4: sv = bitonic_lane_stage<4>(sv, tid, k); [[fallthrough]];
          case 2: sv = bitonic_lane_stage<2>(sv, tid, k); [[fallthrough]];
          default: sv = bitonic_lane_stage<1>(sv, tid, k);
        }
      for (int x = 1; x < P; ++x)
        if (tid == (x * WAVE) / P) split[x] = (int64_t)sv;
    }
    if (tid <= P) pn[tid] = 0;
    if (tid == 0) lpos = 0;
    __syncthreads();
    int q[MAXE];
    int cnt[17];
#pragma unroll
    for (int x = 0; x < 17; ++x) cnt[x] = 0;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      q[j] = tid + j * T < n2 ? part_of(v[j]) : -1;
#pragma unroll
      for (int x = 0; x < 17; ++x) cnt[x] += x == q[j];
    }
#pragma unroll
    for (int x = 0; x < 17; ++x)  // (partition counts: one LDS atomic per wave and partition)
      if (x < P) {
        const int w = (int)wave_sum_f((float)cnt[x]);  // exact: < 2^24
        if ((tid & (WAVE - 1)) == 0 && w) atomicAdd(&pn[x], w);
      }
    // this partition's keys into LDS slots (wave-aggregated)
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      const bool me = q[j] == part;
      const uint64_t m = __ballot(me);
      int base = 0;
      if ((tid & (WAVE - 1)) == 0 && m) base = atomicAdd(&lpos, __popcll(m));
      base = lane_i(base, 0);
      if (me) key[base + __popcll(m & ((1ull << (tid & (WAVE - 1))) - 1ull))] = key_of(tid + j * T, v[j]);
    }
    __syncthreads();
    for (int x = 0; x < part; ++x) off += pn[x];
  } else {
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      const int p = tid + j * T;
      if (p < n2) key[p] = key_of(p, v[j]);
    }
  }
  const int nk = P > 1 ? pn[part] : n2;
  const int n = next_pow2(max(nk, 1));
  for (int p = nk + tid; p < n; p += T) key[p] = ~0ull;
  __syncthreads();
  at(0);
  sort_u64(key, tmp, nk, n, true, true);  // keys distinct
  at(1);
  constexpr int sh_run = 32;  // runs: node (ring plan: key >> 32) / (node, dir) (store plan: key >> 32)
  const int pc = (nk + T - 1) / T, p0 = min(nk, tid * pc), p1 = min(nk, p0 + pc);
  int cr = 0;
  for (int p = p0; p < p1; ++p) cr += (p == 0 || (key[p] >> sh_run) != (key[p - 1] >> sh_run));
  int U;
  int rid = block_excl_scan(cr, sh, &U);
  for (int p = p0; p < p1; ++p)
    if (p == 0 || (key[p] >> sh_run) != (key[p - 1] >> sh_run)) runs[rid++] = p;
  __syncthreads();
  uint64_t* gk = which == 0 ? po.rkeys : po.skeys;
  int* gr = (which == 0 ? po.rruns : po.sruns) + off + part;
  for (int p = tid; p < nk; p += T) gk[off + p] = key[p];
  for (int r = tid; r < U; r += T) gr[r] = off + runs[r];
  if (tid == 0) {
    gr[U] = off + nk;
    po.pc[(which == 0 ? 0 : 2) * TGNX_PLAN_PMAX + part] = U;
    po.pc[(which == 0 ? 1 : 3) * TGNX_PLAN_PMAX + part] = off;
  }
}
template <class AT>
__device__ __forceinline__ void plan_blocks(const Ctx& c, int which, int B, int64_t start, unsigned char* smem, int* sh, AT at) {
  // blocks [0, pplan): ring-plan partitions; [pplan, 2 pplan): store-plan partitions.  One partition (a
  // world-1 batch): the single-workgroup plans (their keys come straight from the events, no compaction)
  const int P = c.pplan;
  if (P > 1) {
    plan_part(c, which < P ? 0 : 1, which % P, P, B, start, smem, sh, at, plan_out(c));
  } else if (which == 0) {
    const int tid = threadIdx.x, T = blockDim.x;
    uint64_t* key;
    int* runs;
    const int U = ring_plan_block(c.ev_src + start, c.ev_dst + start, B, smem, sh, &key, &runs, at, true);
    for (int p = tid; p < 2 * B; p += T) c.rkeys[p] = key[p];
    for (int r = tid; r < U; r += T) c.rruns[r] = runs[r];
    if (tid == 0) {
      c.rruns[U] = 2 * B;
      c.rpc[0] = U;
      c.rpo[0] = 0;
    }
  } else {
    store_plan_block(c, B, start, smem, sh, at);
  }
}
// run r of a partitioned plan -> its key range [a, a + len) (r: the global run index, partitions in node order)
__device__ __forceinline__ bool plan_run(const int* runs, const int* pc, const int* po, int P, int r, int& a, int& len) {
  int base = 0;
  for (int q = 0; q < P; ++q) {
    const int u = pc[q];
    if (r < base + u) {
      const int* g = runs + po[q] + q + (r - base);
      a = g[0];
      len = g[1] - a;
      return true;
    }
    base += u;
  }
  return false;
}
__device__ __forceinline__ int plan_runs(const int* pc, int P) {
  int u = 0;
  for (int q = 0; q < P; ++q) u += pc[q];
  return u;
}
// per-batch plan slot of the split's plan table: rkeys [2 Bmax] u64 | skeys [2 Bmax] u64 | rruns, sruns
// [2 Bmax + 2 + PMAX] i32 each | pc [4 PMAX] i32 (rpc | rpo | spc | spo); a 64-B header {lo, hi, batch,
// Bmax} precedes the slots
__host__ __device__ inline int64_t plan_slot_bytes(int Bmax) {
  const int64_t n2 = 2 * (int64_t)Bmax;
  return ((n2 * 16 + (n2 + 2 + TGNX_PLAN_PMAX) * 8 + 4 * TGNX_PLAN_PMAX * 4) + 255) & ~(int64_t)255;
}
__host__ __device__ inline PlanOut plan_slot(const char* tab, int64_t stride, int Bmax, int64_t b) {
  char* base = const_cast<char*>(tab) + 64 + b * stride;
  const int64_t n2 = 2 * (int64_t)Bmax;
  PlanOut o;
  o.rkeys = reinterpret_cast<uint64_t*>(base);
  o.skeys = o.rkeys + n2;
  o.rruns = reinterpret_cast<int*>(o.skeys + n2);
  o.sruns = o.rruns + n2 + 2 + TGNX_PLAN_PMAX;
  o.pc = o.sruns + n2 + 2 + TGNX_PLAN_PMAX;
  return o;
}
// the plans a consumer reads for the batch starting at event `start`: the table's slot (resident split steps
// with a plan table), else the scan's set
__device__ __forceinline__ PlanOut plan_view(const Ctx& c, int64_t start) {
  if (!c.ptab) return plan_out(c);
  return plan_slot(c.ptab, c.ptab_stride, c.Bplan, (start - c.adv_lo) / c.adv_batch);
}

// K2 (3 workgroups): WG0 ordered bitmap walks -> centres (+ edge offsets, update list) and sampled
// nodes (+ assoc, centre ranks); WG1 / WG2 the batch's ring-insert / message-store plans (they read only
// the batch's events).  Resident train steps: every workgroup takes the batch from the step counters
// and WG0 writes the descriptor into ctl for the later launches (no workgroup of this launch reads it).
// scan_body: workgroup `role` of it (0: walks, 1 .. 2 pplan: plans), any workgroup size T with the
// graph's bitmap words <= 2 T when scan_direct (scan_folds), LDS at smem (tgn_scan_smem)
// ahead: the batch `ahead` past the step counters' (1: the early scan of tgnx_tgn_train_step_pp, before this
// step's counter advance); wdesc: write the batch descriptor into ctl (not while this step's launches still
// read it); LW: capacity of the listed walk's LDS word list (>= 2 x the workgroup size); WPT: bitmap words per thread
// of the register walk (direct / listed), 2 at 1024 threads, 8 for the 256-thread walk that rides in another launch
template <bool TRAIN, class AT, int LW = SCAN_LW, int WPT = 2>
__device__ __forceinline__ void scan_body(const Ctx& c, int role, unsigned char* smem, AT at, int ahead, bool wdesc) {
  __shared__ int sh[40];
  const int tid = threadIdx.x, T = blockDim.x;
  int B, gen;
  int64_t start;
  if (TRAIN && c.adv) {
    const ResDesc d = res_desc(c, ahead);
    B = d.B;
    start = d.start;
    gen = d.gen;
    if (role == 0 && tid == 0) c.cnt[CNT_NB] = (int)(c.ctl[TGNX_CTL_NB] + ahead);  // the batch this set holds
    if (role == 0 && tid == 0 && wdesc) write_desc(c, d);
  } else {
    B = (int)c.ctl[TGNX_CTL_B];
    start = c.ctl[TGNX_CTL_BATCH_START];
    gen = (int)c.ctl[TGNX_CTL_GEN];
  }
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  if (role >= 1) {
    plan_blocks(c, role - 1, B, start, smem, sh, at);
    return;
  }
  // pass 0: the words each thread walks.  Small graphs (<= 2 words per thread): contiguous word ranges
  // (summaries just cleared); large graphs: the nonzero words in word order, from the summaries
  const bool direct = scan_direct(c.words);
  // listed (large graphs, 1 hop): the nonzero node words (a centre is a sampled node, so its word is one
  // of them) from the node summary into an LDS list in word order, then walked as the direct path walks
  // its words (<= 2 per thread, in registers, centres staged for pass 2): 2 dependent global rounds to
  // the sorted sets instead of 4 (summaries -> global word lists -> words -> cent[] -> assoc[])
  __shared__ int lwl[LW];
  bool listed = false;
  int ncw, nnw, nrw = 0;
  if (!direct) {
    const int64_t SW = (c.words + 31) >> 5, sq = (SW + T - 1) / T, s0 = min(SW, tid * sq), s1 = min(SW, s0 + sq);
    uint32_t sv[SCAN_SWR];
    int nz = 0;
#pragma unroll
    for (int j = 0; j < SCAN_SWR; ++j) {
      sv[j] = s0 + j < s1 ? c.nbs[s0 + j] : 0u;
      nz += __popc(sv[j]);
    }
    for (int64_t i = s0 + SCAN_SWR; i < s1; ++i) nz += __popc(c.nbs[i]);
    int tw;
    int o = block_excl_scan(nz, sh, &tw);
    listed = tw <= min(WPT * T, LW);  // (block-uniform)
    if (listed) {
      auto emit = [&](int64_t i, uint32_t m) {
        if (!m) return;
        c.nbs[i] = 0u;
        c.cbs[i] = 0u;
        while (m) {
          const int b = __ffs(m) - 1;
          m &= m - 1;
          lwl[o++] = (int)((i << 5) + b);
        }
      };
#pragma unroll
      for (int j = 0; j < SCAN_SWR; ++j) emit(s0 + j, sv[j]);  // (zero past s1)
      for (int64_t i = s0 + SCAN_SWR; i < s1; ++i) emit(i, c.nbs[i]);
      ncw = nnw = tw;
      if (c.layers == 2) {  // the roots' words for pass 3 (global list, as before)
        int unused;
        occupied_words2(c.rbs, nullptr, c.words, c.rl, nullptr, sh, &nrw, &unused);
        __threadfence_block();
      }
      __syncthreads();
    }
  }
  if (direct) {
    ncw = nnw = (int)c.words;
    if (c.layers == 2) nrw = (int)c.words;
    const int64_t SW = (c.words + 31) >> 5;
    for (int64_t i = tid; i < SW; i += T) {
      c.cbs[i] = c.nbs[i] = 0u;
      if (c.layers == 2) c.rbs[i] = 0u;
    }
  } else if (!listed) {
    occupied_words2(c.cbs, c.nbs, c.words, c.cl, c.nl, sh, &ncw, &nnw);
    if (c.layers == 2) {
      int unused;
      occupied_words2(c.rbs, nullptr, c.words, c.rl, nullptr, sh, &nrw, &unused);
    }
    __threadfence_block();
    __syncthreads();
  }
  auto word = [&](const int* list, int i) -> int64_t { return direct ? (int64_t)i : (int64_t)list[i]; };
  // pass 1: centres (sorted) and sampled nodes (sorted, + assoc): thread t takes a contiguous run of each
  // word list; block scans give the ranks; words are cleared.  Direct (small) graphs: a thread's <= 2 words
  // of both bitmaps stay in registers, and in 1-hop train steps the centres and their node ranks (a
  // centre is a sampled node too: its rank is the word's first node rank + the node bits below it) are
  // staged in LDS for pass 2 — no global round trip for cent[] / assoc[] there.
  const int cq = (ncw + T - 1) / T, c0 = min(ncw, tid * cq), c1 = min(ncw, c0 + cq);
  const int nq = (nnw + T - 1) / T, n0 = min(nnw, tid * nq), n1 = min(nnw, n0 + nq);
  int nc = 0, np = 0;
  uint32_t dcw[WPT] = {}, dnw[WPT] = {};
  int64_t dwi[WPT] = {};  // the words (direct: c0 + j; listed: from the LDS list)
  const bool walk = direct || listed;
  if (walk) {  // c0..c1 == n0..n1, <= WPT words
#pragma unroll
    for (int j = 0; j < WPT; ++j) dwi[j] = direct ? (int64_t)(c0 + j) : (int64_t)lwl[min(c0 + j, max(ncw - 1, 0))];
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      if (c0 + j < c1) {
        dcw[j] = c.cb[dwi[j]];
        dnw[j] = c.nb[dwi[j]];
      }
      nc += __popc(dcw[j]);
      np += __popc(dnw[j]);
    }
  } else {
    for (int i = c0; i < c1; ++i) nc += __popc(c.cb[word(c.cl, i)]);
    for (int i = n0; i < n1; ++i) np += __popc(c.nb[word(c.nl, i)]);
  }
  int R, M, rc, rank;
  block_excl_scan2(nc, np, sh, &rc, &rank, &R, &M);
  const bool fits = R <= c.Rcap && M <= c.Mcap;
  const bool lds_c = walk && TRAIN && R <= 3 * c.Bmax;  // (block-uniform)
  int64_t* lv = reinterpret_cast<int64_t*>(smem);                          // [3 Bmax] centre node
  int* lloc = reinterpret_cast<int*>(smem + (size_t)3 * c.Bmax * 8);       // [3 Bmax] its node rank
  if (walk) {
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      if (c0 + j >= c1) break;
      const int64_t w = dwi[j];
      const int rw = rank;
      uint32_t m = dnw[j];
      if (m) c.nb[w] = 0u;
      while (m) {
        const int b = __ffs(m) - 1;
        m &= m - 1;
        const int64_t v = (w << 5) + b;
        if (fits) c.nid[rank] = v;
        c.assoc[v] = rank;
        ++rank;
      }
      m = dcw[j];
      if (m) c.cb[w] = 0u;
      while (m) {
        const int b = __ffs(m) - 1;
        m &= m - 1;
        if (fits) {
          c.cent[rc] = (w << 5) + b;
          if (lds_c) {
            lv[rc] = (w << 5) + b;
            lloc[rc] = rw + __popc(dnw[j] & ((1u << b) - 1u));
          }
        }
        ++rc;
      }
    }
  } else {
    for (int i = c0; i < c1; ++i) {
      const int64_t w = word(c.cl, i);
      uint32_t m = c.cb[w];
      if (m) c.cb[w] = 0u;
      while (m) {
        const int b = __ffs(m) - 1;
        m &= m - 1;
        if (fits) c.cent[rc] = (w << 5) + b;
        ++rc;
      }
    }
    for (int i = n0; i < n1; ++i) {
      const int64_t w = word(c.nl, i);
      uint32_t m = c.nb[w];
      if (m) c.nb[w] = 0u;
      while (m) {
        const int b = __ffs(m) - 1;
        m &= m - 1;
        const int64_t v = (w << 5) + b;
        if (fits) c.nid[rank] = v;
        c.assoc[v] = rank;
        ++rank;
      }
    }
  }
  if (!fits) {
    if (tid == 0) c.ctl[TGNX_CTL_ERR] |= 4;
    for (int i = tid; i < nrw; i += T) c.rb[word(c.rl, i)] = 0u;  // leave every bitmap empty
    return;
  }
  for (int x = tid; x < M; x += T) c.crank[x] = -1;
  __threadfence_block();
  __syncthreads();
  // pass 2: per centre (contiguous chunk per thread) ring-slot count and update stamp -> edge
  // offsets and the update list (memory_module.py:129 src ∪ dst, sorted)
  const int xc = (R + T - 1) / T, x0 = min(R, tid * xc), x1 = min(R, x0 + xc);
  int ne = 0, nu = 0;
  constexpr int XR = 4;
  if (lds_c && xc <= XR) {  // the chunk's (<= 4) centres in registers across the block scan
    int64_t v[XR] = {};
    int loc[XR] = {}, kv[XR] = {};
    bool up[XR] = {};
#pragma unroll
    for (int j = 0; j < XR; ++j)
      if (x0 + j < x1) {
        v[j] = lv[x0 + j];
        loc[j] = lloc[x0 + j];
      }
#pragma unroll
    for (int j = 0; j < XR; ++j)
      if (x0 + j < x1) {
        kv[j] = c.kval[v[j]];
        up[j] = c.node_gen[v[j]] == gen;
        ne += kv[j];
        nu += up[j];
      }
    int E, U, re, ru;
    block_excl_scan2(ne, nu, sh, &re, &ru, &E, &U);
#pragma unroll
    for (int j = 0; j < XR; ++j)
      if (x0 + j < x1) {
        const int x = x0 + j;
        c.ceoff[x] = re;
        re += kv[j];
        c.cent_loc[x] = loc[j];
        c.crank[loc[j]] = x;
        if (c.x2r) c.x2r[x] = -1;
        if (up[j]) {
          c.upd[ru] = v[j];
          c.upd_loc[ru] = loc[j];
          ++ru;
        }
      }
    if (tid == 0) {
      c.ceoff[R] = E;
      c.cnt[CNT_R] = R;
      c.cnt[CNT_M] = M;
      c.cnt[CNT_E] = E;
      c.cnt[CNT_U] = U;
      c.ctl[TGNX_CTL_SUM_E] += E;
      c.ctl[TGNX_CTL_SUM_S] += M;
    }
  } else {
    for (int x = x0; x < x1; ++x) {
      const int64_t v = c.cent[x];
      ne += c.kval[v];
      nu += c.node_gen[v] == gen;
    }
    int E, U, re, ru;
    block_excl_scan2(ne, nu, sh, &re, &ru, &E, &U);
    for (int x = x0; x < x1; ++x) {
      const int64_t v = c.cent[x];
      const int loc = (int)c.assoc[v];
      c.ceoff[x] = re;
      re += c.kval[v];
      c.cent_loc[x] = loc;
      c.crank[loc] = x;
      if (c.x2r) c.x2r[x] = -1;
      if (c.node_gen[v] == gen) {
        c.upd[ru] = v;
        c.upd_loc[ru] = loc;
        ++ru;
      }
    }
    if (tid == 0) {
      c.ceoff[R] = E;
      c.cnt[CNT_R] = R;
      c.cnt[CNT_M] = M;
      c.cnt[CNT_E] = E;
      c.cnt[CNT_U] = U;
      c.ctl[TGNX_CTL_SUM_E] += E;
      c.ctl[TGNX_CTL_SUM_S] += M;
    }
  }
  if (c.layers != 2) return;
  // pass 3 (2 hops): the roots (sorted) from their bitmap -> root index, outer-centre index (crank is
  // complete after the barrier), root edge offsets (a root's edges are its outer edge range)
  __threadfence_block();
  __syncthreads();
  const int rq = (nrw + T - 1) / T, q0 = min(nrw, tid * rq), q1 = min(nrw, q0 + rq);
  int nr = 0, nre = 0;
  for (int i = q0; i < q1; ++i) {
    const int64_t w = word(c.rl, i);
    uint32_t m = c.rb[w];
    nr += __popc(m);
    while (m) {
      const int b = __ffs(m) - 1;
      m &= m - 1;
      nre += c.kval[(w << 5) + b];
    }
  }
  int R1, E1, r1, e1;
  block_excl_scan2(nr, nre, sh, &r1, &e1, &R1, &E1);
  if (R1 > c.R1cap) {
    if (tid == 0) c.ctl[TGNX_CTL_ERR] |= 4;
    for (int i = tid; i < nrw; i += T) c.rb[word(c.rl, i)] = 0u;
    return;
  }
  for (int i = q0; i < q1; ++i) {
    const int64_t w = word(c.rl, i);
    uint32_t m = c.rb[w];
    if (m) c.rb[w] = 0u;
    while (m) {
      const int b = __ffs(m) - 1;
      m &= m - 1;
      const int64_t v = (w << 5) + b;
      const int x2 = c.crank[c.assoc[v]];
      c.cent1[r1] = v;
      c.r_x2[r1] = x2;
      c.x2r[x2] = r1;
      c.ceoff1[r1] = e1;
      e1 += c.kval[v];
      ++r1;
    }
  }
  if (tid == 0) {
    c.ceoff1[R1] = E1;
    c.cnt[CNT_R1] = R1;
    c.cnt[CNT_E1] = E1;
  }
}
template <bool TRAIN>
__global__ void __launch_bounds__(1024) tgn_scan(Ctx c, int ahead, int wdesc) {
  TGNX_STAMP(2);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  scan_body<TRAIN>(c, (int)blockIdx.x, smem, [&](int slot) { TGNX_STAMP_AT(slot); }, ahead, wdesc != 0);
}

// ------------------------------------------------------------------ messages (memory_module.py:152-207)
// Aggregated message of node n (wave): IdentityMessage [mem[n], mem[other], raw, cos(w (t - lu[n]) + b)]
// of its stored events, LastAggregator (first max t over [msg_s; msg_d], msg_agg.py:15-21) or
// MeanAggregator (msg_agg.py:24-26); lu_new = max t (0 without messages, PyG scatter 'max').
// Loads are batched: each 64-event chunk of the store is fetched lane-parallel (event id, other
// endpoint, t) and broadcast by shuffles; the X row is filled 8 columns per lane at a time from
// selected addresses (unconditional loads, encoding columns blended arithmetically).
__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {  // src wave-uniform (readlane)
  return (int64_t)(((uint64_t)(uint32_t)lane_i((int)(v >> 32), src) << 32) | (uint64_t)(uint32_t)lane_i((int)v, src));
}
// stored event k of node n (k < sc: as source, else as destination): id, other endpoint, t
struct StoreView {
  int64_t so, sc, dof, tot;
};
__device__ __forceinline__ StoreView store_view(const Ctx& c, int64_t n) {
  StoreView s;
  s.so = c.st[4 * n];
  s.sc = c.st[4 * n + 1];
  s.dof = c.st[4 * n + 2];
  s.tot = s.sc + c.st[4 * n + 3];
  return s;
}
__device__ __forceinline__ void store_event(const Ctx& c, const StoreView& s, int64_t k, int64_t& e, int64_t& other,
                                            float& t) {
  const int64_t kk = max((int64_t)0, min(k, s.tot - 1));
  const bool src = kk < s.sc;
  e = *(src ? c.arena + s.so + kk : c.arena + s.dof + (kk - s.sc));
  other = *(src ? c.ev_dst + e : c.ev_src + e);
  t = c.ev_t[e];
}
// EMB (DyRepMemory use_{src,dst}_emb_in_msg, memory_module.py:387-408; aggregation over the update list
// c.upd only): the memory row of a message endpoint is replaced by the endpoint's embedding when it is in
// the update set n_id = src ∪ dst of the batch — c.upd, sorted; its entry's sampled row (upd_loc) gives its
// centre row (crank), which holds the embedding.  (assoc cannot be used: the batch's ring insert, earlier in
// the step, rewrote it.)  self: the store's own node, list entry m — the `src` of every message it stores.
template <bool EMB>
__device__ __forceinline__ const float* msg_row(const Ctx& c, int64_t v, bool self, int m) {
  if (EMB) {
    int u = -1;
    if (self) {
      if (c.emb & 1) u = m;
    } else if (c.emb & 2) {
      int lo = 0, hi = min(c.cnt[CNT_U], c.Ucap);  // first entry >= v
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (c.upd[mid] < v) lo = mid + 1;
        else hi = mid;
      }
      if (lo < min(c.cnt[CNT_U], c.Ucap) && c.upd[lo] == v) u = lo;
    }
    if (u >= 0) return c.zemb + (int64_t)c.crank[c.upd_loc[u]] * c.HC;
  }
  return c.mem + v * c.D;
}
// AG: the aggregation compiled in (0 last, 1 mean, -1 either by c.aggr): the last-only kernel does not carry
// the mean path's registers (233 -> fewer VGPRs: more tgn_agg_emit workgroups resident at once)
template <int AG, bool EMB = false>
__device__ void agg_node(const Ctx& c, int64_t n, int m, int lane, bool grad) {
  const int D = c.D, d = c.d, Qm = c.Qm, enc0 = 2 * D + d;
  const StoreView sv = store_view(c, n);
  const int tot = (int)sv.tot;
  float* X = c.X + (int64_t)m * Qm;
  const float* P = c.params;
  if (tot == 0) {
    for (int k = lane; k < Qm; k += 64) X[k] = 0.f;
    if (grad)
      for (int q = lane; q < D; q += 64) c.s0m[(int64_t)m * D + q] = c.s1m[(int64_t)m * D + q] = 0.f;
    if (lane == 0) {
      c.xw[m] = -1;
      c.trel[m] = 0.f;
      c.lu[m] = 0.f;
    }
    return;
  }
  const float lun = (float)c.lu_buf[n];
  const float* rowN = msg_row<EMB>(c, n, true, m);
  if (AG == 0 || (AG < 0 && c.aggr == 0)) {
    // winner: max t, first index in [msg_s; msg_d] order
    float tb = -INFINITY;
    int kb = 0x7fffffff;
    int64_t eb = 0, ob = 0;
    for (int k0 = 0; k0 < tot; k0 += 64) {
      int64_t e, o;
      float tt;
      store_event(c, sv, k0 + lane, e, o, tt);
      if (k0 + lane < tot && tt > tb) {
        tb = tt;
        kb = k0 + lane;
        eb = e;
        ob = o;
      }
    }
    const float tm = wave_max_f(tb);
    const int kk = wave_min_i(tb == tm ? kb : 0x7fffffff);
    const int wl = __ffsll(__ballot(kb == kk)) - 1;
    const int64_t e = shfl_i64(eb, wl), other = shfl_i64(ob, wl);
    const float tr = tm - lun;
    const float* rowO = msg_row<EMB>(c, other, false, m);
    const float* raw = c.ev_msg + e * d;
    for (int k0 = lane; k0 < Qm; k0 += 64 * 8) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = min(k0 + 64 * i, Qm - 1);
        const float* p = k < D ? rowN + k : k < 2 * D ? rowO + (k - D) : k < enc0 ? raw + (k - 2 * D) : rowN;
        v[i] = *p;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + 64 * i;
        if (k >= Qm) continue;
        const bool enc = k >= enc0;
        float cs = 0.f;
        if (enc) {
          const int q = k - enc0;
          float sn;
          te_sincos(fmaf(P[c.L.te_w + q], tr, P[c.L.te_b + q]), sn, cs);
          if (grad) {
            c.s0m[(int64_t)m * D + q] = sn;
            c.s1m[(int64_t)m * D + q] = sn * tr;
          }
        }
        X[k] = v[i] * f01(!enc) + cs;
      }
    }
    if (lane == 0) {
      c.xw[m] = e;
      c.trel[m] = tr;
      c.lu[m] = tm;
    }
  } else {
    // mean over the stored events in event order (PyG scatter-sum order, then / count).  Messages are
    // taken AGG_MB at a time with all their row loads in flight (a hub node stores ~100 messages of its
    // last batch: one load round per message made agg_emit 83 us on the review-shaped stream)
    constexpr int AGG_MB = 4;
    const float inv = 1.0f / (float)tot;
    float tmax = -INFINITY;
    for (int k0 = 0; k0 < Qm; k0 += 64 * 8) {
      float s[8], s0[8], s1[8], tw[8], tb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] = s0[i] = s1[i] = 0.f;
        const int qq = min(max(k0 + lane + 64 * i - enc0, 0), D - 1);  // encoding weights of this column
        tw[i] = P[c.L.te_w + qq];
        tb[i] = P[c.L.te_b + qq];
      }
      for (int q0 = 0; q0 < tot; q0 += 64) {
        int64_t e_l, o_l;
        float t_l;
        store_event(c, sv, q0 + lane, e_l, o_l, t_l);
        if (k0 == 0 && q0 + lane < tot) tmax = fmaxf(tmax, t_l);
        const int nq = min(64, tot - q0);
        for (int qb = 0; qb < nq; qb += AGG_MB) {
          float v[AGG_MB][8], dt[AGG_MB];
#pragma unroll
          for (int u = 0; u < AGG_MB; ++u) {
            const int q = min(qb + u, nq - 1);
            const int64_t e = shfl_i64(e_l, q), o = shfl_i64(o_l, q);
            dt[u] = lane_f(t_l, q) - lun;
            const float* rowO = msg_row<EMB>(c, o, false, m);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int k = min(k0 + lane + 64 * i, Qm - 1);
              const float* p = k < D ? rowN + k : k < 2 * D ? rowO + (k - D)
                                                    : k < enc0 ? c.ev_msg + e * d + (k - 2 * D) : rowN;
              v[u][i] = *p;
            }
          }
#pragma unroll
          for (int u = 0; u < AGG_MB; ++u) {
            if (qb + u >= nq) continue;  // (not break: it kept the loop rolled)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int k = k0 + lane + 64 * i;
              const bool enc = k >= enc0 && k < Qm;
              float cs = 0.f, sn = 0.f;
              if (enc) te_sincos(fmaf(tw[i], dt[u], tb[i]), sn, cs);
              s[i] += v[u][i] * f01(!enc) + cs;
              s0[i] += sn;
              s1[i] += sn * dt[u];
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + lane + 64 * i;
        if (k >= Qm) continue;
        X[k] = s[i] / (float)tot;
        if (grad && k >= enc0) {
          c.s0m[(int64_t)m * D + (k - enc0)] = s0[i] * inv;
          c.s1m[(int64_t)m * D + (k - enc0)] = s1[i] * inv;
        }
      }
    }
    tmax = wave_max_f(tmax);
    if (lane == 0) {
      c.xw[m] = 1;
      c.trel[m] = 0.f;
      c.lu[m] = tmax;
    }
  }
}

// MeanAggregator for one node by a whole workgroup (train step): the node's stored messages are split
// into 4 contiguous ranges, one per wave, and the partial sums combine in LDS in wave order.  A hub node
// of the review-shaped stream stores ~100-200 messages of its last batch; one wave evaluating D
// time-encoding sin/cos pairs per message ran 84 us (agg_emit), all other waves done long before.
template <bool EMB = false>
__device__ void agg_node_mean_wg(const Ctx& c, int64_t n, int m, bool grad) {
  __shared__ float red[4][3][8][64];
  __shared__ float rmax[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D = c.D, d = c.d, Qm = c.Qm, enc0 = 2 * D + d;
  const StoreView sv = store_view(c, n);
  const int tot = (int)sv.tot;
  float* X = c.X + (int64_t)m * Qm;
  if (tot == 0) {  // workgroup-uniform
    if (w == 0) {
      for (int k = lane; k < Qm; k += 64) X[k] = 0.f;
      if (grad)
        for (int q = lane; q < D; q += 64) c.s0m[(int64_t)m * D + q] = c.s1m[(int64_t)m * D + q] = 0.f;
      if (lane == 0) {
        c.xw[m] = -1;
        c.trel[m] = 0.f;
        c.lu[m] = 0.f;
      }
    }
    return;
  }
  const float lun = (float)c.lu_buf[n];
  const float* rowN = msg_row<EMB>(c, n, true, m);
  const float* P = c.params;
  const int qa = w * tot / 4, qe = (w + 1) * tot / 4;  // this wave's messages (event order)
  constexpr int AGG_MB = 4;
  const float inv = 1.0f / (float)tot;
  float tmax = -INFINITY;
  for (int k0 = 0; k0 < Qm; k0 += 64 * 8) {
    float s[8], s0[8], s1[8], tw[8], tb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s[i] = s0[i] = s1[i] = 0.f;
      const int qq = min(max(k0 + lane + 64 * i - enc0, 0), D - 1);
      tw[i] = P[c.L.te_w + qq];
      tb[i] = P[c.L.te_b + qq];
    }
    for (int q0 = qa; q0 < qe; q0 += 64) {
      int64_t e_l, o_l;
      float t_l;
      store_event(c, sv, q0 + lane, e_l, o_l, t_l);
      if (k0 == 0 && q0 + lane < qe) tmax = fmaxf(tmax, t_l);
      const int nq = min(64, qe - q0);
      for (int qb = 0; qb < nq; qb += AGG_MB) {
        float v[AGG_MB][8], dt[AGG_MB];
#pragma unroll
        for (int u = 0; u < AGG_MB; ++u) {
          const int q = min(qb + u, nq - 1);
          const int64_t e = shfl_i64(e_l, q), o = shfl_i64(o_l, q);
          dt[u] = lane_f(t_l, q) - lun;
          const float* rowO = msg_row<EMB>(c, o, false, m);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int k = min(k0 + lane + 64 * i, Qm - 1);
            const float* p = k < D ? rowN + k : k < 2 * D ? rowO + (k - D)
                                                  : k < enc0 ? c.ev_msg + e * d + (k - 2 * D) : rowN;
            v[u][i] = *p;
          }
        }
#pragma unroll
        for (int u = 0; u < AGG_MB; ++u) {
          if (qb + u >= nq) continue;  // (not break: it kept the loop rolled)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int k = k0 + lane + 64 * i;
            const bool enc = k >= enc0 && k < Qm;
            float cs = 0.f, sn = 0.f;
            if (enc) te_sincos(fmaf(tw[i], dt[u], tb[i]), sn, cs);
            s[i] += v[u][i] * f01(!enc) + cs;
            s0[i] += sn;
            s1[i] += sn * dt[u];
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[w][0][i][lane] = s[i];
      red[w][1][i][lane] = s0[i];
      red[w][2][i][lane] = s1[i];
    }
    if (k0 == 0) {
      const float wm = wave_max_f(tmax);
      if (lane == 0) rmax[w] = wm;
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + lane + 64 * i;
        if (k >= Qm) continue;
        const float a = ((red[0][0][i][lane] + red[1][0][i][lane]) + red[2][0][i][lane]) + red[3][0][i][lane];
        X[k] = a / (float)tot;
        if (grad && k >= enc0) {
          const float b0 = ((red[0][1][i][lane] + red[1][1][i][lane]) + red[2][1][i][lane]) + red[3][1][i][lane];
          const float b1 = ((red[0][2][i][lane] + red[1][2][i][lane]) + red[2][2][i][lane]) + red[3][2][i][lane];
          c.s0m[(int64_t)m * D + (k - enc0)] = b0 * inv;
          c.s1m[(int64_t)m * D + (k - enc0)] = b1 * inv;
        }
      }
      if (k0 == 0 && lane == 0) {
        c.xw[m] = 1;
        c.trel[m] = 0.f;
        c.lu[m] = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
      }
    }
    __syncthreads();
  }
}

// The same MeanAggregator (train step, d <= 192) with lanes over the message's COLUMN CLASSES instead of
// 8 generic X columns: per message a lane loads only what varies — its 2 columns of the other endpoint's
// memory row and its <= 3 raw-message columns (the node's own row is loaded once, the D encoding columns
// are computed) — so 16 messages' rows are in flight per round instead of 4: a hub node of the
// review-shaped stream (~50 messages per wave) walks 4 dependent load rounds instead of 13.  Sums run in
// the same order as agg_node_mean_wg (per wave in event order, waves combined 0..3): bit-identical X rows.
#ifndef TGNX_AGG_MC1
#define TGNX_AGG_MC1 12  // messages per load round of the mean path at d <= 64 (review-shaped A/Bs: 12 0.1025 ms, 8 0.1027, 16 0.1025-0.1037, 24 0.1045, 32 0.1052)
#endif
// RB raw-message columns per lane (3: d <= 192; 1: d <= 64), MC messages whose rows are loaded in one round
// (the same load registers: 16 x (2 + 3) or 24 x (2 + 1))
template <bool EMB = false, int RB = 3, int MC = 16>
__device__ void agg_node_mean_cols(const Ctx& c, int64_t n, int m, bool grad) {
  __shared__ float red[4][3 * TDMAX + 192 + 2 * TDMAX];  // per wave: X columns (Qm) | sin sums | sin·Δt sums
  __shared__ float rmax[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int D = c.D, d = c.d, Qm = c.Qm, enc0 = 2 * D + d;
  const StoreView sv = store_view(c, n);
  const int tot = (int)sv.tot;
  float* X = c.X + (int64_t)m * Qm;
  if (tot == 0) {  // workgroup-uniform
    if (w == 0) {
      for (int k = lane; k < Qm; k += 64) X[k] = 0.f;
      if (grad)
        for (int q = lane; q < D; q += 64) c.s0m[(int64_t)m * D + q] = c.s1m[(int64_t)m * D + q] = 0.f;
      if (lane == 0) {
        c.xw[m] = -1;
        c.trel[m] = 0.f;
        c.lu[m] = 0.f;
      }
    }
    return;
  }
  const float lun = (float)c.lu_buf[n];
  const float* rowN = msg_row<EMB>(c, n, true, m);
  const float* P = c.params;
  // this lane's columns: memory / encoding j = lane + 64 a (j < D), raw r = lane + 64 b (r < d)
  float nv[2], tw[2], tb[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int j = min(lane + 64 * a, D - 1);
    nv[a] = rowN[j];
    tw[a] = P[c.L.te_w + j];
    tb[a] = P[c.L.te_b + j];
  }
  float sN[2] = {0.f, 0.f}, sO[2] = {0.f, 0.f}, sC[2] = {0.f, 0.f}, s0[2] = {0.f, 0.f}, s1[2] = {0.f, 0.f};
  float sR[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) sR[b] = 0.f;
  const int qa = w * tot / 4, qe = (w + 1) * tot / 4;  // this wave's messages (event order)
  float tmax = -INFINITY;
  for (int q0 = qa; q0 < qe; q0 += 64) {
    int64_t e_l, o_l;
    float t_l;
    store_event(c, sv, q0 + lane, e_l, o_l, t_l);
    if (q0 + lane < qe) tmax = fmaxf(tmax, t_l);
    const int nq = min(64, qe - q0);
    for (int qb = 0; qb < nq; qb += MC) {
      float vo[MC][2], vr[MC][RB];
#pragma unroll
      for (int u = 0; u < MC; ++u) {
        const int q = min(qb + u, nq - 1);
        const int64_t e = shfl_i64(e_l, q), o = shfl_i64(o_l, q);
        const float* rowO = msg_row<EMB>(c, o, false, m);
        const float* raw = c.ev_msg + e * d;
#pragma unroll
        for (int a = 0; a < 2; ++a) vo[u][a] = rowO[min(lane + 64 * a, D - 1)];
#pragma unroll
        for (int b = 0; b < RB; ++b) vr[u][b] = raw[min(lane + 64 * b, d - 1)];
      }
#pragma unroll
      for (int u = 0; u < MC; ++u) {
        if (qb + u >= nq) continue;  // (not break: it kept the loop rolled)
        const float dt = lane_f(t_l, qb + u) - lun;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          float sn, cs;
          te_sincos(fmaf(tw[a], dt, tb[a]), sn, cs);
          sN[a] += nv[a];
          sO[a] += vo[u][a];
          sC[a] += cs;
          s0[a] += sn;
          s1[a] += sn * dt;
        }
#pragma unroll
        for (int b = 0; b < RB; ++b) sR[b] += vr[u][b];
      }
    }
  }
  float* rw = red[w];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int j = lane + 64 * a;
    if (j < D) {
      rw[j] = sN[a];
      rw[D + j] = sO[a];
      rw[enc0 + j] = sC[a];
      rw[Qm + j] = s0[a];
      rw[Qm + D + j] = s1[a];
    }
  }
#pragma unroll
  for (int b = 0; b < RB; ++b)
    if (lane + 64 * b < d) rw[2 * D + lane + 64 * b] = sR[b];
  const float wm = wave_max_f(tmax);
  if (lane == 0) rmax[w] = wm;
  __syncthreads();
  const float inv = 1.0f / (float)tot;
  for (int k = threadIdx.x; k < Qm; k += blockDim.x)
    X[k] = (((red[0][k] + red[1][k]) + red[2][k]) + red[3][k]) / (float)tot;
  if (grad)
    for (int j = threadIdx.x; j < D; j += blockDim.x) {
      const int k0 = Qm + j, k1 = Qm + D + j;
      c.s0m[(int64_t)m * D + j] = (((red[0][k0] + red[1][k0]) + red[2][k0]) + red[3][k0]) * inv;
      c.s1m[(int64_t)m * D + j] = (((red[0][k1] + red[1][k1]) + red[2][k1]) + red[3][k1]) * inv;
    }
  if (threadIdx.x == 0) {
    c.xw[m] = 1;
    c.trel[m] = 0.f;
    c.lu[m] = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
  }
  __syncthreads();
}

// last_update the GRU step gives node u (memory_module.py:175-176): max t over its stored messages, 0
// without messages (PyG scatter 'max' fill); wave-uniform
__device__ float store_tmax(const Ctx& c, int64_t u, int lane) {
  const StoreView sv = store_view(c, u);
  if (sv.tot == 0) return 0.f;
  float tb = -INFINITY;
  for (int64_t k0 = 0; k0 < sv.tot; k0 += 64) {
    const int64_t kk = min(k0 + lane, sv.tot - 1);
    const int64_t e = *(kk < sv.sc ? c.arena + sv.so + kk : c.arena + sv.dof + (kk - sv.sc));
    tb = fmaxf(tb, c.ev_t[e]);   // clamped duplicates of the last event do not change the max
  }
  return wave_max_f(tb);
}

// row of a root's embedding: its centre index (2 hops: its root index, via the outer centre)
__device__ __forceinline__ int root_row(const Ctx& c, int64_t v) {
  const int x = c.crank[c.assoc[v]];
  return c.x2r ? c.x2r[x] : x;
}

// K3: blocks [0, nedge): one wave per (centre x, ring slot j) — the sampled edge record (centre-
// ascending, ring order = e_id descending, neighbor_loader.py:26-50; output slot = the centre's edge
// offset + valid slots before j, by ballot) and its Δt encoding (cos -> the lin_edge operand, sin ->
// its backward; emb_module.py:69-72, rel_t = last_update[src] - t, with last_update as the GRU step
// gives it: the max t of the neighbour's stored messages, 0 without any).  Every load of a wave
// depends on at most the previous round (ring row; neighbour; its store; arena; t).
// The rest: mode 0 aggregation over the sampled nodes (train) + zeroing of the backward
// accumulators, mode 1 last_update of the sampled nodes from the buffer (eval scoring), mode 2
// aggregation over a node list (eval update / flush; list == nullptr: nodes base + m).
// zero n floats at p as threads [t, t + nt) of the launch (4-B stores: 16-B ones, and the zeroing moved to the
// edge blocks, measured slower, r5_agg_zero_ab.txt)
__device__ __forceinline__ void zero_span(float* p, int64_t n, int64_t t, int64_t nt) {
  for (int64_t x = t; x < n; x += nt) p[x] = 0.f;
}
// the atomically accumulated backward rows of a train step: dP; 1 hop the dZc copies; 2 hops dP2 (conv2 projections
// of the outer centres) and the root level's dZr copies (dZc = dh1 is written whole by a GEMM)
__device__ void zero_bwd_acc(const Ctx& c, int64_t t, int64_t nt) {
  const int M = c.cnt[CNT_M], R = c.cnt[CNT_R];
  zero_span(c.dP, (int64_t)M * 4 * c.HC, t, nt);
  if (c.layers == 2) {
    const int R1 = c.cnt[CNT_R1];
    zero_span(c.dP2, (int64_t)R * 4 * c.HC, t, nt);
    for (int rp = 0; rp < c.dzrep1; ++rp) zero_span(c.dZr + rp * c.dzstride1, (int64_t)R1 * c.HC, t, nt);
  } else {
    for (int rp = 0; rp < c.dzrep; ++rp) zero_span(c.dZc + rp * c.dzstride, (int64_t)R * c.HC, t, nt);
  }
}
#ifndef TGNX_AGG_WAVES
#define TGNX_AGG_WAVES 0  // waves-per-SIMD floor of tgn_agg_emit (0: the compiler's register count)
#endif
#if TGNX_AGG_WAVES > 0
#define TGNX_AGG_ATTR __attribute__((amdgpu_waves_per_eu(TGNX_AGG_WAVES)))
#else
#define TGNX_AGG_ATTR
#endif
template <int AG, bool EMB = false>
__global__ void __launch_bounds__(256) TGNX_AGG_ATTR tgn_agg_emit(Ctx c, int mode, int nedge, const int64_t* list,
                                                    const int* list_cnt, int n_host, int64_t base, int nevb = 0) {
  TGNX_STAMP(3);
  if (mode != 2) {
    const int B = (int)c.ctl[TGNX_CTL_B];
    if (c.tagchk && blockIdx.x == 0 && threadIdx.x == 0 && B > 0 && c.cnt[CNT_NB] != (int)c.ctl[TGNX_CTL_NB])
      c.ctl[TGNX_CTL_ERR] |= ERR_STALE_SET;  // (this launch's other blocks may compute garbage; later launches skip)
    if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  }
  const int lane = threadIdx.x & 63;
  if ((int)blockIdx.x < nevb) {  // train: the centre row of every root of this rank's events, so that
                                 // tgn_pred_train starts from one index load (root_row: assoc -> rank)
    const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
    const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
    if (c.evj) {  // 16 lanes per root: its record and its edges' neighbour rows (ring slot order, valid
                  // slots compacted: the e_j of its edge range), so the attention in tgn_pred_train<ATT>
                  // reads q, skip and every k / v / edge row in its second round
      const int sl = threadIdx.x & 15, K = c.K;
      for (int x = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; x < 3 * (hi - lo); x += (nevb * blockDim.x) >> 4) {
        const int i = lo + x / 3, r = x % 3;
        const int64_t* src = r == 0 ? c.ev_src : r == 1 ? c.ev_dst : c.neg;
        const int64_t v = src[start + i];
        const int a = (int)c.assoc[v];
        const int64_t e = c.eid[v * K + min(sl, K - 1)], u = c.nbr[v * K + min(sl, K - 1)];
        const bool ok = sl < K && e >= 0;
        const uint32_t m = (uint32_t)(__ballot(ok) >> (threadIdx.x & 48)) & 0xFFFFu;
        const int xr = c.crank[a];
        const int ju = (int)c.assoc[ok ? u : v];
        if (ok) {
          const int idx = __popc(m & ((1u << sl) - 1u));
          c.evj[x * 16 + idx] = ju;
          c.cevj[xr * 16 + idx] = ju;
        }
        if (sl == 0) {
          const int e0 = c.ceoff[xr], e1 = c.ceoff[xr + 1];
          c.evr[x] = xr;
          c.evq[x] = make_int4(xr, a, e0, e1);
          c.cevq[xr] = make_int4(a, e0, e1, 0);
        }
      }
      return;
    }
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < 3 * (hi - lo); x += nevb * blockDim.x) {
      const int i = lo + x / 3, r = x % 3;
      const int64_t* src = r == 0 ? c.ev_src : r == 1 ? c.ev_dst : c.neg;
      if (c.evq) {  // 1 hop: the root's centre row, its P row and edge range (one round for the attention)
        const int a = (int)c.assoc[src[start + i]], xr = c.crank[a];
        c.evr[x] = xr;
        c.evq[x] = make_int4(xr, a, c.ceoff[xr], c.ceoff[xr + 1]);
      } else {
        c.evr[x] = root_row(c, src[start + i]);
      }
    }
    return;
  }
  // then the node part (its workgroups run longest: hub nodes' stores), the sampled-edge part in the last
  // nedge blocks; both loop over their runtime work in strides of their block count
  const int nnode = gridDim.x - nedge - nevb;
  if ((int)blockIdx.x >= nevb + nnode) {
    const int R = c.cnt[CNT_R], K = c.K, D = c.D;
    const float* tw = c.params + c.L.te_w;
    const float* tb = c.params + c.L.te_b;
    for (int pr = ((int)blockIdx.x - nevb - nnode) * 4 + (threadIdx.x >> 6); pr < R * K; pr += nedge * 4) {
      const int x = pr / K, j = pr - x * K;
      const int64_t v = c.cent[x];
      const int ls = min(lane, K - 1);
      const int64_t e_l = c.eid[v * K + ls];
      const int64_t u_l = c.nbr[v * K + ls];
      const float t_l = c.rt[v * K + ls];
      const uint64_t valid = __ballot(lane < K && e_l >= 0);
      if (!((valid >> j) & 1ull)) continue;
      const int o = c.ceoff[x] + __popcll(valid & ((1ull << j) - 1ull));
      const int64_t e = shfl_i64(e_l, j), u = shfl_i64(u_l, j);
      const float te = lane_f(t_l, j);
      const int ju = (int)c.assoc[u];
      const float lu = mode == 0 ? store_tmax(c, u, lane) : (float)c.lu_buf[u];
      if (lane == 0) {
        c.e_j[o] = ju;
        c.e_c[o] = x;
        c.e_id[o] = e;
        c.e_t[o] = te;
      }
      if (c.x2r && lane == 1) {  // 2 hops: a root's edges are its outer edges, same slot order
        const int x1 = c.x2r[x];
        if (x1 >= 0) {
          const int o1 = c.ceoff1[x1] + (o - c.ceoff[x]);
          c.e1_j[o1] = c.crank[ju];
          c.e1_e2[o1] = o;
          c.e1_id[o1] = e;
        }
      }
      const float dt = lu - te;
      if (mode == 0) {  // train: the edge's whole lin_edge operand row [cos enc | msg] (stride D + d), so the
                        // lin_edge / dW_edge GEMMs read dense rows (no event-id gather round per K chunk)
        const int d = c.d, DA = D + d;
        float* row = c.encE + (int64_t)o * DA;
        const float* msg = c.ev_msg + e * d;
        float mv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) mv[i] = msg[min(lane + 64 * i, max(d - 1, 0))];  // (loads before the sincos)
        // (the backward recomputes the sine from the same argument, EpiTeEdge: no [E][D] sine round trip)
        for (int q = lane; q < D; q += 64) row[q] = te_cos(fmaf(tw[q], dt, tb[q]));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (lane + 64 * i < d) row[D + lane + 64 * i] = mv[i];
        for (int q = lane + 256; q < d; q += 64) row[D + q] = msg[q];
      } else {
        for (int q = lane; q < D; q += 64) c.encE[(int64_t)o * D + q] = te_cos(fmaf(tw[q], dt, tb[q]));
      }
    }
    return;
  }
  const int bid = blockIdx.x - nevb, nb = nnode;
  if (mode == 1) {
    const int M = c.cnt[CNT_M];
    for (int x = bid * blockDim.x + threadIdx.x; x < M; x += nb * blockDim.x) c.lu[x] = (float)c.lu_buf[c.nid[x]];
    return;
  }
  if (mode == 0)  // zero the atomically accumulated backward rows
    zero_bwd_acc(c, bid * (int64_t)blockDim.x + threadIdx.x, (int64_t)nb * blockDim.x);
  const int n = mode == 0 ? c.cnt[CNT_M] : (list_cnt ? *list_cnt : n_host);
  if (AG != 0 && c.aggr == 1 && (mode == 0 || list)) {  // MeanAggregator, train / eval update: a workgroup per node (hub
                                             // nodes store many messages); the all-node flush stays wave-per-node
    if (AG == 1 || c.d <= 192) {  // (AG == 1 is launched for d <= 192 only)
      if (c.d <= 64)
        for (int m = bid; m < n; m += nb) agg_node_mean_cols<EMB, 1, TGNX_AGG_MC1>(c, mode == 0 ? c.nid[m] : list[m], m, mode == 0);
      else
        for (int m = bid; m < n; m += nb) agg_node_mean_cols<EMB>(c, mode == 0 ? c.nid[m] : list[m], m, mode == 0);
    } else {
      for (int m = bid; m < n; m += nb) agg_node_mean_wg<EMB>(c, mode == 0 ? c.nid[m] : list[m], m, mode == 0);
    }
    return;
  }
  if constexpr (AG == 1) return;  // (launched for train steps only: the mean path above)
  for (int m = bid * 4 + (threadIdx.x >> 6); m < n; m += nb * 4) {
    const int64_t v = mode == 0 ? c.nid[m] : (list ? list[m] : base + m);
    agg_node<AG, EMB>(c, v, m, lane, mode == 0);
  }
}

// ------------------------------------------------------------------ GEMM operands / epilogues
// Constant operand entries come from these (a pointer select before the load), never from arithmetic on a
// loaded value: `v * 0/1 + c` in a loader made the compiler wait for the load right where fetch() issued it
// (s_waitcnt vmcnt after every chunk's load), so the next chunk's operands were never in flight during the
// current chunk's MFMAs — every K chunk of the GRU GEMM paid a whole load latency.
__device__ __attribute__((aligned(16))) float kZero4[4] = {0.f, 0.f, 0.f, 0.f};
__device__ __attribute__((aligned(16))) float kOne4[4] = {1.f, 1.f, 1.f, 1.f};
// GRU input row m: [aggregated message (Qm) | memory of the node (D)]
struct LoadGruA {
  const float* X;
  const float* mem;
  const int64_t* list;  // node of row m; with `ident`, rows are nodes base + m (list: any valid array)
  int64_t base;
  int Qm, D, ident;
  static constexpr bool k_fast = true;
  using Idx = int64_t;  // the row's node (hoisted out of the K loop)
  static constexpr bool row_idx = true;
  // unconditional load + select: a branch here merges the loaded value in a phi, i.e. one
  // s_waitcnt per element
  __device__ Idx index(int m, int) const {
    const int64_t v = list[m];
    return ident ? base + m : v;
  }
  __device__ float load(Idx v, int m, int k) const {
    const float* p = k < Qm ? X + (int64_t)m * Qm + k : mem + v * D + (k - Qm);
    return *p;
  }
  __device__ bool vec4() const { return ((Qm | D) & 3) == 0 && al16(X) && al16(mem); }
  __device__ float4 load4(Idx v, int m, int k) const {
    const float* p = k < Qm ? X + (int64_t)m * Qm + k : mem + v * D + (k - Qm);
    return *reinterpret_cast<const float4*>(p);
  }
};
// GRU weights with gates interleaved by unit: row 4j+g = (r, z, n_input, n_hidden) of unit j over
// the columns [message | memory] (GRUCell weight_ih [3D, Qm], weight_hh [3D, D]).
struct LoadGruW {
  const float *wih, *whh;
  int Qm, D;
  static constexpr bool k_fast = true;
  __device__ const float* at(int n, int k) const {  // branch-free; the zero blocks read kZero4
    const int j = n >> 2, g = n & 3;
    const bool ih = k < Qm;
    const int gr = ih ? min(g, 2) : (g == 3 ? 2 : g);  // weight row block (clamped: always a valid row)
    const bool zero = ih ? g == 3 : g == 2;
    const float* p = ih ? wih + (int64_t)(gr * D + j) * Qm + k : whh + (int64_t)(gr * D + j) * D + (k - Qm);
    return zero ? kZero4 : p;
  }
  __device__ float operator()(int n, int k) const { return *at(n, k); }
  __device__ bool vec4() const { return ((Qm | D) & 3) == 0 && al16(wih) && al16(whh); }
  __device__ float4 load4(int n, int k) const { return *reinterpret_cast<const float4*>(at(n, k)); }
};
// GRUCell (torch gru_cell: r, z = σ(gi + gh), n = tanh(gi_n + r gh_n), h' = (h - n) z + n)
struct EpiGru {
  const float *bih, *bhh, *mem;
  const int64_t* list;
  int64_t base;
  int D;
  float *Z0, *gates;
  float* Hp = nullptr;  // (train step) the row's pre-update memory, stored densely
  // thread x < 64 of a 16 x 16 tile: row x / 4, unit n0 / 4 + x % 4 — its biases and memory entry, loaded
  // with the tile's first operand round (gemm_tile_direct); rowidx(r) = row r's node (LoadGruA's index)
  struct Pre {
    float bs[6], h;
  };
  template <class RI>
  __device__ Pre pre(int m0, int n0, int M, int N, RI rowidx) const {
    Pre p;
    const int x = threadIdx.x & 63, r = x >> 2, u = x & 3;
    const int64_t v = rowidx(r);  // (every lane takes part in the shuffle)
    const int j = min(n0 / 4 + u, max(N / 4 - 1, 0));
    p.bs[0] = bih[j]; p.bs[1] = bhh[j];
    p.bs[2] = bih[D + j]; p.bs[3] = bhh[D + j];
    p.bs[4] = bih[2 * D + j]; p.bs[5] = bhh[2 * D + j];
    p.h = mem[v * D + j];
    return p;
  }
  template <class T>
  __device__ void operator()(const T& t, const Pre& p) const {
    static_assert(T::tm * T::tn / 4 <= 64, "one wave of (row, unit) items");
    const int q4 = t.tn / 4, x = threadIdx.x;
    if (x >= t.tm * q4) return;
    const int r = x / q4, u = x % q4, m = t.m0 + r, j = t.n0 / 4 + u;
    if (m >= t.M || 4 * j >= t.N) return;
    const float* row = t.c + r * t.pitch + 4 * u;
    const float pr = row[0] + (p.bs[0] + p.bs[1]);
    const float pz = row[1] + (p.bs[2] + p.bs[3]);
    const float gin = row[2] + p.bs[4];
    const float ghn = row[3] + p.bs[5];
    const float rr = sigm(pr), zz = sigm(pz);
    const float nn = tanhf(gin + rr * ghn);
    Z0[(int64_t)m * D + j] = (p.h - nn) * zz + nn;
    float4* gp = reinterpret_cast<float4*>(gates + ((int64_t)m * D + j) * 4);
    *gp = make_float4(rr, zz, nn, ghn);
    if (Hp) Hp[(int64_t)m * D + j] = p.h;
  }
  template <class T>  // (staged tiles of any shape: the loads after the MFMAs)
  __device__ void operator()(const T& t) const {
    const int q4 = t.tn / 4;
    for (int x = threadIdx.x; x < t.tm * q4; x += blockDim.x) {
      const int r = x / q4, u = x % q4, m = t.m0 + r, j = t.n0 / 4 + u;
      if (m >= t.M || 4 * j >= t.N) continue;
      const float* row = t.c + r * t.pitch + 4 * u;
      const float pr = row[0] + (bih[j] + bhh[j]);
      const float pz = row[1] + (bih[D + j] + bhh[D + j]);
      const float gin = row[2] + bih[2 * D + j];
      const float ghn = row[3] + bhh[2 * D + j];
      const float rr = sigm(pr), zz = sigm(pz);
      const float nn = tanhf(gin + rr * ghn);
      const int64_t v = list ? list[m] : base + m;
      const float h = mem[v * D + j];
      Z0[(int64_t)m * D + j] = (h - nn) * zz + nn;
      float4* gp = reinterpret_cast<float4*>(gates + ((int64_t)m * D + j) * 4);
      *gp = make_float4(rr, zz, nn, ghn);
      if (Hp) Hp[(int64_t)m * D + j] = h;
    }
  }
};
// TransformerConv edge attribute of sampled edge e: [cos(w (lu[src] - t_e) + b) | msg[e_id]]
// (emb_module.py:69-72, rel_t = last_update[edge_index[0]] - t)
struct LoadEdgeAttr {
  const float* enc;  // cos(w rel_t + b) rows, written by tgn_agg_emit
  const int64_t* e_id;
  const float* ev_msg;
  int D, d;
  static constexpr bool k_fast = true;
  using Idx = int64_t;  // the edge's event id (msg row)
  static constexpr bool row_idx = true;
  __device__ Idx index(int e, int) const { return e_id[e]; }
  __device__ float load(Idx id, int e, int k) const {
    const float* p = k < D ? enc + (int64_t)e * D + k : ev_msg + id * d + (k - D);
    return *p;
  }
  __device__ bool vec4() const { return ((D | d) & 3) == 0 && al16(enc) && al16(ev_msg); }
  __device__ float4 load4(Idx id, int e, int k) const {
    const float* p = k < D ? enc + (int64_t)e * D + k : ev_msg + id * d + (k - D);
    return *reinterpret_cast<const float4*>(p);
  }
};
// same operand with rows / columns swapped (B operand of dW_edge = dEᵀ EA)
struct LoadEdgeAttrT {
  LoadEdgeAttr a;
  static constexpr bool k_fast = false;
  using Idx = int64_t;  // k = edge: the index changes per chunk
  static constexpr bool row_idx = false;
  __device__ Idx index(int, int e) const { return a.e_id[e]; }
  __device__ float load(Idx id, int n, int e) const { return a.load(id, e, n); }
};
// 2 hops: the edge attribute of root edge e = that of its outer edge e1_e2[e] (same Δt encoding row,
// same message row); both index loads are independent
struct EdgeRef {
  int64_t id;
  int e2;
};
struct LoadEdgeAttrMap {
  const float* enc;
  const int64_t* e1_id;
  const int* e1_e2;
  const float* ev_msg;
  int D, d;
  static constexpr bool k_fast = true;
  using Idx = EdgeRef;
  static constexpr bool row_idx = true;
  __device__ Idx index(int e, int) const { return EdgeRef{e1_id[e], e1_e2[e]}; }
  __device__ float load(const Idx& r, int, int k) const {
    const float* p = k < D ? enc + (int64_t)r.e2 * D + k : ev_msg + r.id * d + (k - D);
    return *p;
  }
  __device__ bool vec4() const { return ((D | d) & 3) == 0 && al16(enc) && al16(ev_msg); }
  __device__ float4 load4(const Idx& r, int, int k) const {
    const float* p = k < D ? enc + (int64_t)r.e2 * D + k : ev_msg + r.id * d + (k - D);
    return *reinterpret_cast<const float4*>(p);
  }
};
struct LoadEdgeAttrMapT {
  LoadEdgeAttrMap a;
  static constexpr bool k_fast = false;
  using Idx = EdgeRef;
  static constexpr bool row_idx = false;
  __device__ Idx index(int, int e) const { return a.index(e, 0); }
  __device__ float load(const Idx& r, int n, int e) const { return a.load(r, e, n); }
};
// node-embedding input row m: train z0 (GRU output), eval memory[nid[m]] (memory_module.py:121-122)
// train: row e of a root-level edge operand = row map[e] of the outer edges' [cos enc | msg] rows (2 hops)
struct LoadAttrMap {
  const float* rows;
  const int* map;
  int ld;
  static constexpr bool k_fast = true;
  using Idx = int;
  static constexpr bool row_idx = true;
  __device__ Idx index(int e, int) const { return map[e]; }
  __device__ float load(Idx r, int, int k) const { return rows[(int64_t)r * ld + k]; }
  __device__ bool vec4() const { return (ld & 3) == 0 && al16(rows); }
  __device__ float4 load4(Idx r, int, int k) const { return *reinterpret_cast<const float4*>(rows + (int64_t)r * ld + k); }
};
struct LoadAttrMapT {
  LoadAttrMap a;
  static constexpr bool k_fast = false;
  using Idx = int;  // k = root edge: the index changes per chunk
  static constexpr bool row_idx = false;
  __device__ Idx index(int, int e) const { return a.map[e]; }
  __device__ float load(Idx r, int n, int) const { return a.rows[(int64_t)r * a.ld + n]; }
};
struct LoadZ {
  const float* Z0;
  const float* mem;
  const int64_t* nid;
  int D, eval;
  static constexpr bool k_fast = true;
  using Idx = int64_t;
  static constexpr bool row_idx = true;
  __device__ Idx index(int m, int) const {
    const int64_t v = nid[m];
    return eval ? v : 0;
  }
  __device__ float load(Idx v, int m, int k) const {
    const float* p = eval ? mem + v * D + k : Z0 + (int64_t)m * D + k;
    return *p;
  }
  __device__ bool vec4() const { return (D & 3) == 0 && al16(Z0) && al16(mem); }
  __device__ float4 load4(Idx v, int m, int k) const {
    const float* p = eval ? mem + v * D + k : Z0 + (int64_t)m * D + k;
    return *reinterpret_cast<const float4*>(p);
  }
};
// row n < 4 HC of the stacked projections [q; k; v; skip] -> (linear g, row r): compares, not an integer
// division (a ~40-instruction routine per element inside the GEMM loaders' K loop)
__device__ __forceinline__ int proj_g(int n, int HC) { return (n >= HC) + (n >= 2 * HC) + (n >= 3 * HC); }
// stacked [W_query; W_key; W_value; W_skip] rows (n / HC selects the linear)
struct LoadProjW {
  const float* w;  // wq; projection g at w + g * pw
  int64_t pw;
  int HC, D;
  static constexpr bool k_fast = true;
  __device__ float operator()(int n, int k) const {
    const int g = proj_g(n, HC), r = n - g * HC;
    return w[g * pw + (int64_t)r * D + k];
  }
  __device__ bool vec4() const { return ((D | (int)pw) & 3) == 0 && al16(w); }
  __device__ float4 load4(int n, int k) const {
    const int g = proj_g(n, HC), r = n - g * HC;
    return *reinterpret_cast<const float4*>(w + g * pw + (int64_t)r * D + k);
  }
};
struct EpiProj {
  const float* b;  // bq; projection g at b + g * pb
  int64_t pb;
  float* P;
  int HC;
  template <class T>
  __device__ void operator()(const T& t) const {
    float v[T::per];
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int n = t.n0 + T::col_of(i);
      const int g = proj_g(n, HC), q = n - g * HC;
      v[i] = t(T::row_of(i), T::col_of(i)) + (n < t.N ? b[g * pb + q] : 0.f);
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int m = t.m0 + T::row_of(i), n = t.n0 + T::col_of(i);
      if (m < t.M && n < t.N) P[(int64_t)m * t.N + n] = v[i];
    }
  }
};

// ------------------------------------------------------------------ attention (TransformerConv)
// Wave per centre x (node row i): lane l < C holds channel l (head 0) and C + l (head 1).
// P row = [q | k | v | skip] (lin_query / key / value / skip + biases); Ep row = lin_edge(edge_attr).
// score_eh = (q_i · (k_j + e))_h / sqrt(C); alpha = PyG softmax (max-shifted, +1e-16); attention
// dropout (train); out_i = Σ_e alpha~ (v_j + e) + skip_i.  Lane e keeps edge e's per-edge scalars.
// keyed by (centre node, neighbour e_id): the same mask whichever rank / batch position samples the edge
__device__ __forceinline__ float att_keep(const Ctx& c, uint64_t seed, int x, int e, int h) {
  return keep32(drop_base(seed, (uint64_t)c.att_salt, (uint64_t)c.cent[x], (uint64_t)c.e_id[e]), (uint32_t)h, c.p,
                c.inv_keep);
}
constexpr int ATT_EB = 16;  // edges whose neighbour rows are loaded in one batch (ring K <= 32: <= 2 batches)
// TransformerConv forward of centre x (row i of P, edges [e0, e0 + ne)), one wave: returns this lane's
// output pair (channel lane of both heads, lane < C).  A centre with 1..ATT_EB edges issues the k, v and
// edge rows of every edge and its skip row as one round (each edge row loaded once for k + e and v + e);
// longer rings walk ATT_EB-edge load batches.  Train: the softmax weights go to alpha (tgn_attn_bwd).
// jrec >= 0 (a per-root record, lanes 0..ne-1): lane e's neighbour row of edge e, instead of e_j
// st != nullptr (train): the alpha / alk / Qo stores are left in *st for the caller to issue later (tgn_pred_train
// issues them after its first barrier: an LDS read after that barrier waits for vmcnt(0) — the staging wave's LDS-DMA
// is tracked by vmcnt — and would otherwise wait for these stores to land)
struct AttnStores {
  float a0, a1, t0, t1, q0, q1, o0, o1;
  int x, e0, ne;
  __device__ void issue(const Ctx& c, int lane) const {
    if (lane < ne) {
      c.alpha[(int64_t)(e0 + lane) * 2] = a0;
      c.alpha[(int64_t)(e0 + lane) * 2 + 1] = a1;
      if (c.kvf) {
        c.alk[(int64_t)(e0 + lane) * 2] = t0;
        c.alk[(int64_t)(e0 + lane) * 2 + 1] = t1;
      }
    }
    if (c.kvf && lane < c.C) {
      float* qo = c.Qo + (int64_t)x * 2 * c.HC;
      qo[lane] = q0;
      qo[c.C + lane] = q1;
      qo[c.HC + lane] = o0;
      qo[c.HC + c.C + lane] = o1;
    }
  }
};
template <bool TRAIN, int EB = ATT_EB, class CK = NoCheckpoint>
__device__ __forceinline__ float2 attn_centre(const Ctx& c, int x, int i, int e0, int ne, int lane, int jrec = -1,
                                              AttnStores* st = nullptr, CK ck = CK{}) {
  const int C = c.C, HC = c.HC;
  const float on = f01(lane < C);
  const int l0 = min(lane, C - 1);
  const float* Pi = c.P + (int64_t)i * 4 * HC;
  const float q0 = Pi[l0], q1 = Pi[C + l0];
  const float sqc = sqrtf((float)C);
  const int jl = jrec >= 0 ? jrec : c.e_j[e0 + min(lane, max(ne - 1, 0))];   // lane e: the neighbour row of edge e
  const float sk0 = Pi[3 * HC + l0], sk1 = Pi[3 * HC + C + l0];
  // the attention-dropout key (centre node, lane's edge e_id) and seed, loaded with the first rows instead
  // of after the softmax
  uint64_t dseed = 0, dnode = 0, deid = 0;
  if (TRAIN) {
    dseed = (uint64_t)c.ctl[TGNX_CTL_SEED];
    dnode = (uint64_t)c.cent[x];
    deid = (uint64_t)c.e_id[e0 + min(lane, max(ne - 1, 0))];
  }
  float my0 = -INFINITY, my1 = -INFINITY;
  float o0 = 0.f, o1 = 0.f;
  float t0, t1;
  auto softmax = [&]() {
    const float mx0 = wave_max_f(my0), mx1 = wave_max_f(my1);
    const float ex0 = lane < ne ? expf(my0 - mx0) : 0.f, ex1 = lane < ne ? expf(my1 - mx1) : 0.f;
    const float a0 = ex0 / (wave_sum_f(ex0) + 1e-16f), a1 = ex1 / (wave_sum_f(ex1) + 1e-16f);
    t0 = a0;
    t1 = a1;
    if (TRAIN && lane < ne) {
      if (c.drop) {
        const uint32_t base = drop_base(dseed, (uint64_t)c.att_salt, dnode, deid);
        t0 *= keep32(base, 0u, c.p, c.inv_keep);
        t1 *= keep32(base, 1u, c.p, c.inv_keep);
      }
      if (st) {
        st->a0 = a0;
        st->a1 = a1;
        st->t0 = t0;
        st->t1 = t1;
      } else {
        c.alpha[(int64_t)(e0 + lane) * 2] = a0;
        c.alpha[(int64_t)(e0 + lane) * 2 + 1] = a1;
        if (c.kvf) {
          c.alk[(int64_t)(e0 + lane) * 2] = t0;
          c.alk[(int64_t)(e0 + lane) * 2 + 1] = t1;
        }
      }
    }
  };
  // kvf: the centre's q and aggregated message output (every root of the centre writes equal values)
  auto put_qo = [&]() {
    if (TRAIN && st) {
      st->q0 = q0;
      st->q1 = q1;
      st->o0 = o0;
      st->o1 = o1;
      st->x = x;
      st->e0 = e0;
      st->ne = ne;
      return;
    }
    if (TRAIN && c.kvf && lane < C) {
      float* qo = c.Qo + (int64_t)x * 2 * HC;
      qo[lane] = q0;
      qo[C + lane] = q1;
      qo[HC + lane] = o0;
      qo[HC + C + lane] = o1;
    }
  };
  if (ne > 0 && ne <= EB) {  // every ring of K <= 16: one load round
    float k0[EB], k1[EB], v0[EB], v1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = min(u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      const float ea = Ee[l0], eb = Ee[C + l0];
      k0[u] = Pj[HC + l0] + ea;
      k1[u] = Pj[HC + C + l0] + eb;
      v0[u] = Pj[2 * HC + l0] + ea;
      v1[u] = Pj[2 * HC + C + l0] + eb;
    }
    // (no early exit: a runtime `break` kept these loops rolled — indexed register reads, one edge's reduction
    // after another; the clamped rows of edges >= ne are reduced and discarded)
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const float p0 = wave_sum_f(q0 * k0[u] * on), p1 = wave_sum_f(q1 * k1[u] * on);
      if (lane == u && u < ne) { my0 = p0; my1 = p1; }
    }
    // the scale once per lane (lane e holds edge e's scores): the same quotients as per edge, one division
    // instead of one (a ~10-instruction dependent sequence) per edge and head
    if (lane < ne) { my0 /= sqc; my1 /= sqc; }
    softmax();
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // (t of lanes >= ne is 0: the clamped rows add exact zeros)
      o0 += v0[u] * lane_f(t0, u);
      o1 += v1[u] * lane_f(t1, u);
    }
    put_qo();
    return make_float2(o0 + sk0, o1 + sk1);
  }
  for (int b = 0; b < ne; b += EB) {
    float k0[EB], k1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // all loads of the batch in flight
      const int e = min(b + u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      k0[u] = Pj[HC + l0] + Ee[l0];
      k1[u] = Pj[HC + C + l0] + Ee[C + l0];
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const float p0 = wave_sum_f(q0 * k0[u] * on), p1 = wave_sum_f(q1 * k1[u] * on);
      if (lane == b + u && b + u < ne) { my0 = p0; my1 = p1; }
    }
  }
  if (lane < ne) { my0 /= sqc; my1 /= sqc; }
  softmax();
  for (int b = 0; b < ne; b += EB) {
    float v0[EB], v1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = min(b + u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      v0[u] = Pj[2 * HC + l0] + Ee[l0];
      v1[u] = Pj[2 * HC + C + l0] + Ee[C + l0];
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // (t of lanes >= ne is 0)
      o0 += v0[u] * lane_f(t0, b + u);
      o1 += v1[u] * lane_f(t1, b + u);
    }
  }
  put_qo();
  return make_float2(o0 + sk0, o1 + sk1);
}
// One root's 1-hop train attention in the paired-channel lane layout (tgn_pred_train<ATT>): lanes 0-31 carry head 0,
// lanes 32-63 head 1, lane (h, j) channels 2j and 2j + 1 of head h (j < C / 2): one float2 load per row part instead
// of two scalar ones, and one 32-lane reduction per edge scores both heads (two full-wave reductions per edge in
// attn_centre).  Edges [e0, e0 + ne), ne <= EB, neighbour rows from the per-root record (jrec, lane e).  Needs C even
// and C <= 64.  Returns this lane's two output channels (z[chan], z[chan + 1]; chan = -1 on an idle lane); the alpha /
// alk / Qo stores are left in *st (issued after the predictor's first barrier, as attn_centre's).
struct AttnStoresPair {
  float a0, a1, t0, t1;
  float2 q, o;
  int x, e0, ne, chan;
  __device__ void issue(const Ctx& c, int lane) const {
    if (lane < ne) {
      c.alpha[(int64_t)(e0 + lane) * 2] = a0;
      c.alpha[(int64_t)(e0 + lane) * 2 + 1] = a1;
      if (c.kvf) {
        c.alk[(int64_t)(e0 + lane) * 2] = t0;
        c.alk[(int64_t)(e0 + lane) * 2 + 1] = t1;
      }
    }
    if (c.kvf && chan >= 0) {
      float* qo = c.Qo + (int64_t)x * 2 * c.HC;
      *reinterpret_cast<float2*>(qo + chan) = q;
      *reinterpret_cast<float2*>(qo + c.HC + chan) = o;
    }
  }
};
template <int EB>
__device__ __forceinline__ float2 attn_root_pair(const Ctx& c, int x, int i, int e0, int ne, int lane, int jrec,
                                                 AttnStoresPair* st) {
  const int C = c.C, HC = c.HC, hc = C >> 1;
  const int h = lane >> 5, j = lane & 31;
  const bool act = j < hc;
  const int ch = h * C + 2 * (act ? j : hc - 1);  // (rows are 8-B aligned: HC even, ch even)
  const float on = f01(act);
  const float* Pi = c.P + (int64_t)i * 4 * HC;
  const float2 q = *reinterpret_cast<const float2*>(Pi + ch);
  const float2 sk = *reinterpret_cast<const float2*>(Pi + 3 * HC + ch);
  const float sqc = sqrtf((float)C);
  const uint64_t dseed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const uint64_t dnode = (uint64_t)c.cent[x];
  const uint64_t deid = (uint64_t)c.e_id[e0 + min(lane, max(ne - 1, 0))];
  float2 k[EB], v[EB];
#pragma unroll
  for (int u = 0; u < EB; ++u) {
    const int e = min(u, ne - 1);
    const float* Pj = c.P + (int64_t)lane_i(jrec, e) * 4 * HC;
    const float2 ee = *reinterpret_cast<const float2*>(c.Ep + (int64_t)(e0 + e) * HC + ch);
    const float2 kk = *reinterpret_cast<const float2*>(Pj + HC + ch);
    const float2 vv = *reinterpret_cast<const float2*>(Pj + 2 * HC + ch);
    k[u] = make_float2(kk.x + ee.x, kk.y + ee.y);
    v[u] = make_float2(vv.x + ee.x, vv.y + ee.y);
  }
  float my0 = -INFINITY, my1 = -INFINITY;
#pragma unroll
  for (int u = 0; u < EB; ++u) {
    const float pr = half_sum_f((q.x * k[u].x + q.y * k[u].y) * on);
    const float p0 = lane_f(pr, 0), p1 = lane_f(pr, 32);
    if (lane == u && u < ne) { my0 = p0; my1 = p1; }
  }
  if (lane < ne) { my0 /= sqc; my1 /= sqc; }
  const float mx0 = wave_max_f(my0), mx1 = wave_max_f(my1);
  const float ex0 = lane < ne ? expf(my0 - mx0) : 0.f, ex1 = lane < ne ? expf(my1 - mx1) : 0.f;
  const float a0 = ex0 / (wave_sum_f(ex0) + 1e-16f), a1 = ex1 / (wave_sum_f(ex1) + 1e-16f);
  float t0 = a0, t1 = a1;
  if (lane < ne && c.drop) {
    const uint32_t base = drop_base(dseed, (uint64_t)c.att_salt, dnode, deid);
    t0 *= keep32(base, 0u, c.p, c.inv_keep);
    t1 *= keep32(base, 1u, c.p, c.inv_keep);
  }
  float2 o = make_float2(0.f, 0.f);
#pragma unroll
  for (int u = 0; u < EB; ++u) {  // (t of lanes >= ne is 0: the clamped rows add exact zeros)
    const float tu = h ? lane_f(t1, u) : lane_f(t0, u);
    o.x += v[u].x * tu;
    o.y += v[u].y * tu;
  }
  st->a0 = a0;
  st->a1 = a1;
  st->t0 = t0;
  st->t1 = t1;
  st->q = q;
  st->o = o;
  st->x = x;
  st->e0 = e0;
  st->ne = ne;
  st->chan = act ? ch : -1;
  return make_float2(o.x + sk.x, o.y + sk.y);
}
template <bool TRAIN>
__global__ void __launch_bounds__(256) tgn_attn_fwd(Ctx c) {
  TGNX_STAMP(4);
  const int lane = threadIdx.x & 63;
  const int x = blockIdx.x * 4 + (threadIdx.x >> 6);
  // one round for the batch descriptor, the centre count and the centre's row / edge range: the centre
  // arrays hold ccap rows (ceoff ccap + 1), so the read is clamped, and discarded past the runtime count
  const int xc = min(x, max(c.ccap - 1, 0));
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int64_t err = c.ctl[TGNX_CTL_ERR];
  const int R = c.cnt[c.rsel];
  const int i = c.cent_loc[xc];
  const int e0 = c.ceoff[xc], e1 = c.ceoff[xc + 1];
  if (B == 0 || err != 0 || x >= R) return;
  const float2 o = attn_centre<TRAIN>(c, x, i, e0, e1 - e0, lane);
  if (lane < c.C) {
    c.Zc[(int64_t)x * c.HC + lane] = o.x;
    c.Zc[(int64_t)x * c.HC + c.C + lane] = o.y;
  }
}


// ------------------------------------------------------------------ link prediction (decoder.py:12-27)
// Workgroup per event of this rank's slice: h = relu(lin_src(z_s) + lin_dst(z_d)), s = sigmoid(lin_final(h)),
// loss = BCEWithLogits(s_pos, 1) + BCEWithLogits(s_neg, 0) (the reference feeds the sigmoid output to
// BCEWithLogitsLoss), backward rows, dz rows accumulated into the centres' dZc.
// evs row: zs | zp | zn | dhp | dhn | hp | hn (D each) | a_p a_n s_p s_n da_p da_n loss pad
__host__ __device__ inline int evs_stride(int D) { return 7 * D + 8; }
// Wave roles until the first barrier: wave 0 loads the roots' centre rows (written per event by
// tgn_agg_emit, in the ctl round) and their Zc rows; waves 1-3 stage lin_src / lin_dst (LDS, pitch D + 1:
// conflict-free rows and columns)
// and the bias / output-layer vectors.  vmcnt retires in issue order, so a chain load queued behind the
// 80 KB of weights in the same wave would wait for all of them; separate waves keep separate queues.
// (Read from global memory directly, the forward's W[o][k] with lanes over o touched 64 cache lines per
// load instruction.)
__host__ __device__ inline size_t tgn_pred_smem(int D) { return (size_t)2 * D * (D + 1) * sizeof(float); }
constexpr int PRED_SU = 16;  // float4 per staging thread per matrix per round (D <= 110: one round)
// nmk > 0 (pipelined resident step): the last nmk blocks mark the NEXT batch instead (mark_body, ahead 1):
// the ring insert of this batch ran beside the GRU, and nothing of this step reads what marking writes.
// ATT (1-hop train): the TransformerConv forward of the event's three roots runs here too — waves 1-3 one
// root each (attn_centre, its row / edge range from the per-root record tgn_agg_emit wrote), writing the
// embedding rows straight into LDS, while wave 0 stages the weights: no tgn_attn_fwd launch, and the
// attention chain overlaps the weight staging.  A centre shared by several roots is computed by each of
// them, identically (its alpha stores write equal values).
// kvf: the sampled edges sorted by neighbour row (counting sort in LDS, one workgroup riding in the predictor
// launch, off the step's critical path), so that the attention backward's edge blocks see long runs of equal
// neighbours and sum each run before one atomic (order within a row: LDS-atomic order).  Rows past the LDS
// (cap counters) cannot occur: the host takes this path only when every row fits (else ERR_SORT_CAP).
__device__ void edge_sort_body(const Ctx& c, int* cntr, int cap) {
  __shared__ int wsum[256];
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int E = level_edges(c), M = c.cnt[CNT_M];
  const int t = threadIdx.x;
  if (M + 1 > cap) {  // (the host enables the sort for Mtr + 1 <= cap only)
    if (t == 0) c.ctl[TGNX_CTL_ERR] |= ERR_SORT_CAP;
    return;
  }
  for (int m = t; m < M; m += 256) cntr[m] = 0;
  __syncthreads();
  for (int e = t; e < E; e += 256) atomicAdd(&cntr[c.e_j[e]], 1);
  __syncthreads();
  const int per = (M + 255) / 256, m0 = min(t * per, M), m1 = min(m0 + per, M);
  int sum = 0;
  for (int m = m0; m < m1; ++m) sum += cntr[m];
  wsum[t] = sum;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the per-thread sums
    const int v = t >= o ? wsum[t - o] : 0;
    __syncthreads();
    wsum[t] += v;
    __syncthreads();
  }
  int run = wsum[t] - sum;
  for (int m = m0; m < m1; ++m) {
    const int n = cntr[m];
    cntr[m] = run;
    run += n;
  }
  __syncthreads();
  for (int e = t; e < E; e += 256) {
    const int j = c.e_j[e], x = c.e_c[e];
    const int pos = atomicAdd(&cntr[j], 1);
    c.kj[pos] = j;
    c.kx[pos] = x;
    c.ke[pos] = e;
  }
}

// the NEXT batch's partitioned plans (data-parallel steps whose global batch's plans do not fit the dW_cell
// launch's LDS): plan workgroup `role` (0 .. 2 pplan) into the other parity set (po), batch one past the
// counters; up to 2 x 2048 keys at 256 threads (MAXE 16)
constexpr int PRED_PLAN_MAXE = 16;
__device__ __forceinline__ void pred_plan_body(const Ctx& c, int role, const PlanOut& po, unsigned char* smem) {
  __shared__ int sh[40];
  const ResDesc d = res_desc(c, 1);
  if (d.B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int P = c.pplan;
  plan_part<PRED_PLAN_MAXE>(c, role < P ? 0 : 1, role % P, P, d.B, d.start, smem, sh, NoCheckpoint{}, po);
}
// the split's plan table (tgnx_tgn_plan_table): workgroup (batch b, plan role) sorts batch b's ring-insert or
// message-store plan partition into slot b — the plans are a function of the event table alone, so the whole
// split's are built once per binding instead of by every step's scan
__global__ void __launch_bounds__(1024) tgn_plan_table_kernel(Ctx c, char* tab, int64_t stride, int64_t lo, int64_t hi,
                                                              int64_t batch) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm_[];
  __shared__ int sh[40];
  const int P = c.pplan, b = (int)(blockIdx.x / (2 * P)), role = (int)(blockIdx.x % (2 * P));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int64_t* h = reinterpret_cast<int64_t*>(tab);
    h[0] = lo; h[1] = hi; h[2] = batch; h[3] = c.Bplan; h[4] = P;
  }
  const int64_t start = lo + (int64_t)b * batch;
  const int B = (int)min(batch, hi - start);
  if (B <= 0) return;
  plan_part<8>(c, role < P ? 0 : 1, role % P, P, B, start, psm_, sh, NoCheckpoint{}, plan_slot(tab, stride, c.Bplan, b));
}
constexpr int ZH_MAX = 4;  // float4 columns per wave it holds (D <= 128 at 8 waves)
// waves per workgroup: 1 hop (ATT) 8 — waves 1-3 the roots' attention, waves 0 and 4-7 the weight staging, then
// all 8 share the contractions (the workgroup is alone on its CU: one wave per SIMD left each dependent step's
// latency exposed, measured 38 % of the waves' cycles issuing); 2 hops 4
#ifndef TGNX_DZC_REP
#define TGNX_DZC_REP 4  // 1-hop train: copies of dZc the predictor's workgroups spread their atomics over (a wiki batch's hub
                        // centre is the root of ~90 of its 600 root slots: its row's adds serialise at the memory side;
                        // the no-atomics diagnostic bounds that at 1.3 us).  The attention backward sums the copies with
                        // compile-time unrolled loads in the same round (tgn_attn_bwd<EB, REP>).  Same-box A/B
                        // (profiles/r5/r5_dzc_rep_ab.txt): predictor 12.7-12.9 -> 11.6 us, attention backward +0.5,
                        // step 0.0926 / 0.0928 -> 0.0922 / 0.0922 ms; 8 copies: attention backward +1.3, step 0.0932
#endif
#ifndef TGNX_PRED_WAVES
#define TGNX_PRED_WAVES 8  // 1-hop predictor workgroup waves (4: the round-4 layout, one staging wave)
#endif
#ifndef TGNX_PRED_WAVES2
#define TGNX_PRED_WAVES2 4  // 2-hop predictor workgroup waves: wave 0 loads the roots' embedding rows, the others stage
#endif                      // the weights, all share the contractions (8: 44.5 vs 42.5 us, r6e rocprof)
template <bool ATT>
constexpr int pred_waves() { return ATT ? TGNX_PRED_WAVES : TGNX_PRED_WAVES2; }
#ifndef TGNX_PRED2_STAGE
#define TGNX_PRED2_STAGE 1  // 2 hops: 1 stages lin_src / lin_dst in LDS once per workgroup and loops over events; 0 reads
#endif                      // them from L2, one event per workgroup (uncoalesced rows: comment step 0.2444 vs 0.2395 ms)
#ifndef TGNX_PRED2_WIDE_ATOM
#define TGNX_PRED2_WIDE_ATOM 0  // 2 hops: the dZc adds as whole rows through LDS (the 1-hop form, one more barrier); 0: each
#endif                          // wave adds its own outputs (the round-4 form; ±0, r6i_2hop_ab.txt)
// whether the predictor stages its weights in LDS (1 hop: the attention waves overlap the staging)
template <bool ATT>
constexpr bool pred_stages() { return ATT || TGNX_PRED2_STAGE; }
// EB: edges per attention load batch (attn_centre): 10 for rings of K <= 10 (the reference's sampling size), else 16
template <bool ATT, int EB = ATT_EB>
__global__ void __launch_bounds__(64 * pred_waves<ATT>()) tgn_pred_train(Ctx c, int nmk, int nsrt, PlanOut po, int npl) {
  constexpr int NW = pred_waves<ATT>();
  TGNX_STAMP(5);
  extern __shared__ __attribute__((aligned(16))) float Wl[];  // [2][D][DP]: lin_src, lin_dst
  __shared__ __attribute__((aligned(16))) float z[3][TDMAX];
  __shared__ float part[NW][3][TDMAX];
  __shared__ float dhw[NW][2][TDMAX];  // each wave's own copy of dh (no barrier between the epilogue and the backward)
  __shared__ float vsb[TDMAX], vdb[TDMAX], vfw[TDMAX + 1];  // lin_src.bias, lin_dst.bias, lin_final (w | b)
  __shared__ int scr[3];
  if ((int)blockIdx.x >= (int)gridDim.x - nmk - nsrt - npl) {  // riding jobs (mark: entries dealt to 256 threads;
                                                                // sort: 256 threads; plans: any block width)
    if ((int)blockIdx.x >= (int)gridDim.x - nmk) {  // (the dynamic LDS holds >= 3 x MARK_LDS_WORDS words)
      mark_body<true>(c, (int)blockIdx.x - ((int)gridDim.x - nmk), nmk, 1, reinterpret_cast<uint32_t*>(Wl));
    } else if ((int)blockIdx.x >= (int)gridDim.x - nmk - nsrt) {
      if (threadIdx.x >= 256) return;
      edge_sort_body(c, reinterpret_cast<int*>(Wl), (int)(tgn_pred_smem(c.D) / 4));
    } else {
      pred_plan_body(c, (int)blockIdx.x - ((int)gridDim.x - nmk - nsrt - npl), po, reinterpret_cast<unsigned char*>(Wl));
    }
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // D % 8 == 4 (D = 100): unpadded rows are conflict-free both for b128 row reads with lanes over rows
  // (start banks 4 D o mod 64 distinct over 16 lanes) and for b32 column reads, and the LDS image is the
  // global one (b128 stores); other D: pitch D + 1, element stores
  const int D = c.D;
  constexpr bool STW = pred_stages<ATT>();
  const bool flat = !STW || D % 8 == 4;
  const int DP = flat ? D : D + 1;
  // the weights: the LDS image (STW), else the parameter rows in global memory (L2-resident, read by every workgroup)
  float* Wsrc = STW ? Wl : c.params + c.L.lsw;
  float* Wdst = STW ? Wl + D * DP : c.params + c.L.ldw;
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const int64_t err = c.ctl[TGNX_CTL_ERR];
  constexpr int NST = ATT ? (NW - 3) * 64 : (NW - 1) * 64;  // staging threads: ATT waves 0, 4 .. NW-1; else 1 .. NW-1
  // a workgroup takes events slot, slot + G, ... (G = the event workgroups, at most one per CU: the weights are
  // staged once per workgroup, and its LDS leaves room for one workgroup per CU, so a batch of more events than
  // CUs ran in dispatch rounds of a whole workgroup each; pred_groups)
  const int G = (int)gridDim.x - nmk - nsrt - npl;
  for (int slot = blockIdx.x;; slot += G) {
  const bool first = slot == (int)blockIdx.x;
  const int i = lo + slot;
  const bool live = !(B == 0 || i >= hi || err != 0);
  // (out_ev: the batch's first event, loaded with the first round — a load after the evs-row stores would wait
  // for all of them, vmcnt retiring in order)
  const int64_t bstart = c.out_ev ? c.ctl[TGNX_CTL_BATCH_START] : 0;
  AttnStores ast;  // ATT, waves 1-3: the attention's alpha / alk / Qo stores, issued after the first barrier
  ast.ne = 0;
  ast.x = -1;
  AttnStoresPair asp;  // (the paired-channel form's)
  asp.x = -1;
  if (ATT && wv >= 1 && wv <= 3) {
    const int r = wv - 1;
    const int4 q = c.evq[3 * slot + r];  // {centre row, P row, edge range}; slot < max_batch: in bounds
    const int jr = c.evj ? c.evj[(3 * slot + r) * 16 + (lane & 15)] : -1;  // the edges' neighbour rows
    if (!live) return;
    bool paired = false;
    if (c.evj && q.w - q.z <= EB && (c.C & 1) == 0 && c.C <= 64) {
      paired = true;
      const float2 o = attn_root_pair<EB>(c, q.x, q.y, q.z, q.w - q.z, lane, max(jr, 0), &asp);
      if (asp.chan >= 0) {
        z[r][asp.chan] = o.x;
        z[r][asp.chan + 1] = o.y;
        if (c.emb) {  // DyRep embedding messages read the centre's embedding (every root of it writes equal values)
          c.Zc[(int64_t)q.x * c.HC + asp.chan] = o.x;
          c.Zc[(int64_t)q.x * c.HC + asp.chan + 1] = o.y;
        }
      }
      if (lane == 0) scr[r] = q.x;
    }
    if (!paired) {
      const float2 o = attn_centre<true, EB>(c, q.x, q.y, q.z, q.w - q.z, lane, c.evj && q.w - q.z <= 16 ? max(jr, 0) : -1,
                                             &ast);
      if (lane < c.C) {
        z[r][lane] = o.x;
        z[r][c.C + lane] = o.y;
        if (c.emb) {  // DyRep embedding messages read the centre's embedding (every root of it writes equal values)
          c.Zc[(int64_t)q.x * c.HC + lane] = o.x;
          c.Zc[(int64_t)q.x * c.HC + c.C + lane] = o.y;
        }
      }
      if (lane == 0) scr[r] = q.x;
    }
  } else if (!ATT && wv == 0) {
    int cr[3];  // the roots' centre rows (tgn_agg_emit) by rank-local event: issued with the ctl loads
#pragma unroll
    for (int r = 0; r < 3; ++r) cr[r] = c.evr[3 * slot + r];  // slot < max_batch: in bounds
    if (!live) return;
    for (int x = lane; x < 3 * D; x += 64) z[x / D][x % D] = c.Zc[(int64_t)cr[x / D] * D + x % D];
    if (lane < 3) scr[lane] = cr[lane];
  } else {
    const int sw = ATT ? (wv == 0 ? 0 : wv - 3) : wv - 1;  // staging wave index
    const int st = sw * 64 + lane;                        // staging thread index in [0, NST)
    if (blockIdx.x == 0 && st == 0 && first) {
      c.cnt[CNT_LIST] = 3 * (hi - lo);
      {  // this step's Adam scalars for the gradient writers (fused) or tgn_adam (the separate pass after the step)
        const int64_t t = c.ctl[TGNX_CTL_ADAM_T] + (c.adv ? 1 : 0);
        float* sc = reinterpret_cast<float*>(c.ctl + TGNX_CTL_ADAM_SC);
        sc[0] = (float)(c.lr / (1.0 - pow((double)c.b1, (double)t)));
        sc[1] = (float)sqrt(1.0 - pow((double)c.b2, (double)t));
      }
    }
    if (!live) return;
    if (!STW) {  // the biases and the output layer only
      for (int x = st; x < 3 * D + 1; x += NST) {
        const float v = x < D ? c.params[c.L.lsb + x] : x < 2 * D ? c.params[c.L.ldb + x - D]
                      : x < 3 * D ? c.params[c.L.lfw + x - 2 * D] : c.params[c.L.lfb];
        if (x < D) vsb[x] = v;
        else if (x < 2 * D) vdb[x - D] = v;
        else vfw[x - 2 * D] = v;
      }
    }
    // D is even, so D * D % 4 == 0; the flat buffer's blocks are 16-B aligned (tgnx_tgn_param_layout)
    if (STW && first) {  // (later events of the workgroup: the weights are in LDS already)
    const int n4 = D * D / 4;
    const float invD = 1.0f / (float)D;
    const float4* S4 = reinterpret_cast<const float4*>(c.params + c.L.lsw);
    const float4* D4 = reinterpret_cast<const float4*>(c.params + c.L.ldw);
    bool staged = false;
    if (flat && !staged) {  // the LDS image is the global one: global_load_lds_dwordx4 straight into it, no
                                   // registers, every row in flight at once (the waves drain them before the barrier)
      for (int x0 = 0; x0 < n4; x0 += NST) {
        const int x = x0 + st;
        if (x < n4) {  // (a wave's 64 lanes land at consecutive 16-B slots from its base x0 + 64 sw)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S4 + x),
                                           (__attribute__((address_space(3))) void*)(reinterpret_cast<float4*>(Wsrc) + x0 + 64 * sw),
                                           16, 0, 0);
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(D4 + x),
                                           (__attribute__((address_space(3))) void*)(reinterpret_cast<float4*>(Wdst) + x0 + 64 * sw),
                                           16, 0, 0);
        }
      }
      for (int x = st; x < 3 * D + 1; x += NST) {
        const float v = x < D ? c.params[c.L.lsb + x] : x < 2 * D ? c.params[c.L.ldb + x - D]
                      : x < 3 * D ? c.params[c.L.lfw + x - 2 * D] : c.params[c.L.lfb];
        if (x < D) vsb[x] = v;
        else if (x < 2 * D) vdb[x - D] = v;
        else vfw[x - 2 * D] = v;
      }
      // (the barrier below waits for LDS only).  The builtin, not inline asm: the compiler then knows the LDS-DMA
      // has landed, else it keeps it pending past the join with the attention waves and puts a vmcnt(0) before the
      // next LDS read — which waits on the attention's deferred global stores too
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15 = no wait)
      staged = true;
    }
    for (int b0 = 0; b0 < n4 && !staged; b0 += NST * PRED_SU) {
      float4 ws4[PRED_SU], wd4[PRED_SU];
#pragma unroll
      for (int u = 0; u < PRED_SU; ++u) {
        const int x = min(b0 + st + NST * u, n4 - 1);
        ws4[u] = S4[x];
        wd4[u] = D4[x];
      }
      if (b0 == 0)
        for (int x = st; x < 3 * D + 1; x += NST) {
          const float v = x < D ? c.params[c.L.lsb + x] : x < 2 * D ? c.params[c.L.ldb + x - D]
                        : x < 3 * D ? c.params[c.L.lfw + x - 2 * D] : c.params[c.L.lfb];
          if (x < D) vsb[x] = v;
          else if (x < 2 * D) vdb[x - D] = v;
          else vfw[x - 2 * D] = v;
        }
      if (flat) {
#pragma unroll
        for (int u = 0; u < PRED_SU; ++u) {
          const int x = b0 + st + NST * u;
          if (x < n4) {
            reinterpret_cast<float4*>(Wsrc)[x] = ws4[u];
            reinterpret_cast<float4*>(Wdst)[x] = wd4[u];
          }
        }
        continue;
      }
#pragma unroll
      for (int u = 0; u < PRED_SU; ++u) {
        const int x = b0 + st + NST * u;
        if (x < n4) {
          const float vs[4] = {ws4[u].x, ws4[u].y, ws4[u].z, ws4[u].w};
          const float vd[4] = {wd4[u].x, wd4[u].y, wd4[u].z, wd4[u].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {  // row / column of element 4x + j (no integer division: it is a
                                         // ~40-instruction software routine per element)
            const int e = 4 * x + j, o = div_small(e, D, invD), k = e - o * D;
            Wsrc[o * DP + k] = vs[j];
            Wdst[o * DP + k] = vd[j];
          }
        }
      }
    }
    }  // first
  }
  // LDS-only barriers in this kernel (the weights, embedding rows and partial sums are LDS; the attention's
  // alpha stores and the evs rows need not have landed): __syncthreads would wait for vmcnt(0)
  // (every wave's loads are consumed here and no store is in flight yet: a free wait that leaves the compiler's
  // scoreboard empty at the join, so the deferred stores below are not waited for at the next barrier)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (ATT && ast.x >= 0) ast.issue(c, lane);
  if (ATT && asp.x >= 0) asp.issue(c, lane);
  const int cr[3] = {scr[0], scr[1], scr[2]};
  // lin_src(z_s), lin_dst(z_p), lin_dst(z_n), split over the hidden units' inputs k: NW partial sums per output
  if (flat) {  // wave wv takes float4 columns [q0, q0 + nq)
    const int c4 = D / 4, kq = (c4 + NW - 1) / NW, q0 = wv * kq, nq = max(0, min(c4 - q0, kq));
    const float4* z0 = reinterpret_cast<const float4*>(z[0]) + q0;
    const float4* z1 = reinterpret_cast<const float4*>(z[1]) + q0;
    const float4* z2 = reinterpret_cast<const float4*>(z[2]) + q0;
    // the three embedding slices (wave-uniform) read once into registers for both output rounds: the LDS
    // reads were 3 broadcast b128 per 2 weight b128, twice
    if (NW == 8 && kq <= ZH_MAX) {
      float4 x0[ZH_MAX], x1[ZH_MAX], x2[ZH_MAX];
#pragma unroll
      for (int j = 0; j < ZH_MAX; ++j) {
        const bool in = j < nq;
        x0[j] = in ? z0[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        x1[j] = in ? z1[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        x2[j] = in ? z2[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int o = lane + 64 * q;
        if (o < D) {
          const float4* ws = reinterpret_cast<const float4*>(Wsrc + o * D) + q0;
          const float4* wd = reinterpret_cast<const float4*>(Wdst + o * D) + q0;
          float a = 0.f, b = 0.f, d2 = 0.f;
#pragma unroll
          for (int j = 0; j < ZH_MAX; ++j) {
            if (j < nq) {
              const float4 u = ws[j], v = wd[j];
              a += (u.x * x0[j].x + u.y * x0[j].y) + (u.z * x0[j].z + u.w * x0[j].w);
              b += (v.x * x1[j].x + v.y * x1[j].y) + (v.z * x1[j].z + v.w * x1[j].w);
              d2 += (v.x * x2[j].x + v.y * x2[j].y) + (v.z * x2[j].z + v.w * x2[j].w);
            }
          }
          part[wv][0][o] = a;
          part[wv][1][o] = b;
          part[wv][2][o] = d2;
        }
      }
    } else
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      if (o < D) {
        const float4* ws = reinterpret_cast<const float4*>(Wsrc + o * D) + q0;
        const float4* wd = reinterpret_cast<const float4*>(Wdst + o * D) + q0;
        float a = 0.f, b = 0.f, d2 = 0.f;
#pragma unroll 4
        for (int j = 0; j < nq; ++j) {
          const float4 u = ws[j], v = wd[j], x0 = z0[j], x1 = z1[j], x2 = z2[j];
          a += (u.x * x0.x + u.y * x0.y) + (u.z * x0.z + u.w * x0.w);
          b += (v.x * x1.x + v.y * x1.y) + (v.z * x1.z + v.w * x1.w);
          d2 += (v.x * x2.x + v.y * x2.y) + (v.z * x2.z + v.w * x2.w);
        }
        part[wv][0][o] = a;
        part[wv][1][o] = b;
        part[wv][2][o] = d2;
      }
    }
  } else {
    const int kc = (D + NW - 1) / NW, k0 = wv * kc, nk = max(0, min(D - k0, kc));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      if (o < D) {
        float a = 0.f, b = 0.f, d2 = 0.f;
        for (int k = 0; k < nk; ++k) {
          const float ws = Wsrc[o * DP + k0 + k], wd = Wdst[o * DP + k0 + k];
          a += ws * z[0][k0 + k];
          b += wd * z[1][k0 + k];
          d2 += wd * z[2][k0 + k];
        }
        part[wv][0][o] = a;
        part[wv][1][o] = b;
        part[wv][2][o] = d2;
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  TGNX_STAMP_AT(0);
  float* ev = c.evs + (int64_t)i * evs_stride(D);
  // every wave runs the forward epilogue (the same values in each: no dh round through a barrier) and keeps its own
  // copy of dh; wave 0 stores the event's row, outputs and loss term (they drain during the backward)
  float hp[2], hn[2], dhp[2], dhn[2];
  float ap, an, sp, sn, dap, dan;
  const float invB = 1.0f / (float)B;
  {
    auto psum = [&](int r, int o) {
      float s = 0.f;
      if (NW == 8)
        s = ((part[0][r][o] + part[1][r][o]) + (part[2][r][o] + part[3][r][o])) +
            ((part[4][r][o] + part[5][r][o]) + (part[6][r][o] + part[7][r][o]));
      else
        s = (part[0][r][o] + part[1][r][o]) + (part[2][r][o] + part[3][r][o]);
      return s;
    };
    float zp = 0.f, zn = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      hp[q] = hn[q] = 0.f;
      if (o < D) {
        const float s = psum(0, o) + vsb[o];
        const float dp = psum(1, o) + vdb[o];
        const float dn = psum(2, o) + vdb[o];
        hp[q] = fmaxf(s + dp, 0.f);
        hn[q] = fmaxf(s + dn, 0.f);
        zp += vfw[o] * hp[q];
        zn += vfw[o] * hn[q];
      }
    }
    ap = wave_sum_f(zp) + vfw[D];
    an = wave_sum_f(zn) + vfw[D];
    sp = sigm(ap);
    sn = sigm(an);
    dap = (sigm(sp) - 1.0f) * sp * (1.0f - sp) * invB;
    dan = sigm(sn) * sn * (1.0f - sn) * invB;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      const float wf = o < D ? vfw[o] : 0.f;
      dhp[q] = hp[q] > 0.f ? dap * wf : 0.f;
      dhn[q] = hn[q] > 0.f ? dan * wf : 0.f;
      if (o < D) {
        dhw[wv][0][o] = dhp[q];
        dhw[wv][1][o] = dhn[q];
      }
    }
  }
  if (wv == 0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = lane + 64 * q;
      if (o < D) {
        ev[o] = z[0][o];
        ev[D + o] = z[1][o];
        ev[2 * D + o] = z[2][o];
        ev[3 * D + o] = dhp[q];
        ev[4 * D + o] = dhn[q];
        ev[5 * D + o] = hp[q];
        ev[6 * D + o] = hn[q];
      }
    }
    if (lane == 0) {
      float* s = ev + 7 * D;
      s[0] = ap; s[1] = an; s[2] = sp; s[3] = sn; s[4] = dap; s[5] = dan;
      s[6] = (softplus_unit(-sp) + softplus_unit(sn)) * invB;
      c.out_pos[i] = sp;
      c.out_neg[i] = sn;
      if (c.out_ev) {
        const int64_t e = bstart + i;
        c.out_ev[2 * e] = sp;
        c.out_ev[2 * e + 1] = sn;
      }
    }
  }
  TGNX_STAMP_AT(1);
  {
    // dz_s = Wsrcᵀ (dhp + dhn), dz_p = Wdstᵀ dhp, dz_n = Wdstᵀ dhn for the outputs [wv ow, wv ow + ow) of this
    // wave: lanes = KG groups of the hidden units x OL outputs, dh from this wave's own LDS copy, the groups summed
    // across lanes, then the wave's dZc atomics
    constexpr int OL = NW == 8 ? 16 : 32, KG = 64 / OL;
    const int ow = (D + NW - 1) / NW, ol = lane % OL, kg = lane / OL, o = wv * ow + ol, hw = (D + KG - 1) / KG;
    const bool oko = ol < ow && o < D;  // (ow <= OL: D <= 128)
    const int oc = oko ? o : 0, kb = kg * hw;
    float a = 0.f, b = 0.f, d2 = 0.f;
#pragma unroll 5
    for (int j = 0; j < hw; ++j) {
      const int kk = min(kb + j, D - 1);
      const float live_k = f01(kb + j < D);
      const float h0 = dhw[wv][0][kk] * live_k, h1 = dhw[wv][1][kk] * live_k;
      const float w1 = Wsrc[kk * DP + oc], w2 = Wdst[kk * DP + oc];
      a += w1 * (h0 + h1);
      b += w2 * h0;
      d2 += w2 * h1;
    }
    if (KG == 4) {
      a = swap16_sum(a);
      b = swap16_sum(b);
      d2 = swap16_sum(d2);
    }
    a = swap32_sum(a);
    b = swap32_sum(b);
    d2 = swap32_sum(d2);
    float* dz = c.dZc + (int64_t)(slot % c.dzrep) * c.dzstride;
    if (!ATT && !TGNX_PRED2_WIDE_ATOM) {
      if (kg == 0 && oko) {
        atomicAdd(&dz[(int64_t)cr[0] * D + o], a);
        atomicAdd(&dz[(int64_t)cr[1] * D + o], b);
        atomicAdd(&dz[(int64_t)cr[2] * D + o], d2);
      }
    } else {
    // the three rows gathered in LDS first, then added with whole-row wave instructions (contiguous lanes: 6 per
    // workgroup instead of 3 per wave on 13-lane segments — every one of them queues on a hub centre's row)
    __shared__ float dzl[3][TDMAX];
    if (kg == 0 && oko) {
      dzl[0][o] = a;
      dzl[1][o] = b;
      dzl[2][o] = d2;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int x = tid; x < 3 * D; x += 64 * NW) {
      const int r = x >= 2 * D ? 2 : x >= D ? 1 : 0, oo = x - r * D;
      atomicAdd(&dz[(int64_t)cr[r] * D + oo], dzl[r][oo]);
    }
    }
  }
  if (ATT || lo + slot + G >= hi) break;  // (ATT: one event per workgroup — the loop's live ranges spilled the
                                           // 8-wave kernel: 168 -> 256 VGPRs + 47 spilled, predictor 12 -> 20 us)
  // (the next event's rows overwrite z, scr and the partial sums: every wave past this event's last LDS read)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  }  // slot
}

// predictor bias / output-layer / loss reductions over this rank's events (wave per output)
__device__ void lp_vec_body(const Ctx& c, int y, int lane) {
  const int D = c.D;
  if (y >= 3 * D + 2) return;
  const int lo = (int)c.ctl[TGNX_CTL_LO], hi = (int)c.ctl[TGNX_CTL_HI];
  const bool ok = c.ctl[TGNX_CTL_B] > 0 && c.ctl[TGNX_CTL_ERR] == 0;
  const int S = evs_stride(D);
  float s = 0.f;
  for (int i = lo + lane; i < hi && ok; i += 64) {
    const float* ev = c.evs + (int64_t)i * S;
    if (y < 2 * D) s += ev[3 * D + (y % D)] + ev[4 * D + (y % D)];
    else if (y < 3 * D) s += ev[7 * D + 4] * ev[5 * D + (y - 2 * D)] + ev[7 * D + 5] * ev[6 * D + (y - 2 * D)];
    else if (y == 3 * D) s += ev[7 * D + 4] + ev[7 * D + 5];
    else s += ev[7 * D + 6];
  }
  s = wave_sum_f(s);
  if (lane == 0) {
    float* g = c.grads;
    if (y < D) c.adf.put(g, c.L.lsb + y, s);
    else if (y < 2 * D) c.adf.put(g, c.L.ldb + y - D, s);
    else if (y < 3 * D) c.adf.put(g, c.L.lfw + y - 2 * D, s);
    else if (y == 3 * D) c.adf.put(g, c.L.lfb, s);
    else {
      g[c.L.total] = s;  // batch loss slot
      if (c.adf.p && ok)  // fused step: the running loss sum tgn_adam keeps otherwise
        *reinterpret_cast<double*>(c.ctl + TGNX_CTL_LOSS) += (double)s * (double)c.ctl[TGNX_CTL_B];
    }
  }
}

// Attention backward, edge half (kvf: 1-hop train step, the middle blocks of tgn_attn_bwd).  The centre's
// output gradient g = dZc[x] enters linearly: with t = alpha * keep (alk) and the centre's aggregated message
// output o = Σ_e t_e v_e (Qo, written by the forward), Σ_e alpha_e dalpha_e = g · o per head, so
//   ds_e = t_e (g · v_e) - alpha_e (g · o),  dk_e = ds_e q / sqrt(C),  dv_e = t_e g,  dE_e = dk_e + dv_e
// need no other edge of the centre: each edge's (dk, dv) is computed where it is summed into its neighbour's
// dP row (no per-edge dKV round trip, no separate k / v reduction launch), while the centre blocks compute dq.
// Workgroup per chunk of KVE_CH consecutive edges sorted by neighbour in LDS (as kv_reduce_body); a wave takes
// KVE_PW sorted edges, lanes over the channels of both heads, and sums runs of equal neighbours in registers.
#ifndef TGNX_KVE_CH
#define TGNX_KVE_CH 16  // 32 -> 16 (round 6, same box): wiki 0.0846 -> 0.0832 ms, coin-shaped 0.0899 / 0.0906 -> 0.0878 /
                        // 0.0888, review-shaped 0.0996 / 0.1002 -> 0.0990 / 0.0995; 8: 0.0836, 64: 0.0902 (profiles/r6/r6av_*, r6aw_*)
#endif
constexpr int KVE_CH = TGNX_KVE_CH, KVE_PW = KVE_CH / 4;
#ifndef TGNX_KVE_B
#define TGNX_KVE_B 8
#endif
constexpr int KVE_B = TGNX_KVE_B < KVE_PW ? TGNX_KVE_B : KVE_PW;  // edges per load batch of a wave
// (lane l carries channel l of both heads; the paired-channel layout of attn_root_pair measured slower here:
// attention backward 12.0 -> 12.2-12.5 us)
template <int REP = 1>
__device__ void kv_edge_body(const Ctx& c, int bid) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int E = level_edges(c);
  const int eb = bid * KVE_CH;
  const int t = threadIdx.x;
  const bool gs = c.kvs;  // workgroup-uniform
  // globally sorted edges: the chunk's records (and the keys just outside it) loaded in the edge count's round,
  // clamped to the sorted arrays' rows (ktr) and masked by the count after
  int kj0 = 0, kx0 = 0, ke0 = 0, kb = -1;
  if (gs) {
    if (t < KVE_CH) {
      const int ec = min(eb + t, c.ktr - 1);
      kj0 = c.kj[ec];
      kx0 = c.kx[ec];
      ke0 = c.ke[ec];
    } else if (t == KVE_CH) {
      kb = eb > 0 ? c.kj[min(eb - 1, c.ktr - 1)] : -1;
    } else if (t == KVE_CH + 1) {
      kb = c.kj[min(eb + KVE_CH, c.ktr - 1)];
    }
  }
  if (eb >= E) return;  // whole workgroup
  const int ne = min(KVE_CH, E - eb);
  __shared__ int sj[KVE_CH], sx[KVE_CH], se[KVE_CH], sorder[KVE_CH], sb[2];
  // globally sorted: a run whose row has no edge in the neighbouring chunks is the row's whole sum (a plain
  // store); the chunk's first / last runs may continue there (the keys just outside the chunk tell)
  if (gs) {
    if (t == KVE_CH) sb[0] = kb;
    if (t == KVE_CH + 1) sb[1] = eb + ne < E ? kb : -1;  // (ne < KVE_CH: eb + ne = E)
    if (t < KVE_CH) {
      sj[t] = t < ne ? kj0 : INT_MAX;
      sx[t] = kx0;
      se[t] = ke0;
    }
  } else if (t < KVE_CH) {
    const int ec = min(eb + t, E - 1);
    sj[t] = t < ne ? c.e_j[ec] : INT_MAX;
    sx[t] = c.e_c[ec];
    se[t] = ec;
  }
  __syncthreads();
  if (t < ne) {  // stable rank of (neighbour, edge)
    const int key = sj[t];
    int r = 0;
#pragma unroll 16
    for (int u = 0; u < KVE_CH; ++u) {
      const int ju = sj[u];
      r += (ju < key) || (ju == key && u < t);
    }
    sorder[r] = t;
  }
  __syncthreads();
  const int w = t >> 6, lane = t & 63;
  const int i0 = w * KVE_PW;
  // a wave's first and last runs may continue in the neighbouring waves: they go to LDS pieces (slots 2w, 2w + 1,
  // key -1 = none), merged in wave order by wave 0 before their atomics
  __shared__ float ps[8][4][64];
  __shared__ int pk[8];
  if (i0 >= ne) {
    if (lane == 0) pk[2 * w] = pk[2 * w + 1] = -1;
  }
  const int n = max(0, min(KVE_PW, ne - i0));
  const int C = c.C, HC = c.HC;
  // this lane's two channels (oA, oB within HC; clamped for loads) and head of each
  const bool okl = lane < C;
  const float on = f01(okl);
  const int l0 = min(lane, C - 1);
  const int oA = l0, oB = C + l0;
  constexpr int hA = 0, hB = 1;
  const float isq = 1.0f / sqrtf((float)C);
  float s[4] = {0.f, 0.f, 0.f, 0.f};  // run sums: dk (head 0, 1), dv (head 0, 1)
  int jc = n > 0 ? sj[sorder[i0]] : -1;
  bool first = true;  // the open run is the wave's first
  auto flush = [&]() {
    if (okl) {
      float* dst = c.dP + (int64_t)jc * 4 * HC + HC;
      atomicAdd(dst + oA, s[0]);
      atomicAdd(dst + oB, s[1]);
      atomicAdd(dst + HC + oA, s[2]);
      atomicAdd(dst + HC + oB, s[3]);
    }
  };
  auto store = [&]() {  // the row's complete (dk, dv) sums (globally sorted edges)
    if (okl) {
      float* dst = c.dP + (int64_t)jc * 4 * HC + HC;
      dst[oA] = s[0];
      dst[oB] = s[1];
      dst[HC + oA] = s[2];
      dst[HC + oB] = s[3];
    }
  };
  // the wave's sorted edges in batches of KVE_B (all of a batch's loads in flight), runs continuing across
  for (int b0 = 0; b0 < n; b0 += KVE_B) {
    const int nb = min(KVE_B, n - b0);
    int jj[KVE_B], er[KVE_B], xx[KVE_B];
#pragma unroll
    for (int u = 0; u < KVE_B; ++u) {
      const int e = sorder[i0 + b0 + min(u, nb - 1)];
      jj[u] = sj[e];
      xx[u] = sx[e];
      er[u] = se[e];
    }
    float a0[KVE_B], a1[KVE_B], t0[KVE_B], t1[KVE_B];
    float g0[KVE_B], g1[KVE_B], q0[KVE_B], q1[KVE_B], o0[KVE_B], o1[KVE_B], v0[KVE_B], v1[KVE_B];
#pragma unroll
    for (int u = 0; u < KVE_B; ++u) {  // softmax weights, centre rows (g, q, o), the neighbour's v row + edge row
      a0[u] = c.alpha[(int64_t)er[u] * 2 + hA];
      a1[u] = c.alpha[(int64_t)er[u] * 2 + hB];
      t0[u] = c.alk[(int64_t)er[u] * 2 + hA];
      t1[u] = c.alk[(int64_t)er[u] * 2 + hB];
      const float* G = c.dZc + (int64_t)xx[u] * HC;
      const float* Q = c.Qo + (int64_t)xx[u] * 2 * HC;
      const float* Pj = c.P + (int64_t)jj[u] * 4 * HC + 2 * HC;
      const float* Ee = c.Ep + (int64_t)er[u] * HC;
      g0[u] = G[oA];
      g1[u] = G[oB];
#pragma unroll
      for (int rp = 1; rp < REP; ++rp) {  // (the predictor's dZc copies, in copy order; REP = c.dzrep, compile-time
                                          // so that every copy's load is in the batch's one round)
        g0[u] += G[rp * c.dzstride + oA];
        g1[u] += G[rp * c.dzstride + oB];
      }
      q0[u] = Q[oA];
      q1[u] = Q[oB];
      o0[u] = Q[HC + oA];
      o1[u] = Q[HC + oB];
      v0[u] = Pj[oA] + Ee[oA];
      v1[u] = Pj[oB] + Ee[oB];
    }
    // the batch's reductions first, all independent (a runtime `break` in one loop kept it rolled: indexed register
    // reads and one edge's four reductions after another's), then the run bookkeeping
    float gv0[KVE_B], gv1[KVE_B], go0[KVE_B], go1[KVE_B];
#pragma unroll
    for (int u = 0; u < KVE_B; ++u) {
      gv0[u] = wave_sum_f(g0[u] * v0[u] * on);
      gv1[u] = wave_sum_f(g1[u] * v1[u] * on);
      go0[u] = wave_sum_f(g0[u] * o0[u] * on);
      go1[u] = wave_sum_f(g1[u] * o1[u] * on);
    }
#pragma unroll
    for (int u = 0; u < KVE_B; ++u) {
      if (u >= nb) continue;
      if (jj[u] != jc) {  // wave-uniform run boundary
        if (first) {
          for (int q = 0; q < 4; ++q) ps[2 * w][q][lane] = s[q];
          if (lane == 0) pk[2 * w] = jc;
          first = false;
        } else {
          if (gs) store();
          else flush();
        }
        s[0] = s[1] = s[2] = s[3] = 0.f;
        jc = jj[u];
      }
      const float ds0 = (t0[u] * gv0[u] - a0[u] * go0[u]) * isq, ds1 = (t1[u] * gv1[u] - a1[u] * go1[u]) * isq;
      const float dk0 = ds0 * q0[u], dk1 = ds1 * q1[u];
      const float dv0 = t0[u] * g0[u], dv1 = t1[u] * g1[u];
      if (okl) {
        float* dEe = c.dE + (int64_t)er[u] * HC;
        dEe[oA] = dk0 + dv0;
        dEe[oB] = dk1 + dv1;
      }
      s[0] += dk0;
      s[1] += dk1;
      s[2] += dv0;
      s[3] += dv1;
    }
  }
  if (n > 0) {  // the open run: the wave's only (slot 2w) or its last (slot 2w + 1)
    const int sl = first ? 2 * w : 2 * w + 1;
    for (int q = 0; q < 4; ++q) ps[sl][q][lane] = s[q];
    if (lane == 0) {
      pk[sl] = jc;
      if (first) pk[2 * w + 1] = -1;
    }
  }
  __syncthreads();
  if (w != 0) return;
  jc = -1;
  bool firstg = true;  // the open group holds the chunk's first edge
  const int kprev = gs ? sb[0] : -2, knext = gs ? sb[1] : -2;
  for (int sl = 0; sl < 8; ++sl) {
    const int key = pk[sl];
    if (key < 0) continue;
    if (key != jc) {
      if (jc >= 0) {
        if (gs && !(firstg && jc == kprev)) store();
        else flush();
        firstg = false;
      }
      jc = key;
      s[0] = s[1] = s[2] = s[3] = 0.f;
    }
    for (int q = 0; q < 4; ++q) s[q] += ps[sl][q][lane];
  }
  if (jc >= 0) {
    if (gs && !(firstg && jc == kprev) && jc != knext) store();
    else flush();
  }
}

// Backward of tgn_attn_fwd (wave per centre) ‖ [nkv > 0: kv_edge_body blocks; the centre waves then write
// dq and the skip gradient only] ‖ trailing blocks: lp_vec_body.
// dk / dv of an edge belong to its neighbour's row of dP.  They are stored per edge (dKV, plain
// coalesced stores) and summed into dP by tgn_kv_reduce: a hub neighbour is shared by most centres (a
// wiki-shaped hub user sits in ~40 % of the page rings), and per-edge global atomics on its row
// serialised at the L2 (attn_bwd 36 us, 15 us without them).
// nwalk (1-hop parity-set steps with a plan table): the last block walks the NEXT batch's node sets
// into the other parity's set (cw; the plans come from the table), instead of a workgroup of the dW_cell launch
template <int EB, int REP = 1>
__global__ void __launch_bounds__(256) tgn_attn_bwd(Ctx c, int ncb, int nkv, int nwalk, Ctx cw) {
  TGNX_STAMP(6);
  if ((int)blockIdx.x >= (int)gridDim.x - nwalk) {
    extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
    scan_body<true, NoCheckpoint, 512>(cw, 0, wsm, NoCheckpoint{}, 1, false);
    return;
  }
  if ((int)blockIdx.x >= ncb + nkv) {
    lp_vec_body(c, ((int)blockIdx.x - ncb - nkv) * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
    return;
  }
  if ((int)blockIdx.x >= ncb) {
    kv_edge_body<REP>(c, (int)blockIdx.x - ncb);
    return;
  }
  const bool wkv = nkv == 0;  // per-edge dk / dv / dE written here (else by the edge blocks)
  const int lane = threadIdx.x & 63;
  const int x = blockIdx.x * 4 + (threadIdx.x >> 6);
  // first round: batch descriptor, centre count, the centre's row / edge range (clamped, as tgn_attn_fwd);
  // 1 hop with records (tgn_agg_emit): its edges' neighbour rows too, so every row load is in round two
  const int xc = min(x, max(c.ccap - 1, 0));
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int64_t err = c.ctl[TGNX_CTL_ERR];
  const int R = c.cnt[c.rsel];
  int i, e0, e1, jrec = 0;
  if (c.cevj) {
    const int4 q = c.cevq[xc];
    jrec = c.cevj[xc * 16 + (lane & 15)];
    i = q.x;
    e0 = q.y;
    e1 = q.z;
  } else {
    i = c.cent_loc[xc];
    e0 = c.ceoff[xc];
    e1 = c.ceoff[xc + 1];
  }
  if (B == 0 || err != 0 || x >= R) return;
  const int C = c.C, HC = c.HC;
  const bool okl = lane < C;
  const float on = f01(okl);
  const int l0 = min(lane, C - 1);
  const float* Pi = c.P + (int64_t)i * 4 * HC;
  float* dPi = c.dP + (int64_t)i * 4 * HC;
  const float q0 = Pi[l0], q1 = Pi[C + l0];
  float g0 = c.dZc[(int64_t)x * HC + l0], g1 = c.dZc[(int64_t)x * HC + C + l0];
#pragma unroll
  for (int rp = 1; rp < REP; ++rp) {  // (the predictor's dZc copies, in copy order)
    g0 += c.dZc[rp * c.dzstride + (int64_t)x * HC + l0];
    g1 += c.dZc[rp * c.dzstride + (int64_t)x * HC + C + l0];
  }
  g0 *= on;
  g1 *= on;
  const float sqc = sqrtf((float)C);
  const int ne = e1 - e0;
  const int le = e0 + min(lane, max(ne - 1, 0));
  const int jl = c.cevj && ne <= 16 ? max(jrec, 0) : c.e_j[le];
  const uint64_t seed = (uint64_t)c.ctl[TGNX_CTL_SEED];
  const float al0 = c.alpha[(int64_t)le * 2], al1 = c.alpha[(int64_t)le * 2 + 1];
  const float a0 = lane < ne ? al0 : 0.f, a1 = lane < ne ? al1 : 0.f;
  float k0v = 1.f, k1v = 1.f;
  if (lane < ne && c.drop) {
    k0v = att_keep(c, seed, x, e0 + lane, 0);
    k1v = att_keep(c, seed, x, e0 + lane, 1);
  }
  if (ne > 0 && ne <= EB) {  // every ring of K <= 16: v, k and edge rows of all edges in one round
    float kk0[EB], kk1[EB], v0[EB], v1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = min(u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      const float ea = Ee[l0], eb = Ee[C + l0];
      kk0[u] = Pj[HC + l0] + ea;
      kk1[u] = Pj[HC + C + l0] + eb;
      v0[u] = Pj[2 * HC + l0] + ea;
      v1[u] = Pj[2 * HC + C + l0] + eb;
    }
    float da0 = 0.f, da1 = 0.f;
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // (no early exit: it kept the loop rolled; see attn_centre)
      const float p0 = wave_sum_f(g0 * v0[u]), p1 = wave_sum_f(g1 * v1[u]);
      if (lane == u && u < ne) { da0 = p0 * k0v; da1 = p1 * k1v; }
    }
    const float s0 = wave_sum_f(a0 * da0), s1 = wave_sum_f(a1 * da1);
    const float ds0 = a0 * (da0 - s0), ds1 = a1 * (da1 - s1);
    const float t0 = a0 * k0v, t1 = a1 * k1v;
    const float dq0s = ds0 / sqc, dq1s = ds1 / sqc;  // (per lane = per edge: one division, not one per edge)
    float dq0 = 0.f, dq1 = 0.f;
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // (lanes >= ne hold ds = 0: the clamped rows add exact zeros to dq)
      const float d0 = lane_f(dq0s, u), d1 = lane_f(dq1s, u);
      const float b0 = lane_f(t0, u), b1 = lane_f(t1, u);
      float* dEe = c.dE + (int64_t)(e0 + u) * HC;
      float* dKe = c.dKV + (int64_t)(e0 + u) * 2 * HC;  // [dk (HC) | dv (HC)]
      dq0 += d0 * kk0[u];
      dq1 += d1 * kk1[u];
      if (okl && wkv && u < ne) {
        const float dk0 = d0 * q0, dk1 = d1 * q1;
        const float dv0 = b0 * g0, dv1 = b1 * g1;
        dEe[lane] = dk0 + dv0;
        dEe[C + lane] = dk1 + dv1;
        dKe[lane] = dk0;
        dKe[C + lane] = dk1;
        dKe[HC + lane] = dv0;
        dKe[HC + C + lane] = dv1;
      }
    }
    if (okl) {
      dPi[lane] = dq0;
      dPi[C + lane] = dq1;
      dPi[3 * HC + lane] = g0;
      dPi[3 * HC + C + lane] = g1;
    }
    return;
  }
  // d alpha~_eh = Σ_{ch in h} dout (v_j + e); d alpha = d alpha~ * keep
  float da0 = 0.f, da1 = 0.f;
  for (int b = 0; b < ne; b += EB) {
    float v0[EB], v1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = min(b + u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      v0[u] = Pj[2 * HC + l0] + Ee[l0];
      v1[u] = Pj[2 * HC + C + l0] + Ee[C + l0];
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const float p0 = wave_sum_f(g0 * v0[u]), p1 = wave_sum_f(g1 * v1[u]);
      if (lane == b + u && b + u < ne) { da0 = p0 * k0v; da1 = p1 * k1v; }
    }
  }
  // softmax backward: d score = alpha (d alpha - Σ alpha d alpha)
  const float s0 = wave_sum_f(a0 * da0), s1 = wave_sum_f(a1 * da1);
  const float ds0 = a0 * (da0 - s0), ds1 = a1 * (da1 - s1);
  const float t0 = a0 * k0v, t1 = a1 * k1v;
  const float dq0s = ds0 / sqc, dq1s = ds1 / sqc;
  float dq0 = 0.f, dq1 = 0.f;
  for (int b = 0; b < ne; b += EB) {
    float kk0[EB], kk1[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = min(b + u, ne - 1);
      const float* Pj = c.P + (int64_t)lane_i(jl, e) * 4 * HC;
      const float* Ee = c.Ep + (int64_t)(e0 + e) * HC;
      kk0[u] = Pj[HC + l0] + Ee[l0];
      kk1[u] = Pj[HC + C + l0] + Ee[C + l0];
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int e = b + u;  // (e >= ne: ds = 0 there, and no stores)
      const float d0 = lane_f(dq0s, e), d1 = lane_f(dq1s, e);
      const float b0 = lane_f(t0, e), b1 = lane_f(t1, e);
      float* dEe = c.dE + (int64_t)(e0 + e) * HC;
      float* dKe = c.dKV + (int64_t)(e0 + e) * 2 * HC;  // [dk (HC) | dv (HC)]
      dq0 += d0 * kk0[u];
      dq1 += d1 * kk1[u];
      if (okl && wkv && e < ne) {
        const float dk0 = d0 * q0, dk1 = d1 * q1;
        const float dv0 = b0 * g0, dv1 = b1 * g1;
        dEe[lane] = dk0 + dv0;
        dEe[C + lane] = dk1 + dv1;
        dKe[lane] = dk0;
        dKe[C + lane] = dk1;
        dKe[HC + lane] = dv0;
        dKe[HC + C + lane] = dv1;
      }
    }
  }
  if (okl) {
    dPi[lane] = dq0;
    dPi[C + lane] = dq1;
    dPi[3 * HC + lane] = g0;
    dPi[3 * HC + C + lane] = g1;
  }
}

// dP[j][k | v columns] += Σ over edges e with neighbour j of dKV[e] (the zeroed accumulators of
// agg_emit).  Workgroup per chunk of KVR_CH consecutive edges, sorted by neighbour in LDS (rank by
// counting); each wave takes KVR_CH / 4 sorted edges, loads all their rows at once (lanes over columns)
// and sums runs of equal neighbours in registers: one global atomic per (wave, neighbour run, column),
// so a hub row sees a few atomics per chunk instead of one per edge.  (Merging in LDS with ds_add_f32
// instead ran at about one element per two clocks per CU: slower than the contention it removed.)
#ifndef TGNX_KVR_CH
#define TGNX_KVR_CH 32  // 64: 133 VGPRs in the kv_reduce job lowered the whole launch to 3 waves per SIMD (+0.9 us)
#endif
constexpr int KVR_CH = TGNX_KVR_CH;   // edges per workgroup
constexpr int KVR_PW = KVR_CH / 4;    // sorted edges per wave
__device__ void kv_reduce_body(const Ctx& c, int bid) {
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int E = level_edges(c);
  const int eb = bid * KVR_CH;
  if (eb >= E) return;  // whole workgroup
  const int ne = min(KVR_CH, E - eb);
  const int HC = c.HC, H2 = 2 * HC;
  __shared__ int sj[KVR_CH], sorder[KVR_CH];
  const int t = threadIdx.x;
  if (t < KVR_CH) sj[t] = t < ne ? c.e_j[eb + t] : INT_MAX;
  __syncthreads();
  if (t < ne) {  // stable rank of (neighbour, edge); padding keys (INT_MAX, past ne) rank after every edge
    const int key = sj[t];
    int r = 0;
#pragma unroll 16
    for (int u = 0; u < KVR_CH; ++u) {
      const int ju = sj[u];
      r += (ju < key) || (ju == key && u < t);
    }
    sorder[r] = t;
  }
  __syncthreads();
  const int w = t >> 6, lane = t & 63;
  const int i0 = w * KVR_PW;
  if (i0 >= ne) return;
  const int n = min(KVR_PW, ne - i0);
  int jj[KVR_PW], er[KVR_PW];
#pragma unroll
  for (int u = 0; u < KVR_PW; ++u) {
    const int e = sorder[i0 + min(u, n - 1)];
    jj[u] = sj[e];
    er[u] = eb + e;
  }
  for (int c0 = 0; c0 < H2; c0 += 256) {  // 4 columns per lane per pass (one pass at HC <= 128)
    float v[KVR_PW][4];
#pragma unroll
    for (int u = 0; u < KVR_PW; ++u)
#pragma unroll
      for (int p = 0; p < 4; ++p) v[u][p] = c.dKV[(int64_t)er[u] * H2 + min(c0 + lane + 64 * p, H2 - 1)];
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int jc = jj[0];
#pragma unroll
    for (int u = 0; u < KVR_PW; ++u) {
      const bool in = u < n;
      if (in && jj[u] != jc) {  // wave-uniform run boundary
        float* dst = c.dP + (int64_t)jc * 4 * HC + HC + c0 + lane;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          if (c0 + lane + 64 * p < H2) atomicAdd(dst + 64 * p, a[p]);
          a[p] = 0.f;
        }
        jc = jj[u];
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) a[p] += in ? v[u][p] : 0.f;
    }
    float* dst = c.dP + (int64_t)jc * 4 * HC + HC + c0 + lane;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      if (c0 + lane + 64 * p < H2) atomicAdd(dst + 64 * p, a[p]);
  }
}

__global__ void __launch_bounds__(256) tgn_kv_reduce(Ctx c) { kv_reduce_body(c, blockIdx.x); }
// the same work as a BlockJob of a gemmN launch (beside the GEMMs that need only dE, see the train step)
struct KvReduceJob {
  Ctx c;
  __device__ void operator()(int bid, float*) const { kv_reduce_body(c, bid); }
};

// ------------------------------------------------------------------ backward GEMM operands / epilogues
// (n, m) -> z0[m][n], and 1 in the extra column n == D (bias gradient)
struct LoadZ1T {
  const float* Z0;
  int D;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int m) const {
    return *(n < D ? Z0 + (int64_t)m * D + n : kOne4);
  }
};
struct EpiProjGrad {
  float* g;
  int64_t wq, bq, pw, pb;  // projection gi: weights wq + gi pw, bias bq + gi pb
  int HC, D;
  AdamFuse af;
  template <class T>
  static constexpr int nx() { return (T::tm * T::tn + 255) / 256; }
  template <class T, int NI>
  __device__ void items(const T& t, int64_t (&ix)[NI], float (&vx)[NI]) const {
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int x = threadIdx.x + 256 * it;
      const int r = x / T::tn, cc = x % T::tn, row = t.m0 + r, n = t.n0 + cc;
      const bool ok = x < T::tm * T::tn && row < t.M && n < t.N;
      const int gi = proj_g(row, HC), q = row - gi * HC;
      vx[it] = ok ? t(r, cc) : 0.f;
      ix[it] = !ok ? -1 : n < D ? wq + gi * pw + (int64_t)q * D + n : bq + gi * pb + q;
    }
  }
  template <class T>
  __device__ void operator()(const T& t) const {
    int64_t ix[nx<T>()];
    float vx[nx<T>()];
    items(t, ix, vx);
    af.put_n(g, ix, vx);
  }
};
// plain row-major weight gradient (lin_edge): g[off + m ldc + n]
struct EpiGradStore {
  float* g;
  int64_t off;
  int ldc;
  AdamFuse af;
  template <class T>
  static constexpr int nx() { return T::per; }
  template <class T, int NI>
  __device__ void items(const T& t, int64_t (&ix)[NI], float (&vx)[NI]) const {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, n = t.n0 + cc;
      const bool ok = m < t.M && n < t.N;
      vx[i] = ok ? t(r, cc) : 0.f;
      ix[i] = ok ? off + (int64_t)m * ldc + n : -1;
    }
  }
  template <class T>
  __device__ void operator()(const T& t) const {
    int64_t ix[nx<T>()];
    float vx[nx<T>()];
    items(t, ix, vx);
    af.put_n(g, ix, vx);
  }
};
// link predictor weight grads as one GEMM over 3 * nloc rows (block-diagonal K):
// rows r < D: dW_src = Σ (dhp + dhn) zsᵀ ; rows r >= D: dW_dst = Σ dhp zpᵀ + dhn znᵀ
struct LoadLpA {
  const float* evs;
  const int64_t* ctl;
  int D, S;
  static constexpr bool k_fast = false;
  __device__ float operator()(int r, int k) const {
    const int lo = (int)ctl[TGNX_CTL_LO], nloc = max(1, (int)(ctl[TGNX_CTL_HI] - ctl[TGNX_CTL_LO]));
    const int blk = (k >= nloc) + (k >= 2 * nloc), i = lo + k - blk * nloc;  // k < 3 nloc: no division
    const float* ev = evs + (int64_t)i * S;
    const bool src = r < D;
    const int o = src ? r : r - D;
    const float a = ev[3 * D + o], b = ev[4 * D + o];   // dhp, dhn
    return src ? (blk == 0 ? a + b : 0.f) : (blk == 1 ? a : blk == 2 ? b : 0.f);
  }
};
struct LoadLpB {
  const float* evs;
  const int64_t* ctl;
  int D, S;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int k) const {
    const int lo = (int)ctl[TGNX_CTL_LO], nloc = max(1, (int)(ctl[TGNX_CTL_HI] - ctl[TGNX_CTL_LO]));
    const int blk = (k >= nloc) + (k >= 2 * nloc), i = lo + k - blk * nloc;
    return evs[(int64_t)i * S + blk * D + n];
  }
};
struct EpiLpGrad {
  float* g;
  int64_t lsw, ldw;
  int D;
  AdamFuse af;
  template <class T>
  static constexpr int nx() { return (T::tm * T::tn + 255) / 256; }
  template <class T, int NI>
  __device__ void items(const T& t, int64_t (&ix)[NI], float (&vx)[NI]) const {
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int x = threadIdx.x + 256 * it;
      const int r = x / T::tn, cc = x % T::tn, row = t.m0 + r, n = t.n0 + cc;
      const bool ok = x < T::tm * T::tn && row < t.M && n < t.N;
      vx[it] = ok ? t(r, cc) : 0.f;
      ix[it] = ok ? (row < D ? lsw + (int64_t)row * D : ldw + (int64_t)(row - D) * D) + n : -1;
    }
  }
  template <class T>
  __device__ void operator()(const T& t) const {
    int64_t ix[nx<T>()];
    float vx[nx<T>()];
    items(t, ix, vx);
    af.put_n(g, ix, vx);
  }
};
// Δt-encoding parameter grads from a tile of d(encoding) (dA): per row-tile partials
//   tgp[row][n] = Σ_r -dA[r][n] S1[r][n],  tgp[row][D + n] = Σ_r -dA[r][n] S0[r][n]
// (S0 = sin(w Δt + b), S1 = S0 Δt, precomputed), summed in fixed order by TeReduceTail.
template <class T>
__device__ __forceinline__ void te_tile_grad(const T& t, const float* S0, const float* S1, float* tgp,
                                             int D) {
  const int groups = blockDim.x / t.tn;
  const int cc = threadIdx.x % t.tn, g = threadIdx.x / t.tn, n = t.n0 + cc;
  float sw = 0.f, sb = 0.f;
  if (g < groups && n < t.N)
    for (int r = g; r < t.tm && t.m0 + r < t.M; r += groups) {
      const int64_t o = (int64_t)(t.m0 + r) * D + n;
      const float da = -t(r, cc);
      sw += da * S1[o];
      sb += da * S0[o];
    }
  float* red = t.scratch;  // [2][groups][tn]
  if (g < groups) {
    red[g * t.tn + cc] = sw;
    red[(groups + g) * t.tn + cc] = sb;
  }
  __syncthreads();
  if (threadIdx.x < t.tn && n < t.N) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < groups; ++q) {
      a += red[q * t.tn + cc];
      b += red[(groups + q) * t.tn + cc];
    }
    tgp[(int64_t)t.tile_row() * 2 * D + n] = a;
    tgp[(int64_t)t.tile_row() * 2 * D + D + n] = b;
  }
}
// d(edge attr enc) of the sampled edges; S1 = sin Δt formed here from lu / e_t
// (map != nullptr: rows are root edges, their Δt data that of the outer edge map[e]; partial rows from row0)
struct EpiTeEdge {
  const int* e_j;
  const float *e_t, *lu;
  float* tgp;
  int D;
  const int* map = nullptr;
  int row0 = 0;
  const float *tw = nullptr, *tb = nullptr;  // the time encoder: the sine recomputed from Δt
  template <class T>
  __device__ void operator()(const T& t) const {
    constexpr int groups = 256 / T::tn, per = T::tm / groups;
    const int cc = threadIdx.x % T::tn, g = threadIdx.x / T::tn, n = t.n0 + cc;
    int ej[per], e2[per];
    float et[per], sn[per], dt[per];
#pragma unroll
    for (int i = 0; i < per; ++i) {
      const int e = t.m0 + g + groups * i;
      e2[i] = map ? map[min(e, t.M - 1)] : e;
    }
#pragma unroll
    for (int i = 0; i < per; ++i) {
      const int e = t.m0 + g + groups * i;
      const bool ok = e < t.M && n < t.N;
      ej[i] = ok ? e_j[e2[i]] : 0;
      et[i] = ok ? e_t[e2[i]] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < per; ++i) dt[i] = lu[ej[i]] - et[i];
    {  // the forward's own argument (tgn_agg_emit: fmaf(w, lu - t, b), same lu / t), so the same sin
      const int nc = min(n, D - 1);
      const float w = tw[nc], b = tb[nc];
#pragma unroll
      for (int i = 0; i < per; ++i) {
        float cs;
        te_sincos(fmaf(w, dt[i], b), sn[i], cs);
        const int e = t.m0 + g + groups * i;
        if (!(e < t.M && n < t.N)) sn[i] = 0.f;
      }
    }
    float sw = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < per; ++i) {
      const float da = -t(g + groups * i, cc) * sn[i];
      sw += da * dt[i];
      sb += da;
    }
    float* red = t.scratch;
    if (g < groups) {
      red[g * t.tn + cc] = sw;
      red[(groups + g) * t.tn + cc] = sb;
    }
    __syncthreads();
    if (threadIdx.x < t.tn && n < t.N) {
      float a = 0.f, b = 0.f;
      for (int q = 0; q < groups; ++q) {
        a += red[q * t.tn + cc];
        b += red[(groups + q) * t.tn + cc];
      }
      tgp[(int64_t)(row0 + t.tile_row()) * 2 * D + n] = a;
      tgp[(int64_t)(row0 + t.tile_row()) * 2 * D + D + n] = b;
    }
  }
};
// [W_query; W_key; W_value; W_skip] as the B operand of dz0 = dP W: element (n, k) = W_{k/HC}[k%HC][n]
struct LoadProjWT {
  const float* w;  // wq; projection g at w + g * pw
  int64_t pw;
  int HC, D;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int k) const {
    const int g = proj_g(k, HC), r = k - g * HC;
    return w[g * pw + (int64_t)r * D + n];
  }
};
// GRUCell backward from dh' (memory is detached, so only the gate pre-activations get gradients):
// dG[m][4j+g] = (d pre_r, d pre_z, d gi_n, d gh_n)
struct EpiGruBwd {
  const float *gates, *mem;
  const int64_t* nid;
  float* dG;
  int D;
  const float* Hp = nullptr;  // the rows' pre-update memory, stored densely by the GRU forward (no node-id gather)
  // a 16 x 16 tile's element of this thread (GemmTile<16, 16>::row_of / col_of (0)): its node and saved gates,
  // loaded with the tile's first operand round (gemm_tile_direct)
  struct Pre {
    int64_t node;
    float4 gt;
    float h;
  };
  template <class RI>
  __device__ Pre pre(int m0, int n0, int M, int N, RI) const {
    const int m = min(m0 + GemmTile<16, 16>::row_of(0), M - 1), j = min(n0 + GemmTile<16, 16>::col_of(0), N - 1);
    if (Hp) return Pre{0, *reinterpret_cast<const float4*>(gates + ((int64_t)m * D + j) * 4), Hp[(int64_t)m * D + j]};
    return Pre{nid[m], *reinterpret_cast<const float4*>(gates + ((int64_t)m * D + j) * 4), 0.f};
  }
  template <class T>
  __device__ void operator()(const T& t, const Pre& p) const {
    static_assert(T::per == 1, "16 x 16 tiles");
    const int r = T::row_of(0), cc = T::col_of(0), m = t.m0 + r, j = t.n0 + cc;
    const float h = Hp ? p.h : mem[p.node * D + min(j, t.N - 1)];
    if (m >= t.M || j >= t.N) return;
    const float dhp = t(r, cc);
    const float rr = p.gt.x, zz = p.gt.y, nn = p.gt.z, ghn = p.gt.w;
    const float dn = dhp * (1.0f - zz), dz = dhp * (h - nn);
    const float dpn = dn * (1.0f - nn * nn);
    const float dr = dpn * ghn;
    float4* o = reinterpret_cast<float4*>(dG + ((int64_t)m * D + j) * 4);
    *o = make_float4(dr * rr * (1.0f - rr), dz * zz * (1.0f - zz), dpn, dpn * rr);
  }
  template <class T>  // (staged tiles of any shape)
  __device__ void operator()(const T& t) const {
    int64_t node[T::per];
    float4 gt[T::per];
    float h[T::per];
#pragma unroll
    for (int i = 0; i < T::per; ++i) {  // gathers first (no stores in between)
      const int m = t.m0 + T::row_of(i), j = t.n0 + T::col_of(i);
      const bool ok = m < t.M && j < t.N;
      node[i] = ok && !Hp ? nid[m] : 0;
      gt[i] = ok ? *reinterpret_cast<const float4*>(gates + ((int64_t)m * D + j) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int m = min(t.m0 + T::row_of(i), t.M - 1), j = min(t.n0 + T::col_of(i), t.N - 1);
      h[i] = Hp ? Hp[(int64_t)m * D + j] : mem[node[i] * D + t.n0 + T::col_of(i)];
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, j = t.n0 + cc;
      if (m >= t.M || j >= t.N) continue;
      const float dhp = t(r, cc);
      const float rr = gt[i].x, zz = gt[i].y, nn = gt[i].z, ghn = gt[i].w;
      const float dn = dhp * (1.0f - zz), dz = dhp * (h[i] - nn);
      const float dpn = dn * (1.0f - nn * nn);
      const float dr = dpn * ghn;
      float4* o = reinterpret_cast<float4*>(dG + ((int64_t)m * D + j) * 4);
      *o = make_float4(dr * rr * (1.0f - rr), dz * zz * (1.0f - zz), dpn, dpn * rr);
    }
  }
};
// [X | memory | 1] rows as the B operand of dW_gru = dGᵀ [X | H | 1]
struct LoadGruAT1 {
  const float* X;
  const float* mem;
  const int64_t* nid;
  int Qm, D;
  static constexpr bool k_fast = false;
  using Idx = int64_t;  // k = sampled node: its id, per chunk
  static constexpr bool row_idx = false;
  __device__ Idx index(int, int m) const { return nid[m]; }
  __device__ float load(Idx v, int n, int m) const {
    const bool x = n < Qm, one = n >= Qm + D;
    return *(x ? X + (int64_t)m * Qm + n : one ? kOne4 : mem + v * D + (n - Qm));
  }
};
// the same with the rows' pre-update memory stored densely: no node-id round per K chunk
struct LoadGruAT1H {
  const float* X;
  const float* Hp;
  int Qm, D;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int m) const {
    const bool x = n < Qm, one = n >= Qm + D;
    return *(x ? X + (int64_t)m * Qm + n : one ? kOne4 : Hp + (int64_t)m * D + (n - Qm));
  }
};
struct EpiGruWGrad {
  float* g;
  int64_t wih, whh, bih, bhh;
  int Qm, D;
  AdamFuse af;
  template <class T>
  static constexpr int nx() { return 2 * ((T::tm * T::tn + 255) / 256); }  // the (r, z) bias columns feed both b_ih and b_hh
  template <class T, int N2>
  __device__ void items(const T& t, int64_t (&ix)[N2], float (&vx)[N2]) const {
#pragma unroll
    for (int it = 0; it < N2 / 2; ++it) {
      const int x = threadIdx.x + 256 * it;
      const int r = x / T::tn, cc = x % T::tn, row = t.m0 + r, n = t.n0 + cc;
      const bool ok = x < T::tm * T::tn && row < t.M && n < t.N;
      const int j = row >> 2, gg = row & 3;
      const float v = ok ? t(r, cc) : 0.f;
      int64_t a = -1, b = -1;
      if (ok) {
        if (n < Qm) {
          if (gg < 3) a = wih + (int64_t)(gg * D + j) * Qm + n;
        } else if (n < Qm + D) {
          if (gg != 2) a = whh + (int64_t)((gg == 3 ? 2 : gg) * D + j) * D + (n - Qm);
        } else if (gg < 2) {
          a = bih + gg * D + j;
          b = bhh + gg * D + j;
        } else {
          a = gg == 2 ? bih + 2 * D + j : bhh + 2 * D + j;
        }
      }
      ix[2 * it] = a;
      ix[2 * it + 1] = b;
      vx[2 * it] = vx[2 * it + 1] = v;
    }
  }
  template <class T>
  __device__ void operator()(const T& t) const {
    int64_t ix[nx<T>()];
    float vx[nx<T>()];
    items(t, ix, vx);
    af.put_n(g, ix, vx);
  }
};
// encoding columns of W_ih as the B operand of dX_enc = dG W_cat[:, enc]: element (n, r = 4j+g)
struct LoadGruWencT {
  const float* wih;
  int Qm, D, off;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int r) const {
    const int j = r >> 2, gg = r & 3;
    return *(gg == 3 ? kZero4 : wih + (int64_t)(gg * D + j) * Qm + off + n);
  }
};
// ---- RNNCell memory updater (DyRepMemory memory_updater_type = 'rnn', modules/memory_module.py:256-259):
// h' = tanh(W_ih x + b_ih + W_hh h + b_hh), one GEMM column per unit over [message | memory].
struct LoadRnnW {
  const float *wih, *whh;
  int Qm, D;
  static constexpr bool k_fast = true;
  __device__ float operator()(int n, int k) const {
    const float* p = k < Qm ? wih + (int64_t)n * Qm + k : whh + (int64_t)n * D + (k - Qm);
    return *p;
  }
  __device__ bool vec4() const { return ((Qm | D) & 3) == 0 && al16(wih) && al16(whh); }
  __device__ float4 load4(int n, int k) const {
    const float* p = k < Qm ? wih + (int64_t)n * Qm + k : whh + (int64_t)n * D + (k - Qm);
    return *reinterpret_cast<const float4*>(p);
  }
};
struct EpiRnn {
  const float *bih, *bhh;
  int D;
  float* Z0;
  template <class T>
  __device__ void operator()(const T& t) const {
    float b[T::per];
#pragma unroll
    for (int i = 0; i < T::per; ++i) {  // gathers first
      const int j = min(t.n0 + T::col_of(i), D - 1);
      b[i] = bih[j] + bhh[j];
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, j = t.n0 + cc;
      if (m >= t.M || j >= t.N) continue;
      Z0[(int64_t)m * D + j] = tanhf(t(r, cc) + b[i]);
    }
  }
};
// dh' (the dz0 GEMM) -> d(pre-activation) = dh' (1 - h'^2)
struct EpiRnnBwd {
  const float* Z0;
  float* dG;
  int D;
  template <class T>
  __device__ void operator()(const T& t) const {
    float h[T::per];
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int m = min(t.m0 + T::row_of(i), t.M - 1), j = min(t.n0 + T::col_of(i), D - 1);
      h[i] = Z0[(int64_t)m * D + j];
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, j = t.n0 + cc;
      if (m >= t.M || j >= t.N) continue;
      dG[(int64_t)m * D + j] = t(r, cc) * (1.0f - h[i] * h[i]);
    }
  }
};
// dW = dGᵀ [X | H | 1]: row j -> W_ih[j, :Qm], W_hh[j, :], and b_ih[j], b_hh[j] (both get the column sum)
struct EpiRnnWGrad {
  float* g;
  int64_t wih, whh, bih, bhh;
  int Qm, D;
  AdamFuse af;
  template <class T>
  __device__ void operator()(const T& t) const {
    constexpr int NI = (T::tm * T::tn + 255) / 256;
    int64_t ix[2 * NI];
    float vx[2 * NI];
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int x = threadIdx.x + 256 * it;
      const int r = x / T::tn, cc = x % T::tn, j = t.m0 + r, n = t.n0 + cc;
      const bool ok = x < T::tm * T::tn && j < t.M && n < t.N;
      int64_t a = -1, b = -1;
      if (ok) {
        if (n < Qm) a = wih + (int64_t)j * Qm + n;
        else if (n < Qm + D) a = whh + (int64_t)j * D + (n - Qm);
        else {
          a = bih + j;
          b = bhh + j;
        }
      }
      ix[2 * it] = a;
      ix[2 * it + 1] = b;
      vx[2 * it] = vx[2 * it + 1] = ok ? t(r, cc) : 0.f;
    }
    af.put_n(g, ix, vx);
  }
};
// encoding columns of W_ih as the B operand of dX_enc = dG W_ih[:, enc]: element (n, r = unit)
struct LoadRnnWencT {
  const float* wih;
  int Qm, D, off;
  static constexpr bool k_fast = false;
  __device__ float operator()(int n, int r) const { return wih[(int64_t)r * Qm + off + n]; }
};
// the memory updater's functors by cell type (GEMM columns per unit G: GRU 4 interleaved gates, RNN 1)
template <int CELL>
struct CellOps;
template <>
struct CellOps<0> {
  static constexpr int G = 4;
  static __host__ LoadGruW w(const Ctx& c) { return LoadGruW{c.params + c.L.w_ih, c.params + c.L.w_hh, c.Qm, c.D}; }
  static __host__ EpiGru epi(const Ctx& c, const int64_t* list, int64_t base) {
    return EpiGru{c.params + c.L.b_ih, c.params + c.L.b_hh, c.mem, list, base, c.D, c.Z0, c.gates};
  }
  static __host__ EpiGru epi_train(const Ctx& c) {
    EpiGru e = epi(c, c.nid, 0);
    e.Hp = c.Hp;
    return e;
  }
  static __host__ EpiGruBwd bwd(const Ctx& c) {
    return EpiGruBwd{c.gates, c.mem, c.nid, c.dG, c.D, c.Hp};
  }
  // B operand of dW_cell = dGᵀ [X | H | 1]
  static __host__ auto hT(const Ctx& c) {
    return LoadGruAT1H{c.X, c.Hp, c.Qm, c.D};
  }
  static __host__ EpiGruWGrad wgrad(const Ctx& c) {
    return EpiGruWGrad{c.grads, c.L.w_ih, c.L.w_hh, c.L.b_ih, c.L.b_hh, c.Qm, c.D, c.adf};
  }
  static __host__ LoadGruWencT wenc(const Ctx& c) { return LoadGruWencT{c.params + c.L.w_ih, c.Qm, c.D, 2 * c.D + c.d}; }
};
template <>
struct CellOps<1> {
  static constexpr int G = 1;
  static __host__ LoadRnnW w(const Ctx& c) { return LoadRnnW{c.params + c.L.w_ih, c.params + c.L.w_hh, c.Qm, c.D}; }
  static __host__ EpiRnn epi(const Ctx& c, const int64_t*, int64_t) {
    return EpiRnn{c.params + c.L.b_ih, c.params + c.L.b_hh, c.D, c.Z0};
  }
  static __host__ EpiRnn epi_train(const Ctx& c) { return epi(c, c.nid, 0); }
  static __host__ EpiRnnBwd bwd(const Ctx& c) { return EpiRnnBwd{c.Z0, c.dG, c.D}; }
  static __host__ LoadGruAT1 hT(const Ctx& c) { return LoadGruAT1{c.X, c.mem, c.nid, c.Qm, c.D}; }
  static __host__ EpiRnnWGrad wgrad(const Ctx& c) {
    return EpiRnnWGrad{c.grads, c.L.w_ih, c.L.w_hh, c.L.b_ih, c.L.b_hh, c.Qm, c.D, c.adf};
  }
  static __host__ LoadRnnWencT wenc(const Ctx& c) { return LoadRnnWencT{c.params + c.L.w_ih, c.Qm, c.D, 2 * c.D + c.d}; }
};
// message-encoding -> Δt-encoding parameter grads (Last: the winner's Δt; Mean: each stored
// message's Δt with weight 1 / count, folded into s0m / s1m by agg_node), per row-tile partials
struct EpiTeMsg {
  const float *s0m, *s1m;
  float* tgp;
  int D, row0;
  template <class T>
  __device__ void operator()(const T& t) const { te_tile_grad(t, s0m, s1m, tgp + (int64_t)row0 * 2 * D, D); }
};

// Δt-encoding grads: fixed-order sum of the partial rows into grads (before any all-reduce); rides
// as the tail blocks of the weight-gradient fixup launch (TrainTail below)
struct TeReduceTail {
  Ctx c;
  int rows_edge, rows_msg;
  // tail block b: columns [64 b, 64 b + 64) of the 2D (w, b) gradients; wave w sums the rows
  // [w R / 4, (w + 1) R / 4) with 8 loads in flight, the 4 wave sums combine in fixed order
  __device__ __forceinline__ void operator()(int bid) const {
    __shared__ float red[4][64];
    const int D = c.D, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x = bid * 64 + lane;
    if (bid * 64 >= 2 * D) return;
    const int B = (int)c.ctl[TGNX_CTL_B];
    if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
    const int E = c.cnt[CNT_E], M = c.cnt[CNT_M];
    const int re = min(rows_edge, (E + G32::TM - 1) / G32::TM), rm = min(rows_msg, (M + G32::TM - 1) / G32::TM);
    // 2 hops: the root edges' rows (conv2's lin_edge) follow at tgp_e1
    const int re1 = c.layers == 2 ? min(c.tgp_rows - c.tgp_e1, (c.cnt[CNT_E1] + G32::TM - 1) / G32::TM) : 0;
    const int R = re + rm + re1, r0 = wv * R / 4, r1 = (wv + 1) * R / 4;
    const int xc = min(x, 2 * D - 1);
    float s = 0.f;
    for (int r = r0; r < r1; r += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = min(r + u, r1 - 1);
        const int row = rr < re ? rr : rr < re + rm ? rows_edge + (rr - re) : c.tgp_e1 + (rr - re - rm);
        v[u] = c.tgp[(int64_t)row * 2 * D + xc];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u] * f01(r + u < r1);
    }
    red[wv][lane] = s;
    __syncthreads();
    if (wv == 0 && x < 2 * D) {
      const float tot = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
      c.adf.put(c.grads, (x < D ? c.L.te_w : c.L.te_b - D) + x, tot);
    }
  }
};

// ------------------------------------------------------------------ optimizer + state update
// Adam over the flat buffer; the last nrb blocks (data parallel, after the exchange) write the exchanged
// memory rows instead (tgn_apply_rows' body).  Skipped when the step's batch was empty (STEP_B: a
// pipelined step's descriptor already holds the next batch).
__device__ void apply_rows_body(float* mem, int64_t* lu, float* rows, int64_t nrows, int D, int64_t N, int bid, int nb);
__global__ void __launch_bounds__(256) tgn_adam(Ctx c, float* rows, int64_t nrows, int nrb) {
  TGNX_STAMP(7);
  if ((int)blockIdx.x >= (int)gridDim.x - nrb) {
    apply_rows_body(c.mem, c.lu_buf, rows, nrows, c.D, c.N, (int)blockIdx.x - ((int)gridDim.x - nrb), nrb);
    return;
  }
  // one load round: the step's B / error words and Adam scalars (tgn_pred_train wrote them for this t) with this
  // thread's elements (the separate optimizer pass of the data-parallel step heads the next step's graph)
  const int64_t n4 = c.L.total / 4;
  const int nab = (int)gridDim.x - nrb;
  float4* P4 = reinterpret_cast<float4*>(c.params);
  float4* M4 = reinterpret_cast<float4*>(c.am);
  float4* V4 = reinterpret_cast<float4*>(c.av);
  const float4* G4 = reinterpret_cast<const float4*>(c.grads);
  const int64_t B = c.ctl[TGNX_CTL_STEP_B], err = c.ctl[TGNX_CTL_ERR];
  const float* sc = reinterpret_cast<const float*>(c.ctl + TGNX_CTL_ADAM_SC);
  const float step = sc[0], bc2s = sc[1];
  if (blockIdx.x == 0 && threadIdx.x == 0 && B != 0 && err == 0)
    *reinterpret_cast<double*>(c.ctl + TGNX_CTL_LOSS) += (double)c.grads[c.L.total] * (double)B;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n4; x += (int64_t)nab * blockDim.x) {
    const float4 g = G4[x];
    float4 m = M4[x], v = V4[x], p = P4[x];
    if (B == 0 || err != 0) return;
    adam1(g.x, m.x, v.x, p.x, c.b1, c.b2, c.eps, step, bc2s);
    adam1(g.y, m.y, v.y, p.y, c.b1, c.b2, c.eps, step, bc2s);
    adam1(g.z, m.z, v.z, p.z, c.b1, c.b2, c.eps, step, bc2s);
    adam1(g.w, m.w, v.w, p.w, c.b1, c.b2, c.eps, step, bc2s);
    M4[x] = m;
    V4[x] = v;
    P4[x] = p;
  }
}

// data-parallel row header (TGNX_TGN_ROW): node, last_update as floats holding exact integers < 2^24
// (node; last_update bits 0-23, 24-47, 48-63), so that the rows survive the summing exchange (the
// all-reduce that carries them adds only zeros to them).  Unused slot: node -1.
__device__ __forceinline__ void xrow_header(float* h, int64_t v, int64_t luv) {
  const uint64_t b = (uint64_t)luv;
  h[0] = (float)v;
  h[1] = (float)(uint32_t)(b & 0xFFFFFFull);
  h[2] = (float)(uint32_t)((b >> 24) & 0xFFFFFFull);
  h[3] = (float)(uint32_t)(b >> 48);
}
// ring insert of the batch (neighbor_loader.py:52-104): wave per node run of the ring plan (4 per block)
__device__ __forceinline__ void ring_merge_block(const Ctx& c, int blk, int B, int64_t start) {
  const int r = blk * 4 + (threadIdx.x >> 6);
  const PlanOut pv = plan_view(c, start);
  int a, len;
  if (plan_run(pv.rruns, pv.pc, pv.pc + TGNX_PLAN_PMAX, c.pplan, r, a, len))  // r = the node's rank among the batch's nodes
    ring_merge_run(c.nbr, c.eid, c.rt, c.K, c.ev_src + start, c.ev_dst + start, c.ev_t + start, B,
                   c.ctl[TGNX_CTL_CUR_EID], c.assoc, pv.rkeys, a, len, r, threadIdx.x & 63);
}
// update_state pieces (memory_module.py:126-150, :180-191) and the ring insert, by block range:
// [0, nmem): memory / last_update of the update list from the GRU rows (wave per node; train rows
// are the sampled nodes' rows via assoc, eval / flush rows are list positions);
// [nmem, nmem + nst): message stores of the batch; the rest: ring merge, wave per node run.
__device__ __forceinline__ void update_body(const Ctx& c, int blk, int nmem, int nst, int mem_mode, const int64_t* list,
                            const int* list_cnt, int n_host, int64_t base) {
  const int lane = threadIdx.x & 63;
  if (blk < nmem) {
    const int RW = TGNX_TGN_ROW(c.D);
    if (mem_mode == 0 && (c.ctl[TGNX_CTL_B] == 0 || c.ctl[TGNX_CTL_ERR] != 0)) {
      // nothing updated: every exchange slot of this rank unused (the slots hold zeros since the last
      // apply, which would otherwise read as node 0)
      if (c.xrows)
        for (int u = blk * blockDim.x + threadIdx.x; u < c.xcap; u += nmem * blockDim.x) c.xrows[(int64_t)u * RW] = -1.f;
      return;
    }
    const int n = list_cnt ? *list_cnt : n_host;
    float* xr = mem_mode == 0 ? c.xrows : nullptr;
    if (xr && n > c.xcap) {
      if (blk == 0 && threadIdx.x == 0) *c.errw |= 8;
      return;
    }
    for (int u = blk * 4 + (threadIdx.x >> 6); u < n; u += nmem * 4) {
      const int64_t v = list ? list[u] : base + u;
      const int m = mem_mode == 0 ? c.upd_loc[u] : u;
      const int64_t luv = (int64_t)c.lu[m];
      const float* zrow = c.Zupd && mem_mode == 0 ? c.Zupd + (int64_t)u * c.D : c.Z0 + (int64_t)m * c.D;
      for (int k = lane; k < c.D; k += 64) {
        const float z = zrow[k];
        c.mem[v * c.D + k] = z;
        if (xr) xr[(int64_t)u * RW + 4 + k] = z;
      }
      if (lane == 0) {
        c.lu_buf[v] = luv;
        if (xr) xrow_header(xr + (int64_t)u * RW, v, luv);
      }
    }
    if (xr)  // unused slots
      for (int u = n + blk * blockDim.x + threadIdx.x; u < c.xcap; u += nmem * blockDim.x) xr[(int64_t)u * RW] = -1.f;
    return;
  }
  const int B = (int)c.ctl[TGNX_CTL_B];
  if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  if (blk < nmem + nst) {
    const int bid = blk - nmem;
    const PlanOut pv = plan_view(c, start);
    const int* spc = pv.pc + 2 * TGNX_PLAN_PMAX;
    const int n2 = 2 * B, U = plan_runs(spc, c.pplan);
    const int64_t ab = 2 * start;  // arena slot of this batch
    for (int p = bid * blockDim.x + threadIdx.x; p < n2; p += nst * blockDim.x)
      c.arena[ab + p] = start + (int64_t)(pv.skeys[p] & 0xFFFFFFFFull);
    for (int r = bid * blockDim.x + threadIdx.x; r < U; r += nst * blockDim.x) {
      int a, len;
      plan_run(pv.sruns, spc, spc + TGNX_PLAN_PMAX, c.pplan, r, a, len);
      const uint64_t k = pv.skeys[a];
      const int64_t v = (int64_t)(k >> 33);
      const int dir = (int)((k >> 32) & 1u);
      c.st[4 * v + 2 * dir] = ab + a;
      c.st[4 * v + 2 * dir + 1] = len;
    }
    return;
  }
  ring_merge_block(c, blk - nmem - nst, B, start);
}
// the train step's ring insert, riding in the GRU ‖ lin_edge launch: nothing after tgn_agg_emit reads the
// ring (the sampled edges are copied out), and the next batch's marking runs after it
struct RingMergeJob {
  Ctx c;
  __device__ void operator()(int bid, float*) const {
    const int B = (int)c.ctl[TGNX_CTL_B];
    if (B == 0 || c.ctl[TGNX_CTL_ERR] != 0) return;
    ring_merge_block(c, bid, B, c.ctl[TGNX_CTL_BATCH_START]);
  }
};
// pipelined step: the next batch's marking riding in a launch after the ring insert (nb 256-thread blocks;
// the launch's LDS holds the block's bitmaps)
struct MarkNextJob {
  Ctx c;
  int nb;
  __device__ void operator()(int bid, float* smem) const {
    mark_body<true>(c, bid, nb, 1, reinterpret_cast<uint32_t*>(smem));
  }
};
#ifndef TGNX_SCAN_T
#define TGNX_SCAN_T TGN_SCAN_THREADS  // train-step scan workgroup size (experiments)
#endif
#ifndef TGNX_MD_CAP200
#define TGNX_MD_CAP200 512  // grid cap of the step's M x D GEMMs (dz0, dX_enc) per 200 events of the rank's batch (env
                            // TGNX_MD_CAP200): 7 column tiles at D = 100, ~30 row tiles at B = 200 (A/B 0.0966 vs 0.0971 ms with 1024)
#endif
#ifndef TGNX_PLANS_IN_PRED
#define TGNX_PLANS_IN_PRED 4  // parity-set steps whose plans have 2..N partitions: the plans in the predictor launch (0: never; DP floor A/B at world 2 / 4 / 8: N = 4 0.1034 / 0.1078 / 0.1283 ms, 16 0.1040 / 0.1087 / 0.1328, 0 0.1039 / 0.1176 / 0.1285)
#endif
#ifndef TGNX_SCAN_AT
#define TGNX_SCAN_AT 7  // parity step: the launch the next batch's scan rides in (7: dW_gru; 6: dz0, 0.1005 vs 0.0965 ms)
#endif

__global__ void __launch_bounds__(256) tgn_update(Ctx c, int nmem, int nst, int mem_mode, const int64_t* list,
                                                  const int* list_cnt, int n_host, int64_t base) {
  update_body(c, blockIdx.x, nmem, nst, mem_mode, list, list_cnt, n_host, base);
}

// the message-store half of update_state, riding in the launch before the fixup (dW_gru ‖ dX_enc):
// nothing after tgn_agg_emit reads the stores
struct StoreJob {
  Ctx c;
  int nst;
  __device__ void operator()(int bid, float*) const { update_body(c, bid, 0, nst, 0, nullptr, nullptr, 0, 0); }
};
// One block in the same launch: copies what the fixup reads of the step descriptor (ctl words, counts,
// update list) for fixup_view — the pipelined step's next-batch scan runs inside the fixup launch and
// rewrites them — then advances the resident step counters (what tgnn_advance did at the start of the
// step; after this launch only the next batch's scan reads them).
// noadv (tgnx_tgn_train_step_pp): the counters advance in the fixup launch instead (the next batch's scan
// rides in this launch and reads them)
__device__ __forceinline__ void advance_counters(int64_t* ctl) {
  ctl[TGNX_CTL_GEN] += 1;
  ctl[TGNX_CTL_NB] += 1;
  ctl[TGNX_CTL_STEP_B] = ctl[TGNX_CTL_B];
  if (ctl[TGNX_CTL_B] > 0) ctl[TGNX_CTL_ADAM_T] += 1;
}
struct SnapJob {
  Ctx c;
  int noadv;
  __device__ void operator()(int, float*) const {
    const int tid = threadIdx.x, U = min(c.cnt[CNT_U], c.Ucap);
    for (int i = tid; i < TGNX_CTL_WORDS; i += blockDim.x) c.snap_ctl[i] = c.ctl[i];
    for (int i = tid; i < CNT_WORDS; i += blockDim.x) c.snap_cnt[i] = c.cnt[i];
    for (int i = tid; i < U; i += blockDim.x) {
      c.snap_upd[i] = c.upd[i];
      c.snap_upd_loc[i] = c.upd_loc[i];
    }
    if (!c.adv || noadv) return;  // (block-uniform)
    __syncthreads();
    if (tid == 0) advance_counters(c.ctl);
  }
};
// the fixup launch's Ctx: SnapJob's copies in place of the live descriptor
static inline Ctx fixup_view(const Ctx& c) {
  Ctx f = c;
  f.ctl = c.snap_ctl;
  f.cnt = c.snap_cnt;
  f.upd = c.snap_upd;
  f.upd_loc = c.snap_upd_loc;
  if (f.adf.p) f.adf.ctl = c.snap_ctl;
  return f;
}
// the next batch's scan as extra workgroups of the dW_cell / dX_enc launch (tgnx_tgn_train_step_pp): into the
// other parity's set (c), batch one past the counters (they advance in the fixup launch), no descriptor
// write (the fixup launch writes it)
// (blocks: the walk (role 0) and the 2 pplan plan roles, or the walk alone when the plans ride in the
// predictor launch: large global batches, tgn_pred_train's plan blocks)
struct ScanJob {
  Ctx c;
  __device__ void operator()(int bid, float* smem) const {
    scan_body<true, NoCheckpoint, 8 * 256, 8>(c, bid, reinterpret_cast<unsigned char*>(smem), NoCheckpoint{}, 1, false);
  }
};
// tail blocks of the train step's fixup launch: [0, nscan) the next batch's scan (pipelined steps whose
// scan fits the launch's LDS and 256-thread workgroups, scan_folds; `nxt` = the live Ctx), then the
// Δt-encoding reduction (nte blocks), then the memory / last_update half of update_state (nmem blocks;
// nothing in the fixup reads memory).  te.c is the fixup's view (fixup_view).
// wdesc (tgnx_tgn_train_step_pp, whose next batch was scanned earlier in the step): the first Δt block also
// advances the step counters and writes the next batch's descriptor into the live ctl (nothing in this
// launch reads them: te.c is the snapshot)
struct TrainTail {
  TeReduceTail te;
  Ctx nxt;
  int nscan, nte, nmem, wdesc;
  __device__ __forceinline__ void operator()(int bid, float* smem) const {
    if (bid < nscan) scan_body<true, NoCheckpoint, 512>(nxt, bid, reinterpret_cast<unsigned char*>(smem), NoCheckpoint{}, 0, true);
    else if ((bid -= nscan) < nte) {
      if (wdesc && bid == 0 && threadIdx.x == 0) {  // (te.c reads the snapshot: nothing here reads these words)
        advance_counters(nxt.ctl);
        write_desc(nxt, res_desc(nxt, 0));
      }
      te(bid);
    }
    else update_body(te.c, bid - nte, nmem, 0, 0, te.c.upd, te.c.cnt + CNT_U, 0, 0);
  }
};

// data parallel: the exchanged memory rows of every rank -> memory / last_update (wave per row); the
// rows are zeroed after use (the next step's exchange sums every rank's slot into them)
__device__ void apply_rows_body(float* mem, int64_t* lu, float* rows, int64_t nrows, int D, int64_t N, int bid,
                                int nb) {
  const int lane = threadIdx.x & 63, RW = TGNX_TGN_ROW(D);
  for (int64_t u = bid * 4 + (threadIdx.x >> 6); u < nrows; u += (int64_t)nb * 4) {
    float* row = rows + u * RW;
    const float h0 = row[0], h1 = row[1], h2 = row[2], h3 = row[3];
    const int64_t v = (int64_t)h0;
    const bool ok = h0 >= 0.f && v < N;
    for (int k = lane; k < D; k += 64) {
      if (ok) mem[v * D + k] = row[4 + k];
      row[4 + k] = 0.f;
    }
    if (lane < 4) row[lane] = 0.f;
    if (ok && lane == 0)
      lu[v] = (int64_t)((uint64_t)(uint32_t)h1 | ((uint64_t)(uint32_t)h2 << 24) | ((uint64_t)(uint32_t)h3 << 48));
  }
}
__global__ void __launch_bounds__(256) tgn_apply_rows(float* mem, int64_t* lu, float* rows, int64_t nrows, int D,
                                                      int64_t N) {
  apply_rows_body(mem, lu, rows, nrows, D, N, blockIdx.x, gridDim.x);
}
}  // namespace tgn
}  // namespace tgnx

// ================================================================== host side
namespace tgnx {
namespace tgn {

__global__ void tgn_reset_kernel(float* mem, int64_t nm, int64_t* lu, int64_t* st, int64_t N) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < nm; x += (int64_t)gridDim.x * blockDim.x) mem[x] = 0.f;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < N; x += (int64_t)gridDim.x * blockDim.x) {
    lu[x] = 0;
    st[4 * x] = st[4 * x + 1] = st[4 * x + 2] = st[4 * x + 3] = 0;
  }
}
__global__ void tgn_clear_store(int64_t* st, int64_t N) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < N; x += (int64_t)gridDim.x * blockDim.x)
    st[4 * x + 1] = st[4 * x + 3] = 0;
}

// eval scoring: workgroup per event, threads over its [pos, negatives] candidates:
// s = sigmoid(lin_final(relu(Hs[src] + Hd[cand]))) (Hs / Hd = lin_src / lin_dst of the centres),
// then the TGB rank rule: rank = 0.5 (#neg > pos + #neg >= pos) + 1.
__global__ void __launch_bounds__(256) tgn_score(Ctx c) {
  __shared__ float hs[TDMAX], wf[TDMAX];
  __shared__ float spos;
  __shared__ int cnt2[2];
  const int B = (int)c.ctl[TGNX_CTL_B];
  const int i = blockIdx.x;
  if (B == 0 || i >= B || c.ctl[TGNX_CTL_ERR] != 0) return;
  const int D = c.D, Kn = c.Kn, tid = threadIdx.x;
  const int64_t start = c.ctl[TGNX_CTL_BATCH_START];
  const int cs = root_row(c, c.ev_src[start + i]);
  for (int k = tid; k < D; k += blockDim.x) {
    hs[k] = c.Hs[(int64_t)cs * D + k];
    wf[k] = c.params[c.L.lfw + k];
  }
  if (tid == 0) cnt2[0] = cnt2[1] = 0;
  __syncthreads();
  const float bf = c.params[c.L.lfb];
  auto score = [&](int64_t node) {
    const float* hd = c.Hd + (int64_t)root_row(c, node) * D;
    float a = 0.f;
    for (int k = 0; k < D; ++k) a += wf[k] * fmaxf(hs[k] + hd[k], 0.f);
    return sigm(a + bf);
  };
  if (tid == 0) {
    spos = score(c.ev_dst[start + i]);
    c.out_pos[i] = spos;
  }
  __syncthreads();
  const float sp = spos;
  int opt = 0, pes = 0;
  for (int q = tid; q < Kn; q += blockDim.x) {
    const float s = score(c.neg[(start + i) * Kn + q]);
    c.out_neg[(int64_t)i * Kn + q] = s;
    opt += s > sp;
    pes += s >= sp;
  }
  atomicAdd(&cnt2[0], opt);
  atomicAdd(&cnt2[1], pes);
  __syncthreads();
  if (tid == 0) c.mrr[i] = 1.0 / (0.5 * ((double)cnt2[0] + (double)cnt2[1]) + 1.0);
}

static size_t carve(size_t& off, size_t bytes) {
  size_t o = off;
  off += (bytes + 255) & ~size_t(255);
  return o;
}
struct Caps {
  int B, Kn, Qtr, Qcap, Rtr, Rcap, Mtr, Mcap, Etr, Ecap, Ucap, Qm, D, d, HC;
  int cell, G;  // memory updater (0 GRU, 1 RNN) and its GEMM columns per unit (4: r, z, n_in, n_hid; 1)
  int layers, R1tr, R1cap, E1tr, E1cap;  // 2 hops: root level (R*/E*/M* above: the outer sample)
  int64_t N;
};
static int cfg_layers(const tgnx_tgn_config* cfg) { return cfg->layers == 2 ? 2 : 1; }
static Caps make_caps(const tgnx_tgn_config* cfg) {
  Caps k;
  k.N = cfg->num_nodes;
  k.B = cfg->max_batch;
  k.Kn = cfg->max_neg < 1 ? 1 : cfg->max_neg;
  k.D = cfg->mem_dim;
  k.d = cfg->msg_dim;
  k.HC = k.D;
  k.Qm = 3 * k.D + k.d;
  const int K = cfg->ring;
  auto cap = [&](int64_t x) { return (int)(x < k.N ? x : k.N); };
  k.Qtr = 3 * k.B;
  k.Qcap = k.B * (2 + k.Kn);
  if (k.Qcap < k.Qtr) k.Qcap = k.Qtr;
  k.layers = cfg_layers(cfg);
  k.cell = cfg->updater;
  k.G = k.cell ? 1 : 4;
  k.R1tr = cap(k.Qtr);
  k.R1cap = cap(k.Qcap);
  k.Rtr = k.layers == 2 ? cap((int64_t)k.R1tr * (K + 1)) : k.R1tr;
  k.Rcap = k.layers == 2 ? cap((int64_t)k.R1cap * (K + 1)) : k.R1cap;
  k.Mtr = cap((int64_t)k.Rtr * (K + 1));
  k.Mcap = cap((int64_t)k.Rcap * (K + 1));
  k.Etr = k.Rtr * K;
  k.Ecap = k.Rcap * K;
  k.E1tr = k.layers == 2 ? k.R1tr * K : 0;
  k.E1cap = k.layers == 2 ? k.R1cap * K : 0;
  k.Ucap = cap(2 * (int64_t)k.B);
  return k;
}
// split count of a long-K weight-gradient GEMM: ~2k rows of K per split (2-hop edge sets are ~10x the
// 1-hop ones), at least 8
static int ksplit(int K, int smin) { return std::max(smin, std::min(64, K / 2048)); }
// minimum split counts of the deferred weight-gradient GEMMs (their partials make an HBM round trip through
// the fixup launch: fewer splits, less traffic, longer K chains per workgroup)
#ifndef TGNX_S_WE
#define TGNX_S_WE 8
#endif
#ifndef TGNX_S_WP
#define TGNX_S_WP 4
#endif
#ifndef TGNX_S_WG
#define TGNX_S_WG 2  // (runtime-capped: 3 at the wiki shape; A/B 0.1022 vs 0.1027 ms with 4, and 25 % fewer partials)
#endif
#ifndef TGNX_S_LP
#define TGNX_S_LP 10  // (one 64-deep chunk per split at B = 200: A/B 0.1010 vs 0.1022 ms with 5; dW_edge 16 and dW_proj 8 splits: ±0)
#endif
#ifndef TGNX_DWE_SMAX
#define TGNX_DWE_SMAX 64  // (experiments: caps on the split counts of dW_edge / dW_gru)
#endif
#ifndef TGNX_DWG_SMAX
#define TGNX_DWG_SMAX 2  // (dW_gru split-K: same-box A/B 0.0965 vs 0.0970 ms with the 3 splits of the K / 2048 rule, a third fewer partials)
#endif
// the deferred (split-K) weight-gradient GEMMs of a train step
static GemmShape shp_dWe(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(k.HC, k.D + k.d, k.Etr, nullptr, nullptr, cnt ? cnt + CNT_E : nullptr, std::min(TGNX_DWE_SMAX, ksplit(k.Etr, TGNX_S_WE))); }
static GemmShape shp_dWp(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(4 * k.HC, k.D + 1, k.Mtr, nullptr, nullptr, cnt ? cnt + CNT_M : nullptr, ksplit(k.Mtr, TGNX_S_WP)); }
// 2 hops: conv2's projections (K = outer centres) and lin_edge (K = root edges)
static GemmShape shp_dWp2(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(4 * k.HC, k.D + 1, k.Rtr, nullptr, nullptr, cnt ? cnt + CNT_R : nullptr, ksplit(k.Rtr, 4)); }
static GemmShape shp_dWe2(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(k.HC, k.D + k.d, k.E1tr, nullptr, nullptr, cnt ? cnt + CNT_E1 : nullptr, ksplit(k.E1tr, 8)); }
static GemmShape shp_dWlp(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(2 * k.D, k.D, 3 * k.B, nullptr, nullptr, cnt ? cnt + CNT_LIST : nullptr, std::max(TGNX_S_LP, std::min(64, (3 * k.B + 63) / 64))); }
static GemmShape shp_dWg(const Caps& k, const int* cnt) { return gemm_shape_split<GW>(k.G * k.D, k.Qm + k.D + 1, k.Mtr, nullptr, nullptr, cnt ? cnt + CNT_M : nullptr, std::min(TGNX_DWG_SMAX, ksplit(k.Mtr, TGNX_S_WG))); }
struct WsLay {
  size_t cb, nb, cbs, nbs, cl, nl, rbs, rl, kval, cnt, cent, cent_loc, ceoff, crank, upd_loc, nid, upd, e_j, e_c, kj, kx, ke, e_id, e_t, X, trel, lu, xw, gates, Z0, P,
      Ep, alpha, alk, Qo, Zc, Hp, evs, evr, evq, evj, cevq, cevj, Hs, Hd, dZc, dP, dE, dKV, dG, tgp, encE, s0m, s1m, pA, pB, pC, pD, rkeys, rruns, skeys, sruns, pcnt,
      snap, rb, x2r, cent1, r_x2, ceoff1, e1_j, e1_e2, e1_id, P2, Ep2, alpha1, Zr, dZr, dP2, dE2, pE, pF,
      uX, uZ, uG, ulu, uxw, utrel, total;
  int tgp_rows, tgp_e1;
  // the scan's per-batch outputs of the second parity (tgnx_tgn_train_step_pp: a step reads its parity's
  // set while the next batch's scan writes the other)
  size_t cnt2, cent2, cent_loc2, ceoff2, crank2, upd_loc2, nid2, upd2, rkeys2, rruns2, skeys2, sruns2, pcnt2;
  size_t x2r2, cent12, r_x22, ceoff12;  // (2 hops)
};
static WsLay make_ws(const tgnx_tgn_config* cfg, const Caps& k) {
  WsLay W;
  size_t off = 0;
  const int64_t words = (k.N + 31) / 32 + 1;
  const int D = k.D, HC = k.HC;
  W.cb = carve(off, words * 4);
  W.nb = carve(off, words * 4);
  const int64_t swords = (words + 31) / 32 + 1;
  W.cbs = carve(off, swords * 4);
  W.nbs = carve(off, swords * 4);
  W.cl = carve(off, words * 4);
  W.nl = carve(off, words * 4);
  W.kval = carve(off, (size_t)k.N * 4);
  W.cnt = carve(off, CNT_WORDS * 4);
  W.cent = carve(off, (size_t)k.Rcap * 8);
  W.cent_loc = carve(off, (size_t)k.Rcap * 4);
  W.ceoff = carve(off, (size_t)(k.Rcap + 1) * 4);
  W.crank = carve(off, (size_t)k.Mcap * 4);
  W.upd_loc = carve(off, (size_t)k.Ucap * 4);
  W.nid = carve(off, (size_t)k.Mcap * 8);
  W.upd = carve(off, (size_t)k.Ucap * 8);
  W.e_j = carve(off, (size_t)k.Ecap * 4);
  W.e_c = carve(off, (size_t)k.Ecap * 4);
  W.kj = carve(off, (size_t)k.Etr * 4);
  W.kx = carve(off, (size_t)k.Etr * 4);
  W.ke = carve(off, (size_t)k.Etr * 4);
  W.e_id = carve(off, (size_t)k.Ecap * 8);
  W.e_t = carve(off, (size_t)k.Ecap * 4);
  W.X = carve(off, (size_t)k.Mcap * k.Qm * 4);
  W.trel = carve(off, (size_t)k.Mcap * 4);
  W.lu = carve(off, (size_t)k.Mcap * 4);
  W.xw = carve(off, (size_t)k.Mcap * 8);
  W.gates = carve(off, (size_t)k.Mcap * 4 * D * 4);
  W.Hp = carve(off, (size_t)k.Mcap * D * 4);
  W.Z0 = carve(off, (size_t)k.Mcap * D * 4);
  W.P = carve(off, (size_t)k.Mcap * 4 * HC * 4);
  W.Ep = carve(off, (size_t)k.Ecap * HC * 4);
  W.alpha = carve(off, (size_t)k.Etr * TH * 4);
  W.alk = carve(off, (size_t)k.Etr * TH * 4);
  W.Qo = carve(off, (size_t)k.Rtr * 2 * HC * 4);
  W.Zc = carve(off, (size_t)k.Rcap * HC * 4);
  W.evs = carve(off, (size_t)k.B * evs_stride(D) * 4);
  W.evr = carve(off, (size_t)k.B * 3 * 4);
  W.evq = carve(off, (size_t)k.B * 3 * 16);
  W.evj = carve(off, (size_t)k.B * 3 * 16 * 4);
  W.cevq = carve(off, (size_t)k.Rcap * 16);
  W.cevj = carve(off, (size_t)k.Rcap * 16 * 4);
  W.Hs = carve(off, (size_t)k.Rcap * D * 4);
  W.Hd = carve(off, (size_t)k.Rcap * D * 4);
  W.dZc = carve(off, (size_t)k.Rtr * HC * 4 * (k.layers == 2 ? 1 : TGNX_DZC_REP));
  W.dP = carve(off, (size_t)k.Mtr * 4 * HC * 4);
  W.dE = carve(off, (size_t)k.Etr * HC * 4);
  W.dKV = carve(off, (size_t)(k.Etr > k.E1tr ? k.Etr : k.E1tr) * 2 * HC * 4);  // both levels (used in turn)
  W.dG = carve(off, (size_t)k.Mtr * 4 * D * 4);
  W.tgp_e1 = (k.Etr + G32::TM - 1) / G32::TM + (k.Mtr + G32::TM - 1) / G32::TM;
  W.tgp_rows = W.tgp_e1 + (k.E1tr + G32::TM - 1) / G32::TM;
  W.tgp = carve(off, (size_t)W.tgp_rows * 2 * D * 4);
  W.encE = carve(off, (size_t)k.Ecap * (D + k.d) * 4);  // train: [cos enc | msg] rows; eval: cos rows (stride D)
  W.s0m = carve(off, (size_t)k.Mtr * D * 4);
  W.s1m = carve(off, (size_t)k.Mtr * D * 4);
  W.pA = carve(off, gemm_partial_floats(shp_dWe(k, nullptr)) * 4);
  W.pB = carve(off, gemm_partial_floats(shp_dWp(k, nullptr)) * 4);
  W.pC = carve(off, gemm_partial_floats(shp_dWlp(k, nullptr)) * 4);
  W.pD = carve(off, gemm_partial_floats(shp_dWg(k, nullptr)) * 4);
  const int n2 = 2 * k.B;
  W.rkeys = carve(off, (size_t)n2 * 8);
  W.rruns = carve(off, (size_t)(n2 + 2 + TGNX_PLAN_PMAX) * 4);
  W.skeys = carve(off, (size_t)n2 * 8);
  W.sruns = carve(off, (size_t)(n2 + 2 + TGNX_PLAN_PMAX) * 4);
  W.pcnt = carve(off, (size_t)4 * TGNX_PLAN_PMAX * 4);
  W.snap = carve(off, (size_t)TGNX_CTL_WORDS * 8 + CNT_WORDS * 4 + (size_t)k.Ucap * 12);
  const bool two = k.layers == 2;
  const size_t R1 = two ? k.R1cap : 0, E1 = k.E1cap, R2 = two ? k.Rcap : 0;
  W.rb = carve(off, two ? words * 4 : 0);
  W.rbs = carve(off, two ? swords * 4 : 0);
  W.rl = carve(off, two ? words * 4 : 0);
  W.x2r = carve(off, R2 * 4);
  W.cent1 = carve(off, R1 * 8);
  W.r_x2 = carve(off, R1 * 4);
  W.ceoff1 = carve(off, (R1 + 1) * 4);
  W.e1_j = carve(off, E1 * 4);
  W.e1_e2 = carve(off, E1 * 4);
  W.e1_id = carve(off, E1 * 8);
  W.P2 = carve(off, R2 * 4 * HC * 4);
  W.Ep2 = carve(off, E1 * HC * 4);
  W.alpha1 = carve(off, (size_t)k.E1tr * TH * 4);
  W.Zr = carve(off, R1 * HC * 4);
  W.dZr = carve(off, (two ? (size_t)k.R1tr : 0) * HC * 4);  // (one copy: 4 copies measured slower, 0.2770 -> 0.2942 ms)
  W.dP2 = carve(off, (two ? (size_t)k.Rtr : 0) * 4 * HC * 4);
  W.dE2 = carve(off, (size_t)k.E1tr * HC * 4);
  W.pE = carve(off, two ? gemm_partial_floats(shp_dWp2(k, nullptr)) * 4 : 0);
  W.pF = carve(off, two ? gemm_partial_floats(shp_dWe2(k, nullptr)) * 4 : 0);
  // DyRep embedding messages: the update list's own aggregation / updater rows (train)
  const size_t U = cfg->emb_in_msg ? (size_t)k.Ucap : 0;
  W.uX = carve(off, U * k.Qm * 4);
  W.uZ = carve(off, U * D * 4);
  W.uG = carve(off, U * 4 * D * 4);
  W.ulu = carve(off, U * 4);
  W.uxw = carve(off, U * 8);
  W.utrel = carve(off, U * 4);
  W.cnt2 = carve(off, CNT_WORDS * 4);
  W.cent2 = carve(off, (size_t)k.Rcap * 8);
  W.cent_loc2 = carve(off, (size_t)k.Rcap * 4);
  W.ceoff2 = carve(off, (size_t)(k.Rcap + 1) * 4);
  W.crank2 = carve(off, (size_t)k.Mcap * 4);
  W.upd_loc2 = carve(off, (size_t)k.Ucap * 4);
  W.nid2 = carve(off, (size_t)k.Mcap * 8);
  W.upd2 = carve(off, (size_t)k.Ucap * 8);
  W.rkeys2 = carve(off, (size_t)n2 * 8);
  W.rruns2 = carve(off, (size_t)(n2 + 2 + TGNX_PLAN_PMAX) * 4);
  W.skeys2 = carve(off, (size_t)n2 * 8);
  W.sruns2 = carve(off, (size_t)(n2 + 2 + TGNX_PLAN_PMAX) * 4);
  W.pcnt2 = carve(off, (size_t)4 * TGNX_PLAN_PMAX * 4);
  W.x2r2 = carve(off, R2 * 4);
  W.cent12 = carve(off, R1 * 8);
  W.r_x22 = carve(off, R1 * 4);
  W.ceoff12 = carve(off, two ? (R1 + 1) * 4 : 0);
  W.total = off;
  return W;
}

static int check_cfg(const tgnx_tgn_config* cfg) {
  TGNX_CHECK_ARG(cfg, "tgn: null config");
  TGNX_CHECK_ARG(cfg->heads == TH, "tgn: heads must be %d (emb_module.py:66), got %d", TH, cfg->heads);
  TGNX_CHECK_ARG(cfg->mem_dim > 0 && cfg->mem_dim <= TDMAX && cfg->mem_dim % TH == 0,
                 "tgn: mem_dim must be even and <= %d", TDMAX);
  TGNX_CHECK_ARG(cfg->msg_dim >= 0 && cfg->msg_dim <= 4096, "tgn: bad msg_dim");
  TGNX_CHECK_ARG(cfg->ring > 0 && cfg->ring <= KMAX, "tgn: ring size must be in [1, %d]", KMAX);
  TGNX_CHECK_ARG(cfg->max_batch > 0 && cfg->max_batch <= 2048, "tgn: max_batch must be in [1, 2048]");
  TGNX_CHECK_ARG(cfg->num_nodes > 0 && cfg->num_nodes < (1ll << 31), "tgn: bad num_nodes");
  TGNX_CHECK_ARG(cfg->num_events > 0, "tgn: bad num_events");
  TGNX_CHECK_ARG(cfg->aggr == 0 || cfg->aggr == 1, "tgn: aggr must be 0 (last) or 1 (mean)");
  TGNX_CHECK_ARG(cfg->dropout >= 0.f && cfg->dropout < 1.f, "tgn: bad dropout");
  TGNX_CHECK_ARG(cfg->layers >= 0 && cfg->layers <= 2, "tgn: layers must be 1 or 2, got %d", cfg->layers);
  TGNX_CHECK_ARG(cfg->updater == 0 || cfg->updater == 1, "tgn: updater must be 0 (GRUCell) or 1 (RNNCell)");
  TGNX_CHECK_ARG(cfg->emb_in_msg >= 0 && cfg->emb_in_msg <= 3,
                 "tgn: emb_in_msg is bit 0 use_src_emb_in_msg | bit 1 use_dst_emb_in_msg");
  TGNX_CHECK_ARG(cfg->emb_in_msg == 0 || cfg->layers <= 1,
                 "tgn: DyRep embedding messages (emb_in_msg) are built for the 1-hop embedding (layers = 1)");
  return TGNX_OK;
}

static int make_ctx(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* b, int Kn, Ctx& c, Caps& k, WsLay& W) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(b && b->ctl && b->ws && b->params && b->memory && b->last_update && b->store && b->node_gen &&
                     b->nbr && b->eid && b->rt && b->assoc && b->ev_src && b->ev_dst && b->ev_t && b->ev_msg,
                 "tgn: null buffer");
  k = make_caps(cfg);
  W = make_ws(cfg, k);
  memset(&c, 0, sizeof(c));
  c.N = cfg->num_nodes;
  c.nev = cfg->num_events;
  c.words = (c.N + 31) / 32 + 1;
  c.K = cfg->ring;
  c.D = cfg->mem_dim;
  c.d = cfg->msg_dim;
  c.Qm = k.Qm;
  c.HC = k.HC;
  c.C = k.HC / TH;
  c.aggr = cfg->aggr;
  c.Kn = Kn;
  c.p = cfg->dropout;
  c.inv_keep = 1.0f / (1.0f - cfg->dropout);
  c.lr = cfg->lr;
  c.b1 = cfg->beta1;
  c.b2 = cfg->beta2;
  c.eps = cfg->eps;
  c.ev_src = b->ev_src;
  c.ev_dst = b->ev_dst;
  c.ev_t = b->ev_t;
  c.ev_msg = b->ev_msg;
  c.neg = b->neg;
  c.dst_nodes = b->dst_nodes;
  c.n_dst = b->n_dst;
  c.nbr = b->nbr;
  c.eid = b->eid;
  c.rt = b->rt;
  c.assoc = b->assoc;
  c.mem = b->memory;
  c.lu_buf = b->last_update;
  c.st = b->store;
  c.arena = b->store + 4 * c.N;
  c.node_gen = b->node_gen;
  c.params = b->params;
  c.grads = b->grads;
  c.am = b->adam_m;
  c.av = b->adam_v;
  c.ctl = b->ctl;
  c.out_pos = b->out_pos;
  c.out_neg = b->out_neg;
  c.mrr = b->mrr;
  c.out_ev = b->out_ev;
  c.xrows = b->xrows;
  c.xcap = b->xrows ? (int)std::min<int64_t>(b->xcap, 1 << 30) : 0;
  TGNX_CHECK_ARG(!b->xrows || b->xcap > 0, "tgn: xrows without xcap");
  TGNX_CHECK_ARG(!b->xrows || cfg->num_nodes < (1ll << 24), "tgn: data-parallel row exchange needs num_nodes < 2^24");
  char* ws = reinterpret_cast<char*>(b->ws);
  c.cb = reinterpret_cast<uint32_t*>(ws + W.cb);
  c.nb = reinterpret_cast<uint32_t*>(ws + W.nb);
  c.cbs = reinterpret_cast<uint32_t*>(ws + W.cbs);
  c.nbs = reinterpret_cast<uint32_t*>(ws + W.nbs);
  c.cl = reinterpret_cast<int*>(ws + W.cl);
  c.nl = reinterpret_cast<int*>(ws + W.nl);
  c.kval = reinterpret_cast<int*>(ws + W.kval);
  c.cnt = reinterpret_cast<int*>(ws + W.cnt);
  c.cent = reinterpret_cast<int64_t*>(ws + W.cent);
  c.cent_loc = reinterpret_cast<int*>(ws + W.cent_loc);
  c.ceoff = reinterpret_cast<int*>(ws + W.ceoff);
  c.crank = reinterpret_cast<int*>(ws + W.crank);
  c.upd_loc = reinterpret_cast<int*>(ws + W.upd_loc);
  c.nid = reinterpret_cast<int64_t*>(ws + W.nid);
  c.upd = reinterpret_cast<int64_t*>(ws + W.upd);
  c.e_j = reinterpret_cast<int*>(ws + W.e_j);
  c.e_c = reinterpret_cast<int*>(ws + W.e_c);
  c.kj = reinterpret_cast<int*>(ws + W.kj);
  c.kx = reinterpret_cast<int*>(ws + W.kx);
  c.ke = reinterpret_cast<int*>(ws + W.ke);
  c.e_id = reinterpret_cast<int64_t*>(ws + W.e_id);
  c.e_t = reinterpret_cast<float*>(ws + W.e_t);
  c.X = reinterpret_cast<float*>(ws + W.X);
  c.trel = reinterpret_cast<float*>(ws + W.trel);
  c.lu = reinterpret_cast<float*>(ws + W.lu);
  c.xw = reinterpret_cast<int64_t*>(ws + W.xw);
  c.gates = reinterpret_cast<float*>(ws + W.gates);
  c.Hp = reinterpret_cast<float*>(ws + W.Hp);
  c.Z0 = reinterpret_cast<float*>(ws + W.Z0);
  c.P = reinterpret_cast<float*>(ws + W.P);
  c.Ep = reinterpret_cast<float*>(ws + W.Ep);
  c.alpha = reinterpret_cast<float*>(ws + W.alpha);
  c.alk = reinterpret_cast<float*>(ws + W.alk);
  c.Qo = reinterpret_cast<float*>(ws + W.Qo);
  c.Zc = reinterpret_cast<float*>(ws + W.Zc);
  c.evs = reinterpret_cast<float*>(ws + W.evs);
  c.evr = reinterpret_cast<int*>(ws + W.evr);
  c.evq = k.layers == 2 ? nullptr : reinterpret_cast<int4*>(ws + W.evq);
  c.evj = k.layers == 2 || cfg->ring > 16 ? nullptr : reinterpret_cast<int*>(ws + W.evj);
  c.cevq = c.evj ? reinterpret_cast<int4*>(ws + W.cevq) : nullptr;
  c.cevj = c.evj ? reinterpret_cast<int*>(ws + W.cevj) : nullptr;
  c.Hs = reinterpret_cast<float*>(ws + W.Hs);
  c.Hd = reinterpret_cast<float*>(ws + W.Hd);
  c.dZc = reinterpret_cast<float*>(ws + W.dZc);
  c.dzrep = k.layers == 2 ? 1 : TGNX_DZC_REP;
  c.dzstride = (int64_t)k.Rtr * k.HC;
  c.dzrep1 = 1;
  c.dzstride1 = (int64_t)k.R1tr * k.HC;
  c.dP = reinterpret_cast<float*>(ws + W.dP);
  c.dE = reinterpret_cast<float*>(ws + W.dE);
  c.dKV = reinterpret_cast<float*>(ws + W.dKV);
  c.dG = reinterpret_cast<float*>(ws + W.dG);
  c.tgp = reinterpret_cast<float*>(ws + W.tgp);
  c.encE = reinterpret_cast<float*>(ws + W.encE);
  c.s0m = reinterpret_cast<float*>(ws + W.s0m);
  c.s1m = reinterpret_cast<float*>(ws + W.s1m);
  c.pA = reinterpret_cast<float*>(ws + W.pA);
  c.pB = reinterpret_cast<float*>(ws + W.pB);
  c.pC = reinterpret_cast<float*>(ws + W.pC);
  c.pD = reinterpret_cast<float*>(ws + W.pD);
  c.rkeys = reinterpret_cast<uint64_t*>(ws + W.rkeys);
  c.rruns = reinterpret_cast<int*>(ws + W.rruns);
  c.skeys = reinterpret_cast<uint64_t*>(ws + W.skeys);
  c.sruns = reinterpret_cast<int*>(ws + W.sruns);
  c.rpc = reinterpret_cast<int*>(ws + W.pcnt);
  c.rpo = c.rpc + TGNX_PLAN_PMAX;
  c.spc = c.rpo + TGNX_PLAN_PMAX;
  c.spo = c.spc + TGNX_PLAN_PMAX;
  c.snap_ctl = reinterpret_cast<int64_t*>(ws + W.snap);
  c.snap_upd = c.snap_ctl + TGNX_CTL_WORDS;
  c.snap_cnt = reinterpret_cast<int*>(c.snap_upd + k.Ucap);
  c.snap_upd_loc = c.snap_cnt + CNT_WORDS;
  c.errw = b->ctl + TGNX_CTL_ERR;
  c.pplan = plan_parts(k.B);
  c.Bmax = k.B;
  c.Bplan = k.B;
  c.Qcap = k.Qcap;
  c.Rcap = k.Rcap;
  c.Mcap = k.Mcap;
  c.Ecap = k.Ecap;
  c.ktr = std::max<int64_t>(1, k.Etr);
  c.Ucap = k.Ucap;
  c.tgp_rows = W.tgp_rows;
  c.L = make_lay(c.D, c.d, k.layers, k.cell);
  c.layers = k.layers;
  c.rsel = CNT_R;
  c.ccap = k.Rcap;
  c.att_salt = 7;
  c.emb = cfg->emb_in_msg;
  c.zemb = c.Zc;
  if (k.layers == 2) {
    c.rb = reinterpret_cast<uint32_t*>(ws + W.rb);
    c.rbs = reinterpret_cast<uint32_t*>(ws + W.rbs);
    c.rl = reinterpret_cast<int*>(ws + W.rl);
    c.x2r = reinterpret_cast<int*>(ws + W.x2r);
    c.cent1 = reinterpret_cast<int64_t*>(ws + W.cent1);
    c.r_x2 = reinterpret_cast<int*>(ws + W.r_x2);
    c.ceoff1 = reinterpret_cast<int*>(ws + W.ceoff1);
    c.e1_j = reinterpret_cast<int*>(ws + W.e1_j);
    c.e1_e2 = reinterpret_cast<int*>(ws + W.e1_e2);
    c.e1_id = reinterpret_cast<int64_t*>(ws + W.e1_id);
    c.P2 = reinterpret_cast<float*>(ws + W.P2);
    c.Ep2 = reinterpret_cast<float*>(ws + W.Ep2);
    c.alpha1 = reinterpret_cast<float*>(ws + W.alpha1);
    c.Zr = reinterpret_cast<float*>(ws + W.Zr);
    c.dZr = reinterpret_cast<float*>(ws + W.dZr);
    c.dP2 = reinterpret_cast<float*>(ws + W.dP2);
    c.dE2 = reinterpret_cast<float*>(ws + W.dE2);
    c.pE = reinterpret_cast<float*>(ws + W.pE);
    c.pF = reinterpret_cast<float*>(ws + W.pF);
    c.R1cap = k.R1cap;
    c.E1cap = k.E1cap;
    c.tgp_e1 = W.tgp_e1;
  }
  return TGNX_OK;
}

// the Ctx of scan-output set p (0: the set every other entry point uses, 1: the second parity)
static Ctx set_view(const Ctx& c, const WsLay& W, char* ws, int p) {
  Ctx v = c;
  auto at = [&](size_t a, size_t b) { return ws + (p ? b : a); };
  v.cnt = reinterpret_cast<int*>(at(W.cnt, W.cnt2));
  v.cent = reinterpret_cast<int64_t*>(at(W.cent, W.cent2));
  v.cent_loc = reinterpret_cast<int*>(at(W.cent_loc, W.cent_loc2));
  v.ceoff = reinterpret_cast<int*>(at(W.ceoff, W.ceoff2));
  v.crank = reinterpret_cast<int*>(at(W.crank, W.crank2));
  v.upd_loc = reinterpret_cast<int*>(at(W.upd_loc, W.upd_loc2));
  v.nid = reinterpret_cast<int64_t*>(at(W.nid, W.nid2));
  v.upd = reinterpret_cast<int64_t*>(at(W.upd, W.upd2));
  v.rkeys = reinterpret_cast<uint64_t*>(at(W.rkeys, W.rkeys2));
  v.rruns = reinterpret_cast<int*>(at(W.rruns, W.rruns2));
  v.skeys = reinterpret_cast<uint64_t*>(at(W.skeys, W.skeys2));
  v.sruns = reinterpret_cast<int*>(at(W.sruns, W.sruns2));
  v.rpc = reinterpret_cast<int*>(at(W.pcnt, W.pcnt2));
  v.rpo = v.rpc + TGNX_PLAN_PMAX;
  v.spc = v.rpo + TGNX_PLAN_PMAX;
  v.spo = v.spc + TGNX_PLAN_PMAX;
  if (c.x2r) {  // 2 hops: the root level's sets
    v.x2r = reinterpret_cast<int*>(at(W.x2r, W.x2r2));
    v.cent1 = reinterpret_cast<int64_t*>(at(W.cent1, W.cent12));
    v.r_x2 = reinterpret_cast<int*>(at(W.r_x2, W.r_x22));
    v.ceoff1 = reinterpret_cast<int*>(at(W.ceoff1, W.ceoff12));
  }
  return v;
}

// 2 hops: the root level as a Ctx for the attention / prediction kernels — centres = roots, node rows =
// outer centres (P2 = conv2's projections of h1), edges = the roots' ring rows, output Zr
// the DyRep embedding-message update of a train step: aggregation / updater rows of the update list in their
// own buffers (the step's GRU rows, gates and aggregated messages are still needed by its backward)
static Ctx emb_view(const Ctx& c, const WsLay& W, char* ws) {
  Ctx e = c;
  e.X = reinterpret_cast<float*>(ws + W.uX);
  e.Z0 = reinterpret_cast<float*>(ws + W.uZ);
  e.gates = reinterpret_cast<float*>(ws + W.uG);
  e.lu = reinterpret_cast<float*>(ws + W.ulu);
  e.xw = reinterpret_cast<int64_t*>(ws + W.uxw);
  e.trel = reinterpret_cast<float*>(ws + W.utrel);
  return e;
}
static Ctx root_view(const Ctx& c) {
  Ctx r = c;
  r.cent = c.cent1;
  r.cent_loc = c.r_x2;
  r.ceoff = c.ceoff1;
  r.e_j = c.e1_j;
  r.e_id = c.e1_id;
  r.P = c.P2;
  r.Ep = c.Ep2;
  r.alpha = c.alpha1;
  r.Zc = c.Zr;
  r.dZc = c.dZr;
  r.dzrep = c.dzrep1;
  r.dzstride = c.dzstride1;
  r.dP = c.dP2;
  r.dE = c.dE2;
  r.e_c = nullptr;  // (the root level's attention backward leaves its (dk, dv) sums to the k / v reduction job:
  r.alk = nullptr;  //  summing them in the attention backward measured slower, r4_kvf_root_ab.txt)
  r.Qo = nullptr;
  r.rsel = CNT_R1;
  r.ccap = c.R1cap;
  r.att_salt = 9;
  return r;
}

// tgn_agg_emit's two grid-stride parts (sampled edges, wave per (centre, ring slot); sampled nodes):
// grids sized from capacities launch mostly idle workgroups, which hold dispatch slots
// (stamps timeline, wiki shape: caps 4096 / 2048 -> 1024 / 512 took agg_emit 16.5 -> 13.9 us)
#ifndef TGNX_AGG_EDGE_CAP
#define TGNX_AGG_EDGE_CAP 1024  // (512: 0.0887 / 0.0886 vs 0.0871 / 0.0872 ms; node cap 128: +-0 — r5_agg_caps_ab.txt)
#endif
#ifndef TGNX_AGG_NODE_CAP
#define TGNX_AGG_NODE_CAP 512
#endif
// the attention backward for a ring of K and the predictor's dZc copy count (compile-time: the copies' loads batched)
using AttnBwdFn = void (*)(Ctx, int, int, int, Ctx);
#ifndef TGNX_ATTB_EB10_2HOP
#define TGNX_ATTB_EB10_2HOP 1  // 2 hops: the attention backward in 10-edge load batches for K <= 10 (0: 16-edge batches)
#endif
static AttnBwdFn attn_bwd_fn(int K, int rep, bool two = false) {
  if (rep == TGNX_DZC_REP && TGNX_DZC_REP > 1) return K <= 10 ? tgn_attn_bwd<10, TGNX_DZC_REP> : tgn_attn_bwd<ATT_EB, TGNX_DZC_REP>;
  return K <= 10 && (!two || TGNX_ATTB_EB10_2HOP) ? tgn_attn_bwd<10, 1> : tgn_attn_bwd<ATT_EB, 1>;
}
// integer knob from the environment (host, read once by the caller's static), else the build default
static inline int env_int(const char* name, int def) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : def;
}
// a GEMM grid cap that scales with the rank's batch (the runtime rows / edges do; the capacity shapes are worst cases)
static inline int cap_per200(const char* env, int per200, int B) {
  const int64_t v = (int64_t)env_int(env, per200) * std::max(B, 1) / 200;
  return (int)std::max<int64_t>(64, std::min<int64_t>(TGNX_GEMM_GRID_CAP, v));
}
static inline int gridn(int64_t n, int per, int cap = 4096) {
  int64_t g = (n + per - 1) / per;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// event workgroups of the 2-hop predictor launch: one per event (its LDS holds one workgroup per CU, so a batch of more
// events than CUs runs in dispatch rounds), or with TGNX_PRED_GROUPS = G at most G workgroups looping over the batch
// with the weights staged once (G = the CU count: comment-shaped B = 600 step 0.2380 / 0.2384 ms against 0.2359 /
// 0.2347 one per event, profiles/r6/r6i_2hop_groups_ab.txt)
static int pred_groups(int B) {
  static const int ncu = std::max(1, env_int("TGNX_PRED_GROUPS", 1 << 30));
  if (B <= ncu) return std::max(B, 1);
  const int per = (B + ncu - 1) / ncu;
  return (B + per - 1) / per;
}
// the GRU of a node list (eval update / flush): messages -> GRUCell (X, Z0 rows 0..n)
template <int CELL>
static void gru_list_c(const Ctx& c, const int64_t* list, const int* list_cnt, int n_host, int64_t base, int mcap,
                       hipStream_t s, bool emb = false) {
  using Cl = CellOps<CELL>;
  if (emb)   // DyRep embedding messages (update of src ∪ dst only)
    tgn_agg_emit<-1, true><<<gridn(mcap, 4, 2048), 256, 0, s>>>(c, 2, 0, list, list_cnt, n_host, base);
  else if (c.aggr == 0)
    tgn_agg_emit<0><<<gridn(mcap, 4, 2048), 256, 0, s>>>(c, 2, 0, list, list_cnt, n_host, base);
  else
    tgn_agg_emit<-1><<<gridn(mcap, 4, 2048), 256, 0, s>>>(c, 2, 0, list, list_cnt, n_host, base);
  const GemmShape g1 = gemm_shape<G32L>(mcap, Cl::G * c.D, c.Qm + c.D, list_cnt);
  gemm_launch<G32L>(g1, LoadGruA{c.X, c.mem, list ? list : c.nid, base, c.Qm, c.D, list ? 0 : 1}, Cl::w(c),
                    Cl::epi(c, list, base), nullptr, s);
}
// the memory update of a node list (eval update, flush): aggregation + the memory updater
static void gru_list(const Ctx& c, const Caps& k, const int64_t* list, const int* list_cnt, int n_host, int64_t base,
                     int mcap, hipStream_t s, bool emb = false) {
  if (k.cell) gru_list_c<1>(c, list, list_cnt, n_host, base, mcap, s, emb);
  else gru_list_c<0>(c, list, list_cnt, n_host, base, mcap, s, emb);
}

}  // namespace tgn
}  // namespace tgnx

using namespace tgnx;
using namespace tgnx::tgn;

extern "C" {

int tgnx_tgn_param_layout(const tgnx_tgn_config* cfg, int64_t* off) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(off, "tgnx_tgn_param_layout: null output");
  const int layers = cfg_layers(cfg);
  const Lay L = make_lay(cfg->mem_dim, cfg->msg_dim, layers, cfg->updater);
  const int64_t v[TGNX_TGN_NPARAM2] = {L.te_w, L.te_b, L.w_ih, L.w_hh, L.b_ih, L.b_hh, L.wk,  L.bk,  L.wq,  L.bq,
                                       L.wv,   L.bv,   L.we,   L.wsk,  L.bsk,  L.lsw,  L.lsb, L.ldw, L.ldb, L.lfw,
                                       L.lfb,  L.wk2,  L.bk2,  L.wq2,  L.bq2,  L.wv2,  L.bv2, L.we2, L.wsk2, L.bsk2};
  const int np = layers == 2 ? TGNX_TGN_NPARAM2 : TGNX_TGN_NPARAM;
  for (int i = 0; i < np; ++i) off[i] = v[i];
  off[np] = L.total;
  return TGNX_OK;
}

size_t tgnx_tgn_ws_bytes(const tgnx_tgn_config* cfg) {
  if (check_cfg(cfg)) return 0;
  return make_ws(cfg, make_caps(cfg)).total;
}

size_t tgnx_tgn_store_words(const tgnx_tgn_config* cfg) {
  if (check_cfg(cfg)) return 0;
  return (size_t)(4 * cfg->num_nodes + 2 * cfg->num_events);
}

size_t tgnx_tgn_plan_table_bytes(const tgnx_tgn_config* cfg, int64_t split_lo, int64_t split_hi, int64_t batch) {
  if (check_cfg(cfg) || batch <= 0 || batch > cfg->max_batch || split_hi < split_lo) return 0;
  const int64_t nb = (split_hi - split_lo + batch - 1) / batch;
  return (size_t)(64 + (nb > 0 ? nb : 1) * plan_slot_bytes(cfg->max_batch));
}

// what each plan table was built for (tgnx_tgn_plan_table), keyed by its device address: the resident parity-set
// steps index slot (batch start - split_lo) / batch with a stride sized by max_batch, so a table built for another
// split, batch or max_batch would silently hand them another batch's plans or read past the table
extern "C++" {  // (inside the C-ABI block)
namespace {
struct PlanTableKey {
  int64_t lo, hi, batch, stride;
  size_t bytes;
};
std::mutex g_ptab_mu;
std::unordered_map<const void*, PlanTableKey>& ptab_registry() {
  static std::unordered_map<const void*, PlanTableKey> m;
  return m;
}
}  // namespace
}  // extern "C++"

int tgnx_tgn_plan_table(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo, int64_t split_hi,
                        int64_t batch, void* table, size_t table_bytes, void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  TGNX_CHECK_ARG(batch > 0 && batch <= cfg->max_batch && split_lo >= 0 && split_hi >= split_lo && split_hi <= c.nev,
                 "tgnx_tgn_plan_table: bad split / batch");
  const size_t need = tgnx_tgn_plan_table_bytes(cfg, split_lo, split_hi, batch);
  TGNX_CHECK_ARG(table && table_bytes >= need && ((uintptr_t)table & 15) == 0,
                 "tgnx_tgn_plan_table: table of tgnx_tgn_plan_table_bytes(...) bytes, 16-B aligned");
  const int64_t nb = (split_hi - split_lo + batch - 1) / batch;
  // a (re)build first forgets what the table held: a failed build leaves it unknown, not valid for its old split
  tgnx_tgn_plan_table_release(table);
  if (nb > 0) {
    const size_t smem = tgn_scan_smem(k.B);
    TGNX_CHECK_ARG(hipFuncSetAttribute(reinterpret_cast<const void*>(&tgn_plan_table_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) == hipSuccess,
                   "tgnx_tgn_plan_table: dynamic LDS of %zu bytes refused", smem);
    tgn_plan_table_kernel<<<(unsigned)(nb * 2 * c.pplan), 1024, smem, as_stream(stream)>>>(
        c, reinterpret_cast<char*>(table), plan_slot_bytes(k.B), split_lo, split_hi, batch);
    TGNX_LAUNCH_CHECK("tgn_plan_table");
  }
  std::lock_guard<std::mutex> lk(g_ptab_mu);
  ptab_registry()[table] = PlanTableKey{split_lo, split_hi, batch, plan_slot_bytes(k.B), need};
  return TGNX_OK;
}

int tgnx_tgn_plan_table_release(const void* table) {
  std::lock_guard<std::mutex> lk(g_ptab_mu);
  ptab_registry().erase(table);
  return TGNX_OK;
}

int tgnx_tgn_reset_state(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf && buf->memory && buf->last_update && buf->store, "tgnx_tgn_reset_state: null buffer");
  const int64_t N = cfg->num_nodes;
  tgn_reset_kernel<<<gridn(N * cfg->mem_dim, 256), 256, 0, as_stream(stream)>>>(buf->memory, N * cfg->mem_dim,
                                                                                 buf->last_update, buf->store, N);
  TGNX_LAUNCH_CHECK("tgn_reset");
  return TGNX_OK;
}

// tgn_pred_train stages the predictor weights in dynamic LDS (up to 2 x 128 x 129 floats)
static bool pred_smem_ok(int D) {
  auto set = [](const void* f) {
    return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tgn_pred_smem(TDMAX)) == hipSuccess;
  };
  static const bool ok = set(reinterpret_cast<const void*>(&tgn_pred_train<false>)) &&
                         set(reinterpret_cast<const void*>(&tgn_pred_train<true, 10>)) &&
                         set(reinterpret_cast<const void*>(&tgn_pred_train<true, ATT_EB>));
  return ok && tgn_pred_smem(D) <= tgn_pred_smem(TDMAX);
}

struct AdvArgs {
  int64_t lo, hi, batch;
  int rank, world;
  uint64_t seed;
};
// pipe (resident world-1 fused steps only): 0 = plain step; 1 = pipelined, this batch already marked and
// scanned by the previous pipelined step; 2 = pipelined, mark + scan this batch first.  A pipelined step
// marks the next batch inside tgn_pred_train and scans it after its own last launch.
extern "C++" {  // (inside the extern "C" block: the cell-templated step)
// the next batch's scan as 256-thread head workgroups of the fixup launch: its LDS within the launch's,
// and (small graphs, walked directly) <= 2 bitmap words per thread
// (k: the global batch, whose plans the scan sorts; kr: the rank's share, whose centres the walk stages)
static inline bool scan_rides(const Ctx& c, const Caps& k, const Caps& kr, size_t lds) {
  return tgn_scan_smem(k.B) <= lds && (size_t)3 * kr.B * 12 <= lds && (!scan_direct(c.words) || c.words <= 2 * 256);
}
static inline bool scan_folds(const Ctx& c, const Caps& k, const Caps& kr) {
  return scan_rides(c, k, kr, (size_t)GEMM_FIX_SMEM * 4);
}
// pp >= 0 (tgnx_tgn_train_step_pp, world 1, 1 hop): the step reads scan-output set pp; the next batch is marked
// in the predictor launch and scanned into set 1 - pp inside the k / v reduction launch (its outputs are then
// written while this step's later launches still read set pp's), the fixup launch only writes its descriptor
template <int CELL>
static int train_step_impl_c(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg, int32_t dropout,
                             void* stream, bool fuse_adam, const AdvArgs* adv, int pipe, int pp) {
  using Cl = CellOps<CELL>;
  const bool no_tail = (pipe & 4) != 0;  // pipelined, but the next batch's scan is the caller's (tgnx_tgn_scan_next)
  pipe &= 3;
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  if (adv) {
    TGNX_CHECK_ARG(adv->batch > 0 && adv->batch <= cfg->max_batch && adv->world >= 1 && adv->rank >= 0 &&
                       adv->rank < adv->world && adv->lo >= 0 && adv->hi >= adv->lo && adv->hi <= c.nev,
                   "tgnx_tgn_train_step_resident: bad cursor arguments (batch, rank / world, or split beyond the "
                   "event table)");
    // the fused step applies Adam to this rank's gradients in place: only a world-1 step has the whole sum
    TGNX_CHECK_ARG(!fuse_adam || adv->world == 1,
                   "tgnx_tgn_train_step_resident: world > 1 steps all-reduce before Adam "
                   "(tgnx_tgn_train_fwd_bwd_resident + exchange + tgnx_tgn_train_update)");
    c.adv = 1;
    c.adv_lo = adv->lo;
    c.adv_hi = adv->hi;
    c.adv_batch = adv->batch;
    c.adv_rank = adv->rank;
    c.adv_world = adv->world;
    c.adv_seed = adv->seed;
  }
  // data parallel: the rank's share ceil(B / world) of the global batch sets every per-rank capacity that
  // sizes a grid or a GEMM shape (roots, sampled nodes / edges, predictor rows, update list): grids sized
  // from the global batch launched ~W x the workgroups a rank needs (tgn_pred_train at world 8: 1,600
  // blocks for 200 events).  The global batch keeps what replays it whole on every rank (ring insert,
  // store update, their plans).  World 1 and the advance-driven form (world read on the device): kr == k.
  tgnx_tgn_config cfg_r = *cfg;
  if (adv) cfg_r.max_batch = (int)((cfg->max_batch + adv->world - 1) / adv->world);
  const Caps kr = make_caps(&cfg_r);
  c.Bmax = kr.B;  // (the scan walk stages the rank's centres in LDS: 3 Bmax entries)
  TGNX_CHECK_ARG(buf->neg && buf->grads && buf->out_pos && buf->out_neg, "tgnx_tgn_train_fwd_bwd: null buffer");
  // DyRep embedding messages need every embedding of src ∪ dst on this rank: world 1 only
  TGNX_CHECK_ARG(!c.emb || !buf->xrows, "tgn: DyRep embedding messages (emb_in_msg) are a world-1 step");
  if (c.emb) c.Zupd = reinterpret_cast<float*>(reinterpret_cast<char*>(buf->ws) + W.uZ);
  if (fuse_adam) {
    TGNX_CHECK_ARG(buf->adam_m && buf->adam_v, "tgnx_tgn_train_step: null optimizer buffer");
    TGNX_CHECK_ARG(!buf->xrows, "tgnx_tgn_train_step: data parallel steps all-reduce before Adam (fwd_bwd + update)");
    c.adf.p = c.params;
    c.adf.m = c.am;
    c.adf.v = c.av;
    c.adf.ctl = c.ctl;
    c.adf.b1 = c.b1;
    c.adf.b2 = c.b2;
    c.adf.eps = c.eps;
    c.adf.keep_g = (buf->flags & TGNX_TGN_NO_GRAD_STORE) ? 0 : 1;
  }
  TGNX_CHECK_ARG(!gen_neg || (buf->dst_nodes && buf->n_dst > 0), "tgnx_tgn_train_fwd_bwd: no destination set");
  TGNX_CHECK_ARG(pipe == 0 || adv, "tgnx_tgn_train_step_pipelined: resident steps only");
  c.gen_neg = gen_neg ? 1 : 0;
  c.drop = dropout && cfg->dropout > 0.f;
  const bool ppm = pp >= 0;
  if (ppm && buf->plan_table) {  // the split's plans from the table built at binding (tgnx_tgn_plan_table)
    PlanTableKey pk{-1, -1, -1, -1, 0};
    bool known = false;
    {
      std::lock_guard<std::mutex> lk(g_ptab_mu);
      const auto it = ptab_registry().find(buf->plan_table);
      if (it != ptab_registry().end()) {
        pk = it->second;
        known = true;
      }
    }
    TGNX_CHECK_ARG(known, "tgn: buf->plan_table was not built by tgnx_tgn_plan_table in this process");
    TGNX_CHECK_ARG(adv, "tgn: plan tables serve the resident parity-set steps only");
    TGNX_CHECK_ARG(pk.lo == adv->lo && pk.hi == adv->hi && pk.batch == adv->batch && pk.stride == plan_slot_bytes(k.B),
                   "tgn: buf->plan_table was built for split [%lld, %lld) batch %lld (slot %lld B), the step runs "
                   "[%lld, %lld) batch %lld (slot %lld B): rebuild it with tgnx_tgn_plan_table",
                   (long long)pk.lo, (long long)pk.hi, (long long)pk.batch, (long long)pk.stride, (long long)adv->lo,
                   (long long)adv->hi, (long long)adv->batch, (long long)plan_slot_bytes(k.B));
    c.ptab = reinterpret_cast<const char*>(buf->plan_table);
    c.ptab_stride = plan_slot_bytes(k.B);
  }
  Ctx cn;  // ppm: the other parity's set (the next batch's scan writes it)
  if (ppm) {
    TGNX_CHECK_ARG(pp <= 1 && pipe != 0 && !no_tail && adv && (!fuse_adam || adv->world == 1),
                   "tgnx_tgn_train_step_pp / tgnx_tgn_train_fwd_bwd_pp: a resident step, parity 0 or 1 "
                   "(Adam fused at world 1 only)");
    char* ws = reinterpret_cast<char*>(buf->ws);
    cn = set_view(c, W, ws, 1 - pp);
    c = set_view(c, W, ws, pp);
    c.tagchk = 1;
  }
  hipStream_t s = as_stream(stream);
  const float* P = c.params;
  float* G = c.grads;
  const int D = c.D, HC = c.HC, Qm = c.Qm, d = c.d;
  if (pipe != 1) {
    const int nmark = gridn(3 * kr.B * 16, 256);
    tgn_mark<true><<<nmark, 256, 0, s>>>(c, nmark);
    TGNX_LAUNCH_CHECK("tgn_mark");
    probe_begin(TGNX_K_ASSEMBLE, s);
    tgn_scan<true><<<1 + 2 * c.pplan, TGNX_SCAN_T, tgn_scan_smem(k.B), s>>>(c, 0, 1);
    probe_end(TGNX_K_ASSEMBLE, s);
    TGNX_LAUNCH_CHECK("tgn_scan");
  }
  const int nedge = gridn((int64_t)kr.Rtr * c.K, 4, TGNX_AGG_EDGE_CAP);
  probe_begin(TGNX_K_EDGE_META, s);
  const int nevb = gridn(3 * kr.B * (c.evj ? 16 : 1), 256);
  const int nagg = nevb + nedge + gridn(kr.Mtr, 4, TGNX_AGG_NODE_CAP);
  const int64_t* nol = nullptr;
  const int* noc = nullptr;
  if (c.aggr == 0)
    launch_k(tgn_agg_emit<0>, dim3(nagg), dim3(256), 0, s, c, 0, nedge, nol, noc, 0, (int64_t)0, nevb);
  else if (c.aggr == 1 && c.d <= 192)
    launch_k(tgn_agg_emit<1>, dim3(nagg), dim3(256), 0, s, c, 0, nedge, nol, noc, 0, (int64_t)0, nevb);
  else
    launch_k(tgn_agg_emit<-1>, dim3(nagg), dim3(256), 0, s, c, 0, nedge, nol, noc, 0, (int64_t)0, nevb);
  probe_end(TGNX_K_EDGE_META, s);
  TGNX_LAUNCH_CHECK("tgn_agg_emit");
  // GRU over every sampled node ‖ lin_edge over every sampled edge (‖ 2 hops: conv2's lin_edge over the
  // root edges)
  const LoadRowK ea{c.encE, kr.Etr, D + d, D + d};  // the edges' [cos enc | msg] rows (tgn_agg_emit, train)
  const bool two = k.layers == 2;
  const LoadAttrMap ea1{c.encE, c.e1_e2, D + d};  // root edge -> its outer edge's row
  const int edge_cap = cap_per200("TGNX_EDGE_CAP200", TGNX_EDGE_CAP200, kr.B);
  const int md_cap = cap_per200("TGNX_MD_CAP200", TGNX_MD_CAP200, kr.B);
  const auto j_gru = gemm_job<G32L>(with_cap(gemm_shape<G32L>(kr.Mtr, Cl::G * D, Qm + D, c.cnt + CNT_M), TGNX_GRU_CAP),
                                    LoadGruA{c.X, c.mem, c.nid, 0, Qm, D, 0}, Cl::w(c), Cl::epi_train(c),
                                    (float*)nullptr);
  const auto j_edge = gemm_job<G32>(with_cap(gemm_shape<G32>(kr.Etr, HC, D + d, c.cnt + CNT_E), edge_cap), ea,
                                    LoadRowK{P + c.L.we, HC, D + d, D + d}, EpiStore{c.Ep, nullptr, HC, 0}, (float*)nullptr);
  const BlockJob<RingMergeJob> j_ring{RingMergeJob{c}, gridn(2 * k.B, 4)};
  probe_begin(TGNX_K_EDGE_FWD, s);
  if (two)
    gemmN_launch(s, j_ring, j_gru, j_edge,
                 gemm_job<G32>(gemm_shape<G32>(kr.E1tr, HC, D + d, c.cnt + CNT_E1), ea1,
                               LoadRowK{P + c.L.we2, HC, D + d, D + d}, EpiStore{c.Ep2, nullptr, HC, 0}, (float*)nullptr));
  else
    gemmN_launch_w<TGNX_GRU_WAVES>(s, j_ring, j_gru, j_edge);
  probe_end(TGNX_K_EDGE_FWD, s);
  TGNX_LAUNCH_CHECK("tgn_gru_edge");
  const int nmark = gridn(3 * kr.B * 16, 256);
  // 1 hop with the attention forward in the predictor: the attention backward computes each edge's (dk, dv)
  // where it sums them (kv_edge_body), so the k / v reduction launch is gone and the GEMMs that need only dE
  // ride in a later launch
  // (2 hops: the outer level, whose attention forward is tgn_attn_fwd; its edges keep the sampling order)
  const bool kvf = true;  // (the separate k / v reduction launch: slower)
  const bool kvs = !two && (size_t)kr.Mtr + 1 <= tgn_pred_smem(c.D) / 4;
  c.kvf = 1;
  c.kvs = kvs ? 1 : 0;
  // a pipelined step marks the next batch in the predictor launch, beside its sort block (in the dz0 launch for
  // graphs marked through summary bitmaps: review-shaped 0.1040 vs 0.1037 ms, not kept)
  probe_begin(TGNX_K_PROJ, s);
  gemmN_launch(s, gemm_job<G32>(gemm_shape<G32>(kr.Mtr, 4 * HC, D, c.cnt + CNT_M), LoadZ{c.Z0, c.mem, c.nid, D, 0},
                             LoadProjW{P + c.L.wq, c.L.pw, HC, D}, EpiProj{P + c.L.bq, c.L.pb, c.P, HC}, (float*)nullptr));
  probe_end(TGNX_K_PROJ, s);
  TGNX_LAUNCH_CHECK("tgn_proj");
  // 1 hop: the attention forward runs inside tgn_pred_train (per root, beside its weight staging)
  const bool att_in_pred = !two;
  if (!att_in_pred) {
    probe_begin(TGNX_K_SEG_FWD, s);
    launch_k(tgn_attn_fwd<true>, dim3(gridn(kr.Rtr, 4, 1 << 20)), dim3(256), 0, s, c);
    probe_end(TGNX_K_SEG_FWD, s);
    TGNX_LAUNCH_CHECK("tgn_attn_fwd");
  }
  Ctx cr = two ? root_view(c) : c;  // the level the predictor reads
  if (two) cr.kvf = cr.kvs = 0;  // conv2's attention backward leaves its (dk, dv) sums to the k / v reduction job
  if (two) {  // conv2 over the roots: projections of h1 (rows = outer centres), attention per root
    gemm_launch<G32>(gemm_shape<G32>(kr.Rtr, 4 * HC, HC, c.cnt + CNT_R), LoadRowK{c.Zc, kr.Rtr, HC, HC},
                     LoadProjW{P + c.L.wq2, c.L.pw, HC, HC}, EpiProj{P + c.L.bq2, c.L.pb, c.P2, HC}, nullptr, s);
    TGNX_LAUNCH_CHECK("tgn_proj2");
    tgn_attn_fwd<true><<<gridn(kr.R1tr, 4, 1 << 20), 256, 0, s>>>(cr);
    TGNX_LAUNCH_CHECK("tgn_attn_fwd2");
  }
  // where the next batch's scan runs (parity-set steps): all of it as the first workgroups of the dW_cell
  // launch when its LDS holds the plans; else, for partitioned plans (data parallel: the global batch's
  // 2 B keys) that fit the predictor launch's LDS, the plans there and the walk alone in the dW_cell launch;
  // else its own launch after the dW_cell launch
  // (with a plan table the scan is the walk alone: it rides when the rank's centres fit the launch's LDS, 1 hop in
  // the attention-backward launch instead of the dW_cell launch)
  // (with a plan table the scan is the walk alone: its LDS is the centre staging, 3 B x 12 bytes, and the small-graph
  // direct walk's <= 2 words per thread; 2 hops: the walk rides in conv1's attention-backward launch)
  // (the attention-backward walk holds 2 bitmap words per thread, the dW_cell launch's ScanJob 8: its LDS word list
  // takes the 2-hop comment-shaped walk's ~1,100 words; 2 hops: the walk rides there — comment-shaped A/B 0.2383 /
  // 0.2397 ms against 0.2462 / 0.2459 for the pipelined step, 0.2504 / 0.2498 in the attention backward; the wide
  // walk in the attention backward cost the wiki step +0.9 %)
  const auto walk_rides = [&](size_t lds, int wpt) {
    return (size_t)3 * kr.B * 12 <= lds && (!scan_direct(c.words) || c.words <= (int64_t)wpt * 256);
  };
  const bool walk_bwd = ppm && c.ptab && !two && walk_rides((size_t)3 * MARK_LDS_WORDS * 4, 2);
  const int nwalk = walk_bwd ? 1 : 0;
  const uint32_t walk_lds = walk_bwd ? (uint32_t)(3 * kr.B * 12 + 16) : 0u;
  const bool scan_w3 = ppm && !walk_bwd && (c.ptab ? walk_rides((size_t)3 * MARK_LDS_WORDS * 4, 8)
                                                   : scan_rides(c, k, kr, (size_t)3 * MARK_LDS_WORDS * 4));
  static const int plans_in_pred = env_int("TGNX_PLANS_IN_PRED", TGNX_PLANS_IN_PRED);  // (runtime A/B switch)
  const bool plans_pred = ppm && !c.ptab && !scan_w3 && plans_in_pred && c.pplan > 1 && c.pplan <= plans_in_pred &&
                          2 * k.B <= PRED_PLAN_MAXE * 256 &&
                          scan_rides(c, kr, kr, (size_t)3 * MARK_LDS_WORDS * 4) &&
                          tgn_scan_smem(k.B) <= tgn_pred_smem(TDMAX);
  const int npl = plans_pred ? 2 * c.pplan : 0;
  probe_begin(TGNX_K_PRED, s);
  TGNX_CHECK_ARG(pred_smem_ok(c.D), "tgn_pred_train: dynamic LDS attribute refused");
  const int nmk = ppm || pipe ? nmark : 0;
  const size_t psm = std::max({att_in_pred || pred_stages<false>() ? tgn_pred_smem(c.D) : (size_t)16,
                               nmk ? (size_t)3 * MARK_LDS_WORDS * 4 : (size_t)0,
                               npl ? tgn_scan_smem(k.B) : (size_t)0});
  const int nsrt = (two ? cr.kvs : kvs) ? 1 : 0;  // (kvs: the rows fit the sort's LDS counters)
  const PlanOut po = plan_out(ppm ? cn : c);
  if (att_in_pred)
    launch_k(c.K <= 10 ? tgn_pred_train<true, 10> : tgn_pred_train<true, ATT_EB>, dim3(kr.B + npl + nsrt + nmk),
             dim3(64 * pred_waves<true>()), (uint32_t)psm, s, cr, nmk, nsrt, po, npl);
  else
    launch_k(tgn_pred_train<false>, dim3((pred_stages<false>() ? pred_groups(kr.B) : kr.B) + npl + nsrt + nmk),
             dim3(64 * pred_waves<false>()), (uint32_t)psm, s, cr,
             nmk, nsrt, po, npl);
  probe_end(TGNX_K_PRED, s);
  TGNX_LAUNCH_CHECK("tgn_pred_train");
  if (c.emb) {
    // DyRepMemory.update_state in train order (memory_module.py:322-325): the memory of src ∪ dst from their
    // stored messages with the embeddings of this batch's forward in place of memory rows (:387-408) — the
    // stores are still the previous batch's (StoreJob runs later); the fixup writes these rows (Zupd)
    const Ctx ce = emb_view(c, W, reinterpret_cast<char*>(buf->ws));
    gru_list_c<CELL>(ce, c.upd, c.cnt + CNT_U, 0, 0, kr.Ucap, s, true);
    TGNX_LAUNCH_CHECK("tgn_emb_update");
  }
  probe_begin(TGNX_K_SEG_BWD, s);
  if (two) {
    // conv2 backward (‖ predictor reductions) -> dP2, dE2; then dh1 = dP2 [Wq2; Wk2; Wv2; Wsk2] ‖ dW_proj2,
    // dW_edge2 (deferred) ‖ conv2's lin_edge -> Δt-encoding partials; then conv backward from dh1
    const int ncb1 = gridn(kr.R1tr, 4, 1 << 20);
    launch_k(attn_bwd_fn(c.K, cr.dzrep, true), dim3(ncb1 + gridn(3 * D + 2, 4)), dim3(256), 0u, s, cr, ncb1, 0, 0, cr);
    TGNX_LAUNCH_CHECK("tgn_attn_bwd2");
    // conv2's (dk, dv) sums ‖ its dE2-only GEMMs (as in the 1-hop step below), then dh1 ‖ dW_proj2
    const auto j_dwe2 = gemm_job<GW>(shp_dWe2(kr, c.cnt), LoadKRow{c.dE2, HC, kr.E1tr, HC}, LoadAttrMapT{ea1},
                                     EpiDeferred{}, c.pF);
    const auto j_denc2 = gemm_job<G32>(gemm_shape<G32>(kr.E1tr, D, HC, c.cnt + CNT_E1), LoadRowK{c.dE2, kr.E1tr, HC, HC},
                                       LoadKRow{P + c.L.we2, D, HC, D + d},
                                       EpiTeEdge{c.e_j, c.e_t, c.lu, c.tgp, D, c.e1_e2, c.tgp_e1, P + c.L.te_w,
                                                 P + c.L.te_b},
                                       (float*)nullptr);
    const auto j_dh1 = gemm_job<G32L>(gemm_shape<G32L>(kr.Rtr, HC, 4 * HC, c.cnt + CNT_R),
                                      LoadRowK{c.dP2, kr.Rtr, 4 * HC, 4 * HC}, LoadProjWT{P + c.L.wq2, c.L.pw, HC, HC},
                                      EpiStore{c.dZc, nullptr, HC, 0}, (float*)nullptr);
    const auto j_dwp2 = gemm_job<GW>(shp_dWp2(kr, c.cnt), LoadKRow{c.dP2, 4 * HC, kr.Rtr, 4 * HC}, LoadZ1T{c.Zc, HC},
                                     EpiDeferred{}, c.pE);
    gemmN_launch(s, BlockJob<KvReduceJob>{KvReduceJob{cr}, gridn(kr.E1tr, KVR_CH, 1 << 20)}, j_dwe2, j_denc2);
    TGNX_LAUNCH_CHECK("tgn_kv_reduce2");
    gemmN_launch(s, j_dh1, j_dwp2);
    TGNX_LAUNCH_CHECK("tgn_dh1");
    const int ncb = gridn(kr.Rtr, 4, 1 << 20), nkv = kvf ? gridn(kr.Etr, KVE_CH, 1 << 20) : 0;
    launch_k(attn_bwd_fn(c.K, c.dzrep, true), dim3(ncb + nkv + nwalk), dim3(256), walk_lds, s, c,
             ncb, nkv, nwalk, nwalk ? cn : c);
  } else {
    const int ncb = gridn(kr.Rtr, 4, 1 << 20);
    const int nkv = kvf ? gridn(kr.Etr, KVE_CH, 1 << 20) : 0;
    launch_k(attn_bwd_fn(c.K, c.dzrep), dim3(ncb + nkv + gridn(3 * D + 2, 4) + nwalk),
             dim3(256), walk_lds, s, c, ncb, nkv, nwalk, nwalk ? cn : c);
  }
  probe_end(TGNX_K_SEG_BWD, s);
  TGNX_LAUNCH_CHECK("tgn_attn_bwd");
  // k / v sums into dP ‖ the GEMMs that need only dE: dW_edge (deferred split-K) and dEnc·W_e (Δt
  // partials of the sampled edges).  Jobs of one gemmN launch add up rather than overlap (measured:
  // the five backward jobs in one launch took 28 us, dz0 alone 16), while kv_reduce leaves most CUs
  // idle: the dE-only GEMMs fill them here instead of lengthening the dP launch below.
  const Ctx cf = fixup_view(c);
  const EpiGradStore e_dWe{G, c.L.we, D + d, cf.adf};
  const auto j_dwe = gemm_job<GW>(shp_dWe(kr, c.cnt), LoadKRow{c.dE, HC, kr.Etr, HC}, LoadKRow{c.encE, D + d, kr.Etr, D + d},
                                  EpiDeferred{}, c.pA);
  const auto j_denc = gemm_job<G32>(with_cap(gemm_shape<G32>(kr.Etr, D, HC, c.cnt + CNT_E), edge_cap), LoadRowK{c.dE, kr.Etr, HC, HC},
                                    LoadKRow{P + c.L.we, D, HC, D + d}, EpiTeEdge{c.e_j, c.e_t, c.lu, c.tgp, D, nullptr, 0, P + c.L.te_w, P + c.L.te_b},
                                    (float*)nullptr);
  // weight gradients (deferred split-K) ‖ ...
  const EpiProjGrad e_dWp{G, c.L.wq, c.L.bq, c.L.pw, c.L.pb, HC, D, cf.adf};
  const EpiLpGrad e_dWlp{G, c.L.lsw, c.L.ldw, D, cf.adf};
  const auto e_dWg = Cl::wgrad(cf);
  // one launch: dW_proj, dW_src/dst (deferred split-K) ‖ dz0 = dP W with the GRU backward in its
  // epilogue — all read only what attn_bwd / kv_reduce / pred_train produced
  const int rows_edge = (kr.Etr + G32::TM - 1) / G32::TM, rows_msg = (kr.Mtr + G32::TM - 1) / G32::TM;
  probe_begin(TGNX_K_EDGE_BWD, s);
  const auto j_dwp = gemm_job<GW>(shp_dWp(kr, c.cnt), LoadKRow{c.dP, 4 * HC, kr.Mtr, 4 * HC}, LoadZ1T{c.Z0, D}, EpiDeferred{}, c.pB);
  const auto j_dwlp = gemm_job<GW>(shp_dWlp(kr, c.cnt), LoadLpA{c.evs, c.ctl, D, evs_stride(D)},
                                   LoadLpB{c.evs, c.ctl, D, evs_stride(D)}, EpiDeferred{}, c.pC);
  const auto j_dz0 = gemm_job<G32L>(with_cap(gemm_shape<G32L>(kr.Mtr, D, 4 * HC, c.cnt + CNT_M), md_cap), LoadRowK{c.dP, kr.Mtr, 4 * HC, 4 * HC},
                                    LoadProjWT{P + c.L.wq, c.L.pw, HC, D}, Cl::bwd(c), (float*)nullptr);
  auto l7 = [&](auto... jobs) {
    gemmN_launch(s, jobs...);
    probe_end(TGNX_K_EDGE_BWD, s);
    TGNX_LAUNCH_CHECK("tgn_wgrad_dz0");
    return TGNX_OK;
  };
  // ‖ the message stores ‖ the fixup's descriptor copy + the counter advance (SnapJob)
  const int nst = gridn(2 * k.B, 256);
  const auto j_dwg = gemm_job<GW>(shp_dWg(kr, c.cnt), LoadKRow{c.dG, Cl::G * D, kr.Mtr, Cl::G * D},
                                  Cl::hT(c), EpiDeferred{}, c.pD);
  const auto j_dxe = gemm_job<GXE>(with_cap(gemm_shape<GXE>(kr.Mtr, D, Cl::G * D, c.cnt + CNT_M), md_cap),
                                    LoadRowK{c.dG, kr.Mtr, Cl::G * D, Cl::G * D}, Cl::wenc(c),
                                    EpiTeMsg{c.s0m, c.s1m, c.tgp, D, rows_edge}, (float*)nullptr);
  // ppm: the next batch's scan (into set 1 - pp; the counters advance in the fixup launch) as this launch's
  // first workgroups when it fits their LDS, else its own launch after it
  const auto j_scan = BlockJob<ScanJob, 3 * MARK_LDS_WORDS>{ScanJob{cn}, walk_bwd ? 0 : plans_pred || c.ptab ? 1 : 1 + 2 * c.pplan};
  const auto j_snap = BlockJob<SnapJob>{SnapJob{c, ppm ? 1 : 0}, 1};
  const auto j_store = BlockJob<StoreJob>{StoreJob{c, nst}, nst};
  // (the scan may ride in the dz0 launch instead: TGNX_SCAN_AT 6)
  const bool scan6 = scan_w3 && TGNX_SCAN_AT == 6;
  const bool walk_w3 = (scan_w3 || plans_pred) && !walk_bwd;  // (the walk rides in the dW_cell launch)
  auto l8 = [&](auto... jobs) {
    probe_begin(TGNX_K_WGRAD3, s);
    // the GEMM jobs before the snapshot / store blocks (0.0970 vs 0.0986 ms with those first)
    // (the edge jobs dEnc / dW_edge first instead: that launch 12.8 -> 14.7 us, r5_w3_jobs_first_ab.txt)
    if (walk_w3 && !scan6)
      gemmN_launch(s, j_scan, j_dxe, j_dwg, jobs..., j_snap, j_store);
    else
      gemmN_launch_w<TGNX_W3_WAVES>(s, j_dxe, j_dwg, jobs..., j_snap, j_store);
    probe_end(TGNX_K_WGRAD3, s);
    TGNX_LAUNCH_CHECK("tgn_wgrad3");
    return TGNX_OK;
  };
  // kvf: the dE-only GEMMs ride in the dW_gru launch (in the dz0 launch: 0.1013 vs 0.0987 ms; dW_proj / dW_lp
  // moved to the dW_gru launch too: 0.1013 - 0.1035), dz0 first in its launch (0.0985 vs 0.0991)
  // (the lambdas return the launch checks' status)
  if (scan6) {
    if ((rc = l7(j_scan, j_dz0, j_dwp, j_dwlp)) || (rc = l8(j_dwe, j_denc))) return rc;
  } else if ((rc = l7(j_dz0, j_dwp, j_dwlp)) || (rc = l8(j_dwe, j_denc))) {  // (dW_edge in the dz0 launch: slower,
    return rc;                                                                 //  r4_dwe_in_dz0_ab.txt)
  }
  if (ppm && !walk_w3 && !walk_bwd) {  // (with a plan table: the walk alone)
    tgn_scan<true><<<c.ptab ? 1 : 1 + 2 * c.pplan, TGNX_SCAN_T, tgn_scan_smem(k.B), s>>>(cn, 1, 0);
    TGNX_LAUNCH_CHECK("tgn_scan_early");
  }
  // split-K sums + epilogues ‖ Δt reduction ‖ update_state's memory half (train order: memory of src ∪
  // dst from this step's GRU rows; the stores and the ring insert ran in earlier launches), reading the
  // step descriptor from SnapJob's copy (cf) — so that the pipelined step's next-batch scan (counters
  // advanced by SnapJob) rides in the same launch as its first workgroups when it fits (scan_folds)
  const int nte = (2 * D + 63) / 64;
  const int nmem = gridn(kr.Ucap, 4, 1024);
  const bool scan_next = pipe && !no_tail && !ppm;
  const bool fold = scan_next && scan_folds(c, k, kr);
  const int nscan = fold ? 1 + 2 * c.pplan : 0;
  const TrainTail tail{TeReduceTail{cf, rows_edge, rows_msg}, c, nscan, nte, nmem, ppm ? 1 : 0};
  probe_begin(TGNX_K_FINISH, s);
  if (two)
    gemm_fixup_launch_h(nscan, nscan + nte + nmem, tail, s, gemm_fix<GW>(shp_dWe(kr, cf.cnt), c.pA, e_dWe),
                        gemm_fix<GW>(shp_dWp(kr, cf.cnt), c.pB, e_dWp), gemm_fix<GW>(shp_dWlp(kr, cf.cnt), c.pC, e_dWlp),
                        gemm_fix<GW>(shp_dWg(kr, cf.cnt), c.pD, e_dWg),
                        gemm_fix<GW>(shp_dWp2(kr, cf.cnt), c.pE, EpiProjGrad{G, c.L.wq2, c.L.bq2, c.L.pw, c.L.pb, HC, HC, cf.adf}),
                        gemm_fix<GW>(shp_dWe2(kr, cf.cnt), c.pF, EpiGradStore{G, c.L.we2, D + d, cf.adf}));
  else
    gemm_fixup_launch_h(nscan, nscan + nte + nmem, tail, s, gemm_fix<GW>(shp_dWe(kr, cf.cnt), c.pA, e_dWe),
                        gemm_fix<GW>(shp_dWp(kr, cf.cnt), c.pB, e_dWp), gemm_fix<GW>(shp_dWlp(kr, cf.cnt), c.pC, e_dWlp),
                        gemm_fix<GW>(shp_dWg(kr, cf.cnt), c.pD, e_dWg));
  probe_end(TGNX_K_FINISH, s);
  TGNX_LAUNCH_CHECK("tgn_fixup_update");
  if (scan_next && !fold) {  // the next batch (counters advanced by SnapJob): sorted node sets, plans, descriptor
    probe_begin(TGNX_K_ASSEMBLE, s);
    tgn_scan<true><<<1 + 2 * c.pplan, TGNX_SCAN_T, tgn_scan_smem(k.B), s>>>(c, 0, 1);
    probe_end(TGNX_K_ASSEMBLE, s);
    TGNX_LAUNCH_CHECK("tgn_scan_next");
  }
  return TGNX_OK;
}

}  // extern "C++"

static int train_step_impl(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg, int32_t dropout,
                           void* stream, bool fuse_adam, const AdvArgs* adv = nullptr, int pipe = 0, int pp = -1) {
  if (cfg && cfg->updater == 1) return train_step_impl_c<1>(cfg, buf, gen_neg, dropout, stream, fuse_adam, adv, pipe, pp);
  return train_step_impl_c<0>(cfg, buf, gen_neg, dropout, stream, fuse_adam, adv, pipe, pp);
}

int tgnx_tgn_train_fwd_bwd(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg, int32_t dropout,
                           void* stream) {
  return train_step_impl(cfg, buf, gen_neg, dropout, stream, false);
}

int tgnx_tgn_train_step(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg, int32_t dropout,
                        void* stream) {
  return train_step_impl(cfg, buf, gen_neg, dropout, stream, true);
}

int tgnx_tgn_train_step_resident(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                 int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                 int32_t dropout, void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, rank, world, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, true, &a);
}

int tgnx_tgn_train_step_pipelined(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                  int64_t split_hi, int64_t batch, uint64_t base_seed, int32_t dropout,
                                  int32_t prefetched, void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, 0, 1, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, true, &a, prefetched ? 1 : 2);
}

int tgnx_tgn_train_step_pp(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo, int64_t split_hi,
                           int64_t batch, uint64_t base_seed, int32_t dropout, int32_t prefetched, int32_t parity,
                           void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, 0, 1, base_seed};
  TGNX_CHECK_ARG(parity == 0 || parity == 1, "tgnx_tgn_train_step_pp: parity must be 0 or 1");
  return train_step_impl(cfg, buf, 1, dropout, stream, true, &a, prefetched ? 1 : 2, parity);
}

int tgnx_tgn_train_fwd_bwd_pp(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                              int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                              int32_t dropout, int32_t prefetched, int32_t parity, int32_t apply_prev, float* rows,
                              int64_t nrows, void* stream) {
  TGNX_CHECK_ARG(parity == 0 || parity == 1, "tgnx_tgn_train_fwd_bwd_pp: parity must be 0 or 1");
  TGNX_CHECK_ARG(!apply_prev || (nrows >= 0 && (nrows == 0 || rows)), "tgnx_tgn_train_fwd_bwd_pp: bad rows");
  if (apply_prev) {  // the previous step's exchanged rows + Adam (tgnx_tgn_apply_rows_update) at the head of this step
    const int rc = tgnx_tgn_apply_rows_update(cfg, buf, rows, nrows, stream);
    if (rc) return rc;
  }
  const AdvArgs a{split_lo, split_hi, batch, rank, world, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, false, &a, prefetched ? 1 : 2, parity);
}

int tgnx_tgn_train_fwd_bwd_split(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                 int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                 int32_t dropout, int32_t prefetched, void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, rank, world, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, false, &a, (prefetched ? 1 : 2) | 4);
}

int tgnx_tgn_scan_next(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo, int64_t split_hi,
                       int64_t batch, int32_t rank, int32_t world, uint64_t base_seed, void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  TGNX_CHECK_ARG(batch > 0 && batch <= cfg->max_batch && world >= 1 && rank >= 0 && rank < world && split_lo >= 0 &&
                     split_hi >= split_lo && split_hi <= c.nev,
                 "tgnx_tgn_scan_next: bad cursor arguments");
  c.adv = 1;
  c.adv_lo = split_lo;
  c.adv_hi = split_hi;
  c.adv_batch = batch;
  c.adv_rank = rank;
  c.adv_world = world;
  c.adv_seed = base_seed;
  hipStream_t s = as_stream(stream);
  probe_begin(TGNX_K_ASSEMBLE, s);
  tgn_scan<true><<<1 + 2 * c.pplan, TGNX_SCAN_T, tgn_scan_smem(k.B), s>>>(c, 0, 1);
  probe_end(TGNX_K_ASSEMBLE, s);
  TGNX_LAUNCH_CHECK("tgn_scan_next");
  return TGNX_OK;
}

int tgnx_tgn_train_fwd_bwd_pipelined(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                     int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                     int32_t dropout, int32_t prefetched, void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, rank, world, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, false, &a, prefetched ? 1 : 2);
}

int tgnx_tgn_train_fwd_bwd_resident(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                    int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                    int32_t dropout, void* stream) {
  const AdvArgs a{split_lo, split_hi, batch, rank, world, base_seed};
  return train_step_impl(cfg, buf, 1, dropout, stream, false, &a);
}

int tgnx_tgn_apply_rows(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, float* rows, int64_t nrows,
                        void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf && buf->memory && buf->last_update, "tgnx_tgn_apply_rows: null buffer");
  TGNX_CHECK_ARG(nrows >= 0 && (nrows == 0 || rows), "tgnx_tgn_apply_rows: bad rows");
  if (nrows == 0) return TGNX_OK;
  tgn_apply_rows<<<gridn(nrows, 4, 4096), 256, 0, as_stream(stream)>>>(buf->memory, buf->last_update, rows, nrows,
                                                                        cfg->mem_dim, cfg->num_nodes);
  TGNX_LAUNCH_CHECK("tgn_apply_rows");
  return TGNX_OK;
}

int tgnx_tgn_train_update(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->grads && buf->adam_m && buf->adam_v, "tgnx_tgn_train_update: null optimizer buffer");
  probe_begin(TGNX_K_ADAM, as_stream(stream));
  tgn_adam<<<gridn(c.L.total / 4, 256), 256, 0, as_stream(stream)>>>(c, nullptr, 0, 0);
  probe_end(TGNX_K_ADAM, as_stream(stream));
  TGNX_LAUNCH_CHECK("tgn_adam");
  return TGNX_OK;
}
int tgnx_tgn_apply_rows_update(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, float* rows, int64_t nrows,
                               void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->grads && buf->adam_m && buf->adam_v, "tgnx_tgn_apply_rows_update: null optimizer buffer");
  TGNX_CHECK_ARG(nrows >= 0 && (nrows == 0 || rows), "tgnx_tgn_apply_rows_update: bad rows");
  const int nrb = nrows ? gridn(nrows, 4, 1024) : 0;
  probe_begin(TGNX_K_ADAM, as_stream(stream));
  tgn_adam<<<gridn(c.L.total / 4, 256) + nrb, 256, 0, as_stream(stream)>>>(c, rows, nrows, nrb);
  probe_end(TGNX_K_ADAM, as_stream(stream));
  TGNX_LAUNCH_CHECK("tgn_adam_rows");
  return TGNX_OK;
}

int tgnx_tgn_eval_step(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t Kn, void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  TGNX_CHECK_ARG(cfg && Kn >= 1 && Kn <= (cfg->max_neg < 1 ? 1 : cfg->max_neg), "tgnx_tgn_eval_step: Kn out of range");
  int rc = make_ctx(cfg, buf, Kn, c, k, W);
  if (rc) return rc;
  TGNX_CHECK_ARG(buf->neg && buf->out_pos && buf->out_neg && buf->mrr, "tgnx_tgn_eval_step: null buffer");
  hipStream_t s = as_stream(stream);
  const float* P = c.params;
  const int D = c.D, HC = c.HC, d = c.d;
  const bool two = k.layers == 2;
  const int R1q = (int)std::min<int64_t>(c.N, (int64_t)k.B * (2 + Kn));  // roots
  const int Rq = two ? (int)std::min<int64_t>(c.N, (int64_t)R1q * (c.K + 1)) : R1q;  // (outer) centres
  const int Mq = (int)std::min<int64_t>(c.N, (int64_t)Rq * (c.K + 1));
  const int Eq = Rq * c.K, E1q = two ? R1q * c.K : 0;
  {
    const int nmark = gridn((int64_t)k.B * (2 + Kn) * 16, 256);
    tgn_mark<false><<<nmark, 256, 0, s>>>(c, nmark);
  }
  TGNX_LAUNCH_CHECK("tgn_mark");
  tgn_scan<false><<<1 + 2 * c.pplan, TGN_SCAN_THREADS, tgn_scan_smem(k.B), s>>>(c, 0, 1);
  TGNX_LAUNCH_CHECK("tgn_scan");
  const int nedge = gridn((int64_t)Rq * c.K, 4, 4096);
  tgn_agg_emit<-1><<<nedge + gridn(Mq, 256), 256, 0, s>>>(c, 1, nedge, nullptr, nullptr, 0, 0);
  TGNX_LAUNCH_CHECK("tgn_emit");
  const LoadEdgeAttr ea{c.encE, c.e_id, c.ev_msg, D, d};
  const auto j_edge = gemm_job<G32>(gemm_shape<G32>(Eq, HC, D + d, c.cnt + CNT_E), ea,
                                    LoadRowK{P + c.L.we, HC, D + d, D + d}, EpiStore{c.Ep, nullptr, HC, 0}, (float*)nullptr);
  const auto j_proj = gemm_job<G32>(gemm_shape<G32>(Mq, 4 * HC, D, c.cnt + CNT_M), LoadZ{c.Z0, c.mem, c.nid, D, 1},
                                    LoadProjW{P + c.L.wq, c.L.pw, HC, D}, EpiProj{P + c.L.bq, c.L.pb, c.P, HC},
                                    (float*)nullptr);
  if (two)
    gemmN_launch(s, j_edge, j_proj,
                 gemm_job<G32>(gemm_shape<G32>(E1q, HC, D + d, c.cnt + CNT_E1),
                               LoadEdgeAttrMap{c.encE, c.e1_id, c.e1_e2, c.ev_msg, D, d},
                               LoadRowK{P + c.L.we2, HC, D + d, D + d}, EpiStore{c.Ep2, nullptr, HC, 0}, (float*)nullptr));
  else
    gemmN_launch(s, j_edge, j_proj);
  TGNX_LAUNCH_CHECK("tgn_edge_proj");
  tgn_attn_fwd<false><<<gridn(Rq, 4, 1 << 20), 256, 0, s>>>(c);
  TGNX_LAUNCH_CHECK("tgn_attn_fwd");
  const Ctx cr = two ? root_view(c) : c;
  if (two) {
    gemm_launch<G32>(gemm_shape<G32>(Rq, 4 * HC, HC, c.cnt + CNT_R), LoadRowK{c.Zc, Rq, HC, HC},
                     LoadProjW{P + c.L.wq2, c.L.pw, HC, HC}, EpiProj{P + c.L.bq2, c.L.pb, c.P2, HC}, nullptr, s);
    TGNX_LAUNCH_CHECK("tgn_proj2");
    tgn_attn_fwd<false><<<gridn(R1q, 4, 1 << 20), 256, 0, s>>>(cr);
    TGNX_LAUNCH_CHECK("tgn_attn_fwd2");
  }
  gemm2_launch<G32, G32>(gemm_shape<G32>(R1q, D, D, c.cnt + cr.rsel), LoadRowK{cr.Zc, R1q, D, D},
               LoadRowK{P + c.L.lsw, D, D, D}, EpiStore{c.Hs, P + c.L.lsb, D, 0}, nullptr,
               gemm_shape<G32>(R1q, D, D, c.cnt + cr.rsel), LoadRowK{cr.Zc, R1q, D, D}, LoadRowK{P + c.L.ldw, D, D, D},
               EpiStore{c.Hd, P + c.L.ldb, D, 0}, nullptr, s);
  TGNX_LAUNCH_CHECK("tgn_lin_src_dst");
  tgn_score<<<k.B, 256, 0, s>>>(cr);
  TGNX_LAUNCH_CHECK("tgn_score");
  // update_state in eval order: stores first, then the GRU of src ∪ dst; ring insert
  const int nst = gridn(2 * k.B, 256), nring = gridn(2 * k.B, 4);
  tgn_update<<<nst + nring, 256, 0, s>>>(c, 0, nst, 1, nullptr, nullptr, 0, 0);
  TGNX_LAUNCH_CHECK("tgn_store_insert");
  // (DyRep embedding messages: the eval forward's embeddings of src ∪ dst, memory_module.py:327-329)
  gru_list(c, k, c.upd, c.cnt + CNT_U, 0, 0, k.Ucap, s, c.emb != 0);
  TGNX_LAUNCH_CHECK("tgn_gru_update");
  tgn_update<<<gridn(k.Ucap, 4, 1024), 256, 0, s>>>(c, gridn(k.Ucap, 4, 1024), 0, 1, c.upd, c.cnt + CNT_U, 0, 0);
  TGNX_LAUNCH_CHECK("tgn_memory_write");
  return TGNX_OK;
}

size_t tgnx_tgn_flush_scratch_bytes(const tgnx_tgn_config* cfg) {
  if (check_cfg(cfg)) return 0;
  const Caps k = make_caps(cfg);
  if (cfg->num_nodes <= k.Mcap) return 0;  // one chunk: every row is computed before any is written
  return (size_t)(al4(cfg->num_nodes * (int64_t)cfg->mem_dim) * 4 + cfg->num_nodes * 8);
}

int tgnx_tgn_flush(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* scratch, size_t scratch_bytes,
                   void* stream) {
  Ctx c;
  Caps k;
  WsLay W;
  int rc = make_ctx(cfg, buf, 1, c, k, W);
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  const int chunk = k.Mcap;
  // The reference updates every node from the state before the flush (memory_module.py:212,
  // _update_memory(arange(N)): all rows computed, then written).  The workspace holds Mcap GRU rows, so
  // graphs larger than that run in chunks; a later chunk's messages read the memory / last_update of
  // their other endpoint, which an earlier chunk has already rewritten.  So the chunks read a snapshot
  // of memory / last_update taken before the first write.
  Ctx cr = c;
  if (c.N > chunk) {
    const size_t need = tgnx_tgn_flush_scratch_bytes(cfg);
    TGNX_CHECK_ARG(scratch && scratch_bytes >= need && ((uintptr_t)scratch & 15) == 0,
                   "tgnx_tgn_flush: num_nodes > the workspace's row capacity needs a 16-B aligned scratch of "
                   "tgnx_tgn_flush_scratch_bytes(cfg) bytes");
    float* snap_mem = reinterpret_cast<float*>(scratch);
    int64_t* snap_lu = reinterpret_cast<int64_t*>(snap_mem + al4(c.N * (int64_t)c.D));
    TGNX_HIP_CHECK(hipMemcpyAsync(snap_mem, c.mem, (size_t)c.N * c.D * 4, hipMemcpyDeviceToDevice, s));
    TGNX_HIP_CHECK(hipMemcpyAsync(snap_lu, c.lu_buf, (size_t)c.N * 8, hipMemcpyDeviceToDevice, s));
    cr.mem = snap_mem;
    cr.lu_buf = snap_lu;
  }
  for (int64_t base = 0; base < c.N; base += chunk) {
    const int n = (int)std::min<int64_t>(chunk, c.N - base);
    gru_list(cr, k, nullptr, nullptr, n, base, n, s);
    TGNX_LAUNCH_CHECK("tgn_flush_gru");
    tgn_update<<<gridn(n, 4, 1024), 256, 0, s>>>(c, gridn(n, 4, 1024), 0, 1, nullptr, nullptr, n, base);
    TGNX_LAUNCH_CHECK("tgn_flush_write");
  }
  tgn_clear_store<<<gridn(c.N, 256), 256, 0, s>>>(c.st, c.N);
  TGNX_LAUNCH_CHECK("tgn_clear_store");
  return TGNX_OK;
}


// wave timeline stamps (diagnostic build, see tgnx_common.h)
int tgnx_stamps_set(void* buf, uint32_t cap) {
#ifdef TGNX_STAMPS
  StampRec* b = reinterpret_cast<StampRec*>(buf);
  const unsigned per = cap / 64;
  static unsigned z[64 * 32];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &b, sizeof b) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_cap), &per, sizeof per) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_cnt), z, sizeof z) != hipSuccess) {
    set_error("tgnx_stamps_set: symbol copy failed");
    return TGNX_EHIP;
  }
  return TGNX_OK;
#else
  (void)buf;
  (void)cap;
  set_error("tgnx_stamps_set: library built without TGNX_STAMPS");
  return TGNX_EINVAL;
#endif
}

// records per shard (64 shards of cap / 64 records each; shard s holds records [s * cap/64, ...))
int64_t tgnx_stamps_count(void) {
#ifdef TGNX_STAMPS
  unsigned n[64 * 32];
  if (hipMemcpyFromSymbol(n, HIP_SYMBOL(g_stamp_cnt), sizeof n) != hipSuccess) return -1;
  unsigned mx = 0;
  for (int s = 0; s < 64; ++s) mx = n[s * 32] > mx ? n[s * 32] : mx;
  return mx;
#else
  return -1;
#endif
}

}  // extern "C"
