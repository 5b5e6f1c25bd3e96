/* libtgnx — MI355X-native (gfx950) TGN temporal link-prediction hot path, C ABI.
 *
 * Every entry point takes plain device pointers, int64 sizes and a HIP stream
 * passed as `void*` (a hipStream_t; NULL = the default stream).  Nothing here
 * allocates: scratch comes from a caller-provided workspace whose size the
 * matching *_ws_bytes() query returns, so a sequence of calls can be captured
 * into a HIP graph.  All launches are asynchronous on `stream`.
 *
 * Return value: TGNX_OK (0) or a negative code; tgnx_last_error() then holds a
 * message (thread-local).  Indices are int64 (the reference's torch.long),
 * times are fp32 (the reference casts t to float32, temporal_dataset.py:42,53).
 *
 * The reference has no native layer: its "FFI" is the Python import seam at
 * pyg-mem-tgn.py:16-25.  Each function below cites the reference code it
 * replaces; INTEGRATION.md shows the ctypes binding a maintainer would add.
 */
#ifndef TGNX_H
#define TGNX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TGNX_OK 0
#define TGNX_EINVAL (-1)   /* bad argument / shape / capacity */
#define TGNX_EHIP (-2)     /* HIP launch or runtime error */
#define TGNX_ETOOBIG (-3)  /* size beyond what this build supports */

int tgnx_version(void);
const char* tgnx_last_error(void);

/* ------------------------------------------------------------------------
 * Temporal neighbour ring — LastNeighborLoader (neighbor_loader.py:15-109).
 * State: nbr int64[N*K], eid int64[N*K], t fp32[N*K] (row-major [N,K]), newest
 * first in every row; eid < 0 marks an empty slot; assoc int64[N].
 * ------------------------------------------------------------------------ */

/* reset_state (neighbor_loader.py:106-109): eid = -1, t = -1. */
int tgnx_ring_reset(int64_t* eid, float* t, int64_t num_nodes, int32_t size, void* stream);

/* __call__ (neighbor_loader.py:26-50).  Query n_id[q] (any int64 ids < N).
 * Outputs (capacity cap_nodes >= q*(1+K), cap_edges >= q*K):
 *   out_nid[M]          sorted unique of n_id ∪ valid neighbours
 *   out_ei[2*cap_edges] row 0 (local neighbour) at [0,E), row 1 (local centre) at [cap_edges, cap_edges+E)
 *   out_eid[E], out_t[E] in query-row-major, slot order (centre order, then newest first)
 *   assoc[out_nid[i]] = i
 *   counts[0] = M, counts[1] = E   (device int64[2])
 * Workspace: tgnx_ring_sample_ws_bytes(N, q) bytes, zero-filled before the FIRST call
 * (the kernels leave it zeroed again). */
size_t tgnx_ring_sample_ws_bytes(int64_t num_nodes, int64_t q);
int tgnx_ring_sample(const int64_t* nbr, const int64_t* eid, const float* t, int64_t num_nodes,
                     int32_t size, const int64_t* n_id, int64_t q, int64_t* assoc, int64_t* out_nid,
                     int64_t* out_ei, int64_t* out_eid, float* out_t, int64_t cap_nodes,
                     int64_t cap_edges, int64_t* counts, void* ws, size_t ws_bytes, void* stream);

/* insert (neighbor_loader.py:52-104) of events (src[i], dst[i], t[i]) with
 * e_id = cur_e_id + i, both directions; keeps the K largest e_id per node
 * (and, as the reference does at :100, the K largest t values separately);
 * assoc[unique touched nodes, sorted] = rank.  B <= tgnx_ring_insert_max_batch().
 * Canonical rule for a node with > K entries in one call: the K newest survive. */
int tgnx_ring_insert_max_batch(void);
int tgnx_ring_insert(int64_t* nbr, int64_t* eid, float* t, int64_t num_nodes, int32_t size,
                     const int64_t* src, const int64_t* dst, const float* ev_t, int64_t B,
                     int64_t cur_e_id, int64_t* assoc, void* stream);

/* ------------------------------------------------------------------------
 * Negative destinations — NegLinkSamplerDest.sample (neg_sampler.py:8-23):
 * uniform over dst_nodes[n_dst], redrawn where equal to pos[i].  Counter-based
 * RNG keyed by (seed, offset + i, attempt): replayable, graph-safe.
 * ------------------------------------------------------------------------ */
int tgnx_neg_sample(const int64_t* dst_nodes, int64_t n_dst, const int64_t* pos, int64_t B,
                    uint64_t seed, uint64_t offset, int64_t* out, void* stream);

/* ------------------------------------------------------------------------
 * Dependency blocks — get_block / dependecyAwareBatch (dependencyGraph.py:8-49),
 * host (CPU, single pass, O(E)) and device versions: per batch of `batch`
 * consecutive events, block = 1 + max(last[src], last[dst]).
 * ------------------------------------------------------------------------ */
int tgnx_block_ids_host(const int64_t* src, const int64_t* dst, int64_t num_events, int64_t batch,
                        int64_t* out);

/* ------------------------------------------------------------------------
 * Kernel probe (measurement only): while enabled, every launch of kernel
 * `kernel_id` (TGNX_K_*) is timed on its launch stream — TGN launches by a pair
 * of hipEvents bound to the dispatch itself (hipExtLaunchKernelGGL start / stop:
 * the kernel's begin / end timestamps, as rocprofv3 --kernel-trace reports),
 * other launches by marker events around them (dispatch included);
 * tgnx_probe_read waits for them and returns the summed duration (ms) and the
 * launch count, then clears.  Off by default.
 * ------------------------------------------------------------------------ */
#define TGNX_K_EDGE_FWD 1       /* tgnn_edge_fwd  */
#define TGNX_K_EDGE_BWD 2       /* tgnn_edge_bwd  */
#define TGNX_K_ASSEMBLE 3
#define TGNX_K_PRED 4
#define TGNX_K_FINISH 5
#define TGNX_K_SEG_FWD 6        /* tgnn_seg_fwd (train and eval) */
#define TGNX_K_ADAM 7
#define TGNX_K_SEG_BWD 8        /* tgnn_seg_bwd */
#define TGNX_K_EDGE_META 9      /* tgnn_edge_meta */
#define TGNX_K_KV 10             /* TGN: kv_reduce ‖ dW_edge ‖ dEnc·W_e launch */
#define TGNX_K_PROJ 11           /* TGN: q / k / v / skip projections launch */
#define TGNX_K_WGRAD3 12         /* TGN: dW_gru ‖ dX_enc ‖ message stores ‖ descriptor snapshot launch */
int tgnx_probe_enable(int32_t kernel_id);
int tgnx_probe_read(double* total_ms, int64_t* launches);
/* Workgroup timeline stamps (diagnostic; measurement only): a library built with -DTGNX_STAMPS records, for
 * wave 0 of every workgroup of the TGN step's kernels, {start, end} (s_memrealtime ticks, 100 MHz), kernel
 * id, block and XCC as 32-byte records into `buf`: 64 shards (by block) of cap / 64 records, shard s at
 * record s * (cap / 64); tgnx_stamps_count returns the fullest shard's count (tools/stamps.py).  buf = NULL
 * stops recording.  Without the flag: tgnx_stamps_set returns TGNX_EINVAL and tgnx_stamps_count -1. */
int tgnx_stamps_set(void* buf, uint32_t cap);
int64_t tgnx_stamps_count(void);


/* ------------------------------------------------------------------------
 * TGNN step — the running reference model (model_utils.py:14-237, 422-697) and
 * its epoch loop (epoch_utils.py:15-318), fused.
 *
 * The per-dependency-block loop of model_utils.py:68-157 is evaluated for all
 * blocks of a batch in one parallel pass: every (row, block) embedding is a
 * segment whose in-edges are the root's ring row (sampled at batch start),
 * its self-loop (ones features, t = 0; epoch_utils.py:246-250) and the
 * intra-batch edges of earlier blocks (model_utils.py:151-157); time_assoc as
 * of block i is reconstructed per source node from the batch's sorted touch
 * list.  EdgeGATConv runs in its exact collapsed form: only
 * U_e = attn_e·W_e, U_{l,r} = attn_{l,r}·W_n reach the output (ft is [N,H,1],
 * :560-563), so the embedding is drop(mem) + (1/H)·Σ_h ft_h.
 *
 * ctl is a device int64[TGNX_CTL_WORDS] (24) control block (see TGNX_CTL_*); every kernel of a
 * step reads the batch geometry from it, so a step can be replayed from a
 * HIP graph.  The model's parameters live in one flat fp32 buffer laid out by
 * tgnx_tgnn_param_layout (names = the reference's state_dict keys).
 * ------------------------------------------------------------------------ */
#define TGNX_CTL_BATCH_START 0  /* offset of the batch's first event in the ev_* arrays */
#define TGNX_CTL_CUR_EID 1      /* e_id of that event (neighbor_loader.py:59) */
#define TGNX_CTL_B 2            /* events in the batch (global batch under DP) */
#define TGNX_CTL_GEN 3          /* node-map generation stamp */
#define TGNX_CTL_ADAM_T 4       /* optimizer step count */
#define TGNX_CTL_S 5            /* segments (rows) assembled */
#define TGNX_CTL_E 6            /* edges assembled (train) */
#define TGNX_CTL_LO 7           /* this rank's event slice [lo, hi) */
#define TGNX_CTL_HI 8
#define TGNX_CTL_SEED 9         /* per-batch RNG seed (dropout) */
#define TGNX_CTL_NB 10          /* batches advanced since the last reset */
#define TGNX_CTL_ERR 11         /* device-side error flags (0 = ok) */
#define TGNX_CTL_LOSS 12        /* (double) running sum of loss * B (epoch_utils.py:310) */
#define TGNX_CTL_SUM_E 13       /* running sum of assembled edges (roofline units) */
#define TGNX_CTL_SUM_S 14       /* running sum of assembled segments */
/* 15: internal (fused-Adam step scalars) */
#define TGNX_CTL_STEP_B 16      /* B of the last trained step (tgnx_tgnn_advance / the resident step's last
                                   launch): what tgnx_tgn_train_update checks, since a pipelined step's
                                   descriptor already holds the NEXT batch when its update runs */
#define TGNX_CTL_APPLY 17       /* TGNN resident world-1 step: Adam step count of the update still to apply
                                   (tgnx_tgnn_train_step_resident defers it to the next step's first launch), 0: none */
#define TGNX_CTL_WORDS 24

#define TGNX_TGNN_NPARAM 15     /* te_w te_b attn_l attn_r attn_e Wn bn We be Ws bs Wd bd Wo bo */

typedef struct {
  int64_t num_nodes;  /* N */
  int32_t ring;       /* K = sampling.neighbor[0] */
  int32_t mem_dim;    /* D = gnn.dim_out (time_dim == D, model_utils.py:18); <= 128 */
  int32_t msg_dim;    /* d (edge-feature width); d + D <= 320 */
  int32_t heads;      /* H = gnn.att_head; 8 */
  int32_t max_batch;  /* capacity of B (global batch); <= 2730 */
  int32_t max_neg;    /* capacity of negatives per event (1 train, K' eval) */
  float feat_drop;    /* 0.6 in the reference (model_utils.py:664) */
  float attn_drop;    /* 0.6 (model_utils.py:665) */
  float lr, beta1, beta2, eps;  /* Adam (model_utils.py:709-710) */
} tgnx_tgnn_config;

typedef struct {
  /* events, indexed like the split arrays; the batch starts at ctl[BATCH_START] */
  const int64_t* ev_src;
  const int64_t* ev_dst;
  const float* ev_t;
  const int64_t* ev_blk;   /* dependency block id of each event */
  const float* ev_msg;     /* [*, d] raw message of each event (intra-batch edge features) */
  int64_t* neg;            /* [*, Kn] negatives, same indexing (train: written by the step) */
  const int64_t* dst_nodes;/* unique destinations for train negatives */
  int64_t n_dst;
  const float* feat;       /* feature table indexed by ring e_id [*, d] (epoch_utils.py:224) */
  int64_t* nbr;            /* ring state (neighbor_loader.py:19-22) */
  int64_t* eid;
  float* rt;
  int64_t* assoc;
  float* time_assoc;       /* [N] model_utils.py:22 */
  const float* memory;     /* [N, D] model_utils.py:270 */
  float* params;           /* flat, tgnx_tgnn_param_layout */
  float* grads;            /* same layout + 1 trailing slot (batch loss) */
  float* adam_m;
  float* adam_v;
  int64_t* ctl;            /* int64[TGNX_CTL_WORDS] */
  float* out_pos;          /* [B] logits (event order in train, block order in eval) */
  float* out_neg;          /* [B*Kn] */
  double* mrr;             /* eval: per-batch MRR, indexed by ctl[NB]-1 */
  void* ws;                /* tgnx_tgnn_ws_bytes(cfg) bytes, zero-filled once */
  void* node_map;          /* int32[4*N], zero-filled once (persistent across steps) */
  float* out_ev;           /* optional (NULL: unused): [num_events, 2] train logits by event row (pos at
                              [2e], neg at [2e + 1]): the epoch's outputs for the AP / AUC display
                              (epoch_utils.py:310-317) without a copy per step */
} tgnx_tgnn_buffers;

int tgnx_tgnn_param_layout(const tgnx_tgnn_config* cfg, int64_t* offsets /* [TGNX_TGNN_NPARAM+1] */);
size_t tgnx_tgnn_ws_bytes(const tgnx_tgnn_config* cfg);
/* Byte offset in ws of the int32[TGNX_MISC_WORDS] per-step diagnostics block: [0] node runs of the
 * ring insert plan, [1] last block id; int64 phase timestamps (wall clock) from [16] in builds with
 * -DTGNX_TIMING.  Measurement only. */
#define TGNX_MISC_WORDS 64
size_t tgnx_tgnn_ws_misc_offset(const tgnx_tgnn_config* cfg);

/* Set up the next batch.  mode 0: explicit (batch_start, B, cur_e_id as given);
 * mode 1: resident (next consecutive batch of `batch` events in [split_lo, split_hi),
 * cur_e_id = the event's global index).  Increments GEN and NB; for train also ADAM_T.
 * rank/world slice the batch's rows for data parallelism. */
int tgnx_tgnn_advance(int64_t* ctl, int32_t mode, int64_t batch_start, int64_t B, int64_t cur_e_id,
                      int64_t split_lo, int64_t split_hi, int64_t batch, int32_t rank, int32_t world,
                      uint64_t base_seed, int32_t train, void* stream);

/* Train step, part 1 (epoch_utils.py:196-303 up to loss.backward): negatives (if gen_neg),
 * assembly, collapsed forward, predictor + BCE, backward; writes grads (+ loss slot).  Also applies
 * the batch's neighbor_loader.insert + time_assoc update (epoch_utils.py:304, model_utils.py:81-83)
 * once the forward has read them (nothing later in the step does). */
int tgnx_tgnn_train_fwd_bwd(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t gen_neg,
                            int32_t dropout, void* stream);
/* The same for a resident split with the batch cursor folded in (one launch fewer per step):
 * tgnx_tgnn_advance(ctl, mode 1, ..., split_lo, split_hi, batch, rank, world, base_seed, train 1) followed by
 * tgnx_tgnn_train_fwd_bwd(gen_neg 1), as one call.  The step's first launch derives the batch descriptor from the
 * step counter and publishes it; the counter advances in its second launch.  Same results (ctl words included). */
int tgnx_tgnn_train_fwd_bwd_resident(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int64_t split_lo,
                                     int64_t split_hi, int64_t batch, int32_t rank, int32_t world,
                                     uint64_t base_seed, int32_t dropout, void* stream);
/* World 1: the resident step whole — tgnx_tgnn_train_fwd_bwd_resident (rank 0 of 1) with the update deferred: the
 * step sums its loss and records its update as pending (ctl[TGNX_CTL_APPLY]); the gradient expansion + Adam run in
 * the NEXT call's first launch, beside its batch assembly (8 launches per step, no tgnx_tgnn_train_update).  The
 * parameters therefore lag one step until tgnx_tgnn_apply_pending (call it before reading them; tgnx_tgnn_eval_step
 * applies a pending update itself).  Same results as the separate update, bit for bit. */
int tgnx_tgnn_train_step_resident(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int64_t split_lo,
                                  int64_t split_hi, int64_t batch, uint64_t base_seed, int32_t dropout, void* stream);
/* Apply the update tgnx_tgnn_train_step_resident left pending, if any (two launches; a no-op on the device when
 * nothing is pending). */
int tgnx_tgnn_apply_pending(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, void* stream);
/* Train step, part 2 (optimizer.step): Adam on the (possibly all-reduced) grads, loss sum. */
int tgnx_tgnn_train_update(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, void* stream);
/* Eval step (epoch_utils.py:28-157): Kn negatives per event, logits in block order,
 * per-batch MRR (TGB rank rule), insert, time_assoc as model_utils.py:77-83 leaves it.
 * tile_quirk = 1 pairs negative row r with source r mod B (model_utils.py:192). */
int tgnx_tgnn_eval_step(const tgnx_tgnn_config* cfg, const tgnx_tgnn_buffers* buf, int32_t Kn,
                        int32_t tile_quirk, void* stream);

/* ---------------------------------------------------------------- dense fp32 GEMM
 * C[M,N] = op(A) op(B) (+ bias[N]) (+ C if accumulate) on v_mfma_f32_16x16x4_f32; K > 256 runs
 * split-K with a fixed-order (deterministic) fixup launch.  op(A)(m,k) = trans_a ? A[k*lda+m] : A[m*lda+k];
 * op(B)(k,n) = trans_b ? B[n*ldb+k] : B[k*ldb+n].  `ws` holds tgnx_gemm_f32_ws_bytes(M,N,K) bytes
 * (split partials).  Used by the TGN memory path (modules: Linear /
 * GRUCell / TransformerConv contractions); exported for tests. */
size_t tgnx_gemm_f32_ws_bytes(int64_t M, int64_t N, int64_t K);
int tgnx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int32_t trans_a, const float* B,
                  int64_t ldb, int32_t trans_b, float* C, int64_t ldc, const float* bias, int32_t accumulate,
                  void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- t-CSR temporal graph
 * TGL's ext_full.npz (indptr int64[N+1], indices int64[nnz], eid int64[nnz], ts fp32[nnz]) that
 * utils.py:73 loads (generated by tgb_gen_graph.py, README.md:5, absent from the reference) and TGL's
 * "recent" neighbour sampler (its C++ sampler_core, README.md:2, also absent).  Rows are ordered by
 * event id (= time order for a chronological stream; *chrono = 0 reports a stream whose t decreases
 * somewhere, for which only the event-id cutoff is meaningful).  Parity unpinned for TGL itself; the
 * event-id cutoff is pinned by the reference's LastNeighborLoader goldens. */
size_t tgnx_tcsr_build_ws_bytes(int64_t num_events, int32_t add_reverse);
/* events (src[e], dst[e], t[e]), e = event id; add_reverse: also the (dst -> src) entry (TGL
 * --add_reverse; LastNeighborLoader inserts both directions).  nnz = E or 2E; nnz < 2^31. */
int tgnx_tcsr_build(const int64_t* src, const int64_t* dst, const float* t, int64_t num_events, int64_t num_nodes,
                    int32_t add_reverse, int64_t* indptr, int64_t* indices, int64_t* eid, float* ts, int32_t* chrono,
                    void* ws, size_t ws_bytes, void* stream);
/* For each root q: the K most recent row entries before the cutoff, newest first, into
 * out_*[q*K + j] (j < out_cnt[q]; the rest nbr = eid = -1, t = -1):
 *   mode 0: eid < cut (cut_eid[q], or cut_eid_all when cut_eid is NULL) — LastNeighborLoader's ring
 *           row at a batch start when cut = the batch's first event id (neighbor_loader.py:52-104);
 *   mode 1: ts < cut_t[q] (TGL: strictly before the root's timestamp).
 * out_cnt may be NULL. */
int tgnx_tcsr_sample(const int64_t* indptr, const int64_t* indices, const int64_t* eid, const float* ts,
                     int64_t num_nodes, int32_t K, const int64_t* roots, int64_t Q, int32_t mode, const int64_t* cut_eid,
                     int64_t cut_eid_all, const float* cut_t, int64_t* out_nbr, int64_t* out_eid, float* out_t,
                     int32_t* out_cnt, void* stream);

/* ---------------------------------------------------------------- TGN memory path
 * SURVEY §8 a14–a16 (the PyG TGN of the reference modules/ directory, wired as pyg_model_utils.py:10-36):
 * TGNMemory (modules/memory_module.py:25-215) with IdentityMessage (msg_func.py:12-18) and
 * Last/Mean aggregation (msg_agg.py:15-26), GRUCell memory update, GraphAttentionEmbedding over
 * TransformerConv (emb_module.py:55-73, heads = 2, dropout on the attention), LinkPredictor
 * (decoder.py:12-27, sigmoid output fed to BCE-with-logits as the reference's loop does).
 * The sampler state is the LastNeighborLoader ring above; ctl is the tgnx_tgnn_advance block. */
#define TGNX_TGN_NPARAM 21
/* layers = 2 (SURVEY §8d comment config, "2-hop temporal attention"; the build's extension, no
 * reference parity): the sampler is called again on the 1-hop node set and a second TransformerConv
 * `gnn.conv2` (same shapes as `gnn.conv`) runs on the first one's output; its 9 tensors follow the
 * 21 above in the layout (lin_key w/b, lin_query w/b, lin_value w/b, lin_edge w, lin_skip w/b). */
#define TGNX_TGN_NPARAM2 30
typedef struct {
  int64_t num_nodes;
  int64_t num_events;  /* rows of the event table (e_id space, message-store arena) */
  int32_t ring, mem_dim, msg_dim, heads, max_batch, max_neg;
  int32_t aggr;        /* 0 = LastAggregator, 1 = MeanAggregator */
  float dropout, lr, beta1, beta2, eps;
  int32_t layers;      /* 1 (emb_module.py:55-73) or 2 (2-hop: conv2(conv1(x)) over the 2-hop sample) */
  int32_t updater;     /* memory updater: 0 = GRUCell (TGNMemory memory_module.py:71-72; DyRepMemory 'gru'),
                          1 = RNNCell (DyRepMemory memory_updater_type 'rnn', memory_module.py:256-259):
                          weight_ih [D, Qm], weight_hh [D, D], bias_ih / bias_hh [D] in the same layout slots */
  int32_t emb_in_msg;  /* DyRepMemory (memory_module.py:218-421): bit 0 use_src_emb_in_msg, bit 1
                          use_dst_emb_in_msg (:387-408) — update_state of src ∪ dst builds its messages with the
                          batch's embeddings in place of the memory rows of endpoints in src ∪ dst (train: the
                          train forward's, eval: the eval forward's).  0 = TGNMemory messages.  layers = 1, world 1. */
} tgnx_tgn_config;

typedef struct {
  const int64_t *ev_src, *ev_dst; /* event table [num_events] (e_id rows) */
  const float *ev_t, *ev_msg;     /* [num_events], [num_events, msg_dim] */
  int64_t* neg;                   /* train: [num_events] (written if gen_neg); eval: [num_events, Kn] */
  const int64_t* dst_nodes;
  int64_t n_dst;
  int64_t *nbr, *eid;             /* LastNeighborLoader ring [N,K] */
  float* rt;
  int64_t* assoc;                 /* [N] */
  float* memory;                  /* TGNMemory.memory [N, mem_dim] */
  int64_t* last_update;           /* TGNMemory.last_update [N] */
  int64_t* store;                 /* message stores: tgnx_tgn_store_words(cfg) int64, zero-filled once */
  int32_t* node_gen;              /* int32[N], zero-filled once */
  float *params, *grads, *adam_m, *adam_v; /* flat, tgnx_tgn_param_layout (+1 loss slot in grads) */
  int64_t* ctl;                   /* int64[TGNX_CTL_WORDS] */
  float *out_pos, *out_neg;       /* train: [B] sigmoid outputs; eval: [B], [B, Kn] */
  double* mrr;                    /* eval: per-event reciprocal ranks of the last batch [B] */
  void* ws;                       /* tgnx_tgn_ws_bytes(cfg), zero-filled once */
  float* xrows;                   /* data parallel (ctl world > 1): [xcap, TGNX_TGN_ROW(mem_dim)] rows this
                                     rank's step updated, exchanged after the step; NULL at
                                     world 1 */
  int64_t xcap;                   /* >= 2 * ceil(max_batch / world) */
  float* out_ev;                  /* optional (NULL: unused): [num_events, 2] train outputs by event row —
                                     sigmoid(pos), sigmoid(neg) of event e at [2e], [2e + 1] — so that an
                                     epoch of replayed steps leaves every batch's outputs for the AP / AUC
                                     display (pyg_epoch_utils.py:139-147) without a copy per step */
  const void* plan_table;         /* optional (NULL: unused): the plan table tgnx_tgn_plan_table built for the
                                     split / batch the resident parity-set steps run (tgnx_tgn_train_step_pp,
                                     tgnx_tgn_train_fwd_bwd_pp); they then read every batch's ring-insert and
                                     message-store plans from it and their scan is the node-set walk alone.
                                     Other calls ignore it.  Must be the table tgnx_tgn_plan_table built for
                                     the steps' split_lo / split_hi / batch and this config's max_batch: the
                                     library records that when it builds the table and the steps refuse
                                     (TGNX_EINVAL) a table it did not build or one built for another split. */
  int32_t flags;                  /* TGNX_TGN_* bits below (0: defaults) */
} tgnx_tgn_buffers;
/* tgnx_tgn_buffers.flags: the steps with Adam fused into the gradient writers (tgnx_tgn_train_step*, world 1)
 * update parameters and moments without storing the gradient in buf->grads (the batch loss slot
 * grads[P] is still written); for loops that never read the gradients (the benchmark, the drop-in train()) */
#define TGNX_TGN_NO_GRAD_STORE 1
/* exchanged memory row, all fields floats holding exact integers so that the row survives a SUM exchange
 * (one all-reduce over [gradients | every rank's row slots, zero but the sender's] is the all-gather):
 * node (-1 = unused slot; num_nodes < 2^24), last_update bits 0-23, 24-47, 48-63, memory[D] */
#define TGNX_TGN_ROW(D) ((D) + 4)

int tgnx_tgn_param_layout(const tgnx_tgn_config* cfg,
                          int64_t* offsets /* [TGNX_TGN_NPARAM+1], layers = 2: [TGNX_TGN_NPARAM2+1] */);
size_t tgnx_tgn_ws_bytes(const tgnx_tgn_config* cfg);
size_t tgnx_tgn_store_words(const tgnx_tgn_config* cfg);
/* The ring-insert plan (neighbor_loader.py:52-104: the batch's (node, event, direction) entries in node
 * order, newest first, runs per node) and the message-store plan (memory_module.py:180-191: stable per
 * (node, direction), runs) of every batch of a resident split [split_lo, split_hi) in batches of `batch`
 * (the global batch under data parallelism): a function of the event table alone, so one launch per
 * binding builds what each step's scan would otherwise sort again.  Table: tgnx_tgn_plan_table_bytes bytes
 * (a 64-B header + one slot per batch, sized by max_batch: 2 max_batch entries of 20 B each, i.e. about 40 B
 * per event of the split when batch = max_batch — ~6 MB for the tgbl-wiki train split, ~1.3 GB for a
 * tgbl-comment-sized one of 31M events); hand it to the resident parity-set steps as buf->plan_table. */
size_t tgnx_tgn_plan_table_bytes(const tgnx_tgn_config* cfg, int64_t split_lo, int64_t split_hi, int64_t batch);
int tgnx_tgn_plan_table(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo, int64_t split_hi,
                        int64_t batch, void* table, size_t table_bytes, void* stream);
/* Forget what `table` was built for (the library keeps, per table address, the split / batch it serves, and the
 * steps refuse a table built for another): call before freeing a plan table, so a later allocation at the same
 * address is not taken for it.  A (re)build forgets first and records only after its launch was issued. */
int tgnx_tgn_plan_table_release(const void* table);
/* memory = 0, last_update = 0, message stores empty (memory_module.py:106-110). */
int tgnx_tgn_reset_state(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* stream);
/* Train batch, part 1 (the canonical loop pyg_epoch_utils.py:106-137 carries commented out): negatives
 * (gen_neg), sampler, memory(n_id) with the GRU update of every sampled node, embedding,
 * link prediction, BCE, backward; then update_state (memory / last_update of src ∪ dst, message
 * stores) and the ring insert.  Writes grads (+ loss slot).
 * Data parallel (ctl rank / world from tgnx_tgnn_advance): the roots, GRU, embedding, prediction and
 * loss cover this rank's event slice only (grads are its share of the global-batch mean; sum them
 * across ranks); message stores and the ring insert replay the whole global batch (replicated);
 * the memory rows this rank updated are packed into buf->xrows for the all-gather. */
int tgnx_tgn_train_fwd_bwd(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg,
                           int32_t dropout, void* stream);
/* Train batch in one call at world 1: tgnx_tgn_train_fwd_bwd with Adam folded into the gradient writers
 * (every gradient element's writer also updates its parameter / adam_m / adam_v), equal to fwd_bwd +
 * tgnx_tgn_train_update (grads are still written).  Refused with xrows set (data parallel). */
int tgnx_tgn_train_step(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t gen_neg, int32_t dropout,
                        void* stream);
/* tgnx_tgn_train_step of the next batch of a resident split, with the batch cursor folded in: the
 * same as tgnx_tgnn_advance(ctl, mode 1, ..., split_lo, split_hi, batch, rank, world, base_seed,
 * train 1) followed by tgnx_tgn_train_step(gen_neg 1), one launch fewer.  World 1 only (Adam is folded
 * in as well; world > 1 is refused), split_hi <= num_events.
 * ctl words, in stream order: the step's second launch (the scan) writes the batch descriptor
 * (BATCH_START, B, CUR_EID, LO, HI, SEED) from the unchanged counters; the step's LAST launch advances NB,
 * GEN and (when B > 0) ADAM_T.  So once the call's work has completed, ctl equals what advance + step leave; between
 * the two (e.g. a kernel of the caller's own, enqueued in between) the counters still hold the previous
 * step's values, whereas tgnx_tgnn_advance has already advanced them. */
int tgnx_tgn_train_step_resident(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                 int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                 int32_t dropout, void* stream);
/* tgnx_tgn_train_step_resident (world 1) pipelined across steps: the step marks the NEXT batch of the split
 * inside its predictor launch (its ring insert now runs beside the GRU, before that) and scans it after its
 * own last launch, so the next pipelined call starts at the message aggregation: two launches fewer per
 * step on the critical path.  prefetched = 1: the previous call on these buffers was a pipelined step with
 * the same split / batch / seed and nothing else ran on them since; prefetched = 0: mark + scan this batch
 * first (the first step, or after any other call: eval, flush, reset, another train form, a new cursor).
 * Results equal tgnx_tgn_train_step_resident's step for step (same batches, negatives, dropout streams).
 * ctl after the call: NB / GEN / ADAM_T advanced as for the resident step; the batch descriptor words
 * (BATCH_START .. SEED) and SUM_E / SUM_S already describe / include the NEXT batch, and neg[] holds the
 * next batch's negatives.  Test: tests/test_gpu_tgn.py (pipelined vs resident). */
int tgnx_tgn_train_step_pipelined(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                  int64_t split_hi, int64_t batch, uint64_t base_seed, int32_t dropout,
                                  int32_t prefetched, void* stream);
/* tgnx_tgn_train_step_pipelined with two parities of the scan's per-batch outputs (sorted node / centre sets,
 * edge offsets, update list, insert / store plans, counts) in the workspace: a step reads set `parity`
 * while the next batch is marked in its predictor launch and scanned into set 1 - parity inside its k / v
 * reduction launch, so its last launch (split-K sums, Adam, memory update) no longer waits for the scan.
 * Alternate parity 0, 1, 0, ... across consecutive calls (two HIP graphs); prefetched as for
 * tgnx_tgn_train_step_pipelined (prefetched = 0 marks + scans this batch into set `parity` first).  A step
 * whose set holds another batch (wrong parity) sets ctl[ERR] bit 16 and computes nothing after its first
 * launch.  World 1, 1 or 2 hops (2 hops: the root level's sets are doubled too, and the next batch's node-set
 * walk rides in the dW_cell launch); other calls use set 0 and scan for themselves.  Results equal
 * tgnx_tgn_train_step_pipelined's step for step.  Test: tests/test_gpu_tgn.py (pp vs resident, both hops). */
int tgnx_tgn_train_step_pp(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                           int64_t split_hi, int64_t batch, uint64_t base_seed, int32_t dropout, int32_t prefetched,
                           int32_t parity, void* stream);
/* Data parallel form: tgnx_tgn_train_fwd_bwd with the folded cursor (the exchange, tgnx_tgn_apply_rows and
 * tgnx_tgn_train_update follow).  ctl words as for tgnx_tgn_train_step_resident: the descriptor is written
 * by the first launch, NB / GEN / ADAM_T advance in the last launch of THIS call, so they have advanced
 * by the time the exchange and tgnx_tgn_train_update (which reads ADAM_T) run — the same values the
 * advance + fwd_bwd path gives them.  Test: tests/test_gpu_tgn_dp.py (per rank, folded vs advance +
 * fwd_bwd). */
int tgnx_tgn_train_fwd_bwd_resident(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                    int64_t split_hi, int64_t batch, int32_t rank, int32_t world,
                                    uint64_t base_seed, int32_t dropout, void* stream);
/* tgnx_tgn_train_fwd_bwd_resident pipelined across steps, as tgnx_tgn_train_step_pipelined (world >= 1;
 * Adam is not folded in): the next batch (this rank's slice) is marked inside the k / v reduction launch and
 * scanned after this call's last launch, so the next call starts at the message aggregation.  The exchange
 * and tgnx_tgn_apply_rows_update follow each call (that update reads STEP_B, not B: the descriptor words
 * already describe the next batch).  prefetched as for tgnx_tgn_train_step_pipelined.  Per rank, results
 * equal tgnx_tgn_train_fwd_bwd_resident's step for step.  Test: tests/test_gpu_tgn_dp.py. */
int tgnx_tgn_train_fwd_bwd_pipelined(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                     int64_t split_hi, int64_t batch, int32_t rank, int32_t world,
                                     uint64_t base_seed, int32_t dropout, int32_t prefetched, void* stream);
/* tgnx_tgn_train_fwd_bwd_pipelined without its last launch (the next batch's scan), and that scan alone:
 * fwd_bwd_split, then the exchange started asynchronously, tgnx_tgn_scan_next on the compute stream while
 * the collective runs (the scan touches neither the exchange buffer nor what the update writes), then
 * tgnx_tgn_apply_rows_update after the exchange — the same results as the pipelined call. */
int tgnx_tgn_train_fwd_bwd_split(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                                 int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                                 int32_t dropout, int32_t prefetched, void* stream);
int tgnx_tgn_scan_next(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo, int64_t split_hi,
                       int64_t batch, int32_t rank, int32_t world, uint64_t base_seed, void* stream);
/* The data-parallel step on the parity-set design of tgnx_tgn_train_step_pp (world >= 1, 1 or 2 hops, Adam not
 * folded in): the next batch (this rank's slice) is marked in the predictor launch and scanned into set
 * 1 - parity inside the dW_cell launch; the last launch writes the gradients, packs this rank's updated
 * memory rows into buf->xrows, advances the counters and writes the next descriptor.  One step is this
 * call, then the exchange (the all-reduce of [gradients | row slots]), then tgnx_tgn_apply_rows_update —
 * which this call runs FIRST when apply_prev = 1 (rows / nrows: the whole exchanged row block), so that a
 * step is one graph [apply(k-1) ‖ step k] plus one collective.  apply_prev must be 1 exactly when the
 * previous call's exchange has not yet been applied.  prefetched / parity as tgnx_tgn_train_step_pp.
 * Test: tests/test_gpu_tgn_dp.py (per rank against the split pipelined step) and tests/test_gpu_tgn_dp_worlds.py. */
int tgnx_tgn_train_fwd_bwd_pp(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int64_t split_lo,
                              int64_t split_hi, int64_t batch, int32_t rank, int32_t world, uint64_t base_seed,
                              int32_t dropout, int32_t prefetched, int32_t parity, int32_t apply_prev, float* rows,
                              int64_t nrows, void* stream);
/* tgnx_tgn_apply_rows + tgnx_tgn_train_update in one launch (data parallel, after the exchange). */
int tgnx_tgn_apply_rows_update(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, float* rows, int64_t nrows,
                               void* stream);
/* Data parallel: write the exchanged rows of every rank (rows [nrows, TGNX_TGN_ROW(mem_dim)], slots
 * with node -1 skipped) into memory / last_update, then zero `rows` (ready for the next summing
 * exchange).  Ranks that updated the same node computed the same row (same replicated inputs), so the
 * order does not matter. */
int tgnx_tgn_apply_rows(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, float* rows, int64_t nrows,
                        void* stream);
/* Train batch, part 2: Adam on the (possibly all-reduced) grads, loss sum; nothing when the step's batch
 * (ctl STEP_B) was empty. */
int tgnx_tgn_train_update(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* stream);
/* Eval batch (TGB tgbl link prediction): every event's [pos, Kn negatives] scored with the
 * batch-start memory and ring, per-event reciprocal rank in buf->mrr, then update_state in eval
 * order (store, then GRU update) and the ring insert. */
int tgnx_tgn_eval_step(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, int32_t Kn, void* stream);
/* train(False): update the memory of every node from its stored messages, clear the stores
 * (memory_module.py:209-215).  Every row is computed from the pre-flush state (:212 updates arange(N) at
 * once).  Graphs with more nodes than the workspace's GRU row capacity run in chunks that read a snapshot
 * of memory / last_update: pass a 16-B aligned device scratch of tgnx_tgn_flush_scratch_bytes(cfg) bytes
 * (0 when one chunk holds every node; scratch may then be NULL). */
size_t tgnx_tgn_flush_scratch_bytes(const tgnx_tgn_config* cfg);
int tgnx_tgn_flush(const tgnx_tgn_config* cfg, const tgnx_tgn_buffers* buf, void* scratch, size_t scratch_bytes,
                   void* stream);

/* ---------------------------------------------------------------- per-operator entry points
 * The TGN modules' operators one call each (torch.ops.tgnx.msg_agg_last / msg_agg_mean / gru_update /
 * predictor / edge_attn_fwd / edge_attn_bwd).  The fused steps above do not call these; a caller composing
 * the modules itself does.  Row-major fp32 tensors, int64 indices. */

/* LastAggregator / MeanAggregator (modules/msg_agg.py:15-26).  mode 0 (last): out[r] = msg[argmax_r] with
 * argmax_r the FIRST message (in message order) attaining the largest t among index == r (torch_scatter
 * scatter_max), zeros and argmax_r = n_msg for a row without messages; t is int64 (t_dtype 0, the TGN
 * stores' Long t) or fp32 (t_dtype 1).  mode 1 (mean): out[r] = the messages' sum (sequential, in message
 * order) / their count, zeros for an empty row; t unused (may be NULL).  Deterministic.  An index outside
 * [0, dim_size) is dropped and counted into *n_invalid (a device int64 the caller zeroes; may be NULL).
 * argmax (device int64[dim_size]) may be NULL.  ws: tgnx_msg_agg_ws_bytes(n_msg, dim_size) bytes. */
size_t tgnx_msg_agg_ws_bytes(int64_t n_msg, int64_t dim_size);
int tgnx_msg_agg(int32_t mode, const float* msg, int64_t n_msg, int64_t dim, const int64_t* index, const void* t,
                 int32_t t_dtype, int64_t dim_size, float* out, int64_t* argmax, int64_t* n_invalid, void* ws,
                 size_t ws_bytes, void* stream);

/* TGNMemory.memory_updater (modules/memory_module.py:57,70-78,172): h_out[M,D] = GRUCell (cell 0; weights
 * w_ih [3D,d_in], w_hh [3D,D], torch's r,z,n chunk order) or RNNCell with tanh (cell 1; w_ih [D,d_in],
 * w_hh [D,D]) of x [M,d_in] and h [M,D].  Biases may be NULL.  ws: tgnx_memory_cell_ws_bytes bytes. */
size_t tgnx_memory_cell_ws_bytes(int64_t M, int64_t d_in, int64_t D);
int tgnx_memory_cell(int32_t cell, int64_t M, int64_t d_in, int64_t D, const float* x, const float* h,
                     const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* h_out,
                     void* ws, size_t ws_bytes, void* stream);

/* LinkPredictor (modules/decoder.py:12-27, sigmoid = 1) and EdgePredictor (model_utils.py:165-195,
 * sigmoid = 0: logits): out[i] = w_out · relu(W_src z_src[i mod n_src] + b_src + W_dst z_dst[i] + b_dst) +
 * b_out for i < M (M = n_src: the positive pairs; M = n_src * k: EdgePredictor's `tile` pairing of negative
 * row i with source i mod B, model_utils.py:190).  W_src, W_dst [D,d_in]; w_out [D]; b_out [1]; b_src /
 * b_dst may be NULL.  ws: tgnx_link_predictor_ws_bytes bytes. */
size_t tgnx_link_predictor_ws_bytes(int64_t n_src, int64_t M, int64_t d_in, int64_t D);
int tgnx_link_predictor(int64_t n_src, int64_t M, int64_t d_in, int64_t D, const float* z_src, const float* z_dst,
                        const float* w_src, const float* b_src, const float* w_dst, const float* b_dst,
                        const float* w_out, const float* b_out, int32_t sigmoid, float* out, void* ws,
                        size_t ws_bytes, void* stream);

/* TransformerConv's attention (modules/emb_module.py:21-29; PyG TransformerConv, concat, no beta): for
 * destination i with incoming edges p in [indptr[i], indptr[i+1]) (rows of the per-edge k, v, e [E, H*C];
 * q [n_dst, H*C]), per head h: a_p = q_i·(k_p + e_p) / sqrt(C), α = softmax over i's edges (max subtracted,
 * + 1e-16 in the denominator), out_i = Σ_p α_p (v_p + e_p) (the root weight / skip is the caller's Linear).
 * e may be NULL (no edge features).  alpha [E, H] is written.  1 <= heads <= 8, heads * C <= 256.  indptr is
 * clamped to [0, n_edges].  No attention dropout (eval, or dropout 0).
 * Backward: dq [n_dst, H*C], dk / dv / de [E, H*C] (de = dk + dv, needed only with e) from dout and alpha. */
int tgnx_edge_attn_fwd(int64_t n_dst, int64_t n_edges, int32_t heads, int32_t channels, const float* q,
                       const float* k, const float* v, const float* e, const int64_t* indptr, float* out,
                       float* alpha, void* stream);
int tgnx_edge_attn_bwd(int64_t n_dst, int64_t n_edges, int32_t heads, int32_t channels, const float* dout,
                       const float* q, const float* k, const float* v, const float* e, const int64_t* indptr,
                       const float* alpha, float* dq, float* dk, float* dv, float* de, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TGNX_H */
