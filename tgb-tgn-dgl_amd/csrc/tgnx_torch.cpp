// torch.ops.tgnx — the C ABI of libtgnx (include/tgnx.h) registered as PyTorch operators (SURVEY §8b:
// "wrapped by TORCH_LIBRARY(tgnx, ...) ops").  Host code only: every op checks its tensors, allocates its
// outputs / workspace through PyTorch's caching allocator and calls the C entry point on the current HIP
// stream; errors raise RuntimeError with tgnx_last_error().  The fused TGN / TGNN steps keep their struct
// interface (tgnx_tgn_config / tgnx_tgn_buffers, driven by tgnx/tgn.py); these ops are the building blocks a
// torch caller composes directly:
//
//   ring_reset / ring_sample / ring_insert   LastNeighborLoader reset_state / __call__ / insert
//                                            (neighbor_loader.py:106-109, :26-50, :52-104); also registered under
//                                            SURVEY §8b's names reset / sample_recent / insert_recent
//   neg_sample                               NegLinkSamplerDest.sample (neg_sampler.py:8-23)
//   block_ids                                get_block / dependecyAwareBatch (dependencyGraph.py:8-49), CPU
//   tcsr_build / tcsr_sample                 TGL's ext_full.npz + recent sampler (utils.py:73, README.md:2-5)
//   gemm_f32                                 the modules' Linear contractions on the MFMA GEMM
//   msg_agg_last / msg_agg_mean              LastAggregator / MeanAggregator (modules/msg_agg.py:15-26)
//   gru_update                               TGNMemory.memory_updater GRUCell / RNNCell (memory_module.py:70-78)
//   predictor                                LinkPredictor (decoder.py:12-27) / EdgePredictor (model_utils.py:165-195)
//   edge_attn_fwd / edge_attn_bwd            TransformerConv's attention (emb_module.py:21-29, PyG semantics)
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <initializer_list>
#include <tuple>

#include "../../include/tgnx.h"

namespace {

// the current stream OF THE CURRENT DEVICE: every op first makes its tensors' device current (a device guard,
// restored on return), so the launch goes to that device's stream with that device's pointers
void* cur_stream() { return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream().stream()); }

// every device tensor of an op on one device (the one its guard selects)
void same_device(const at::Tensor& ref, std::initializer_list<const at::Tensor*> xs) {
  for (const at::Tensor* x : xs)
    TORCH_CHECK(x->device() == ref.device(), "tgnx: all tensors of an op must be on one device: ", ref.device(),
                " and ", x->device());
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == TGNX_OK, what, " failed (", rc, "): ", tgnx_last_error());
}

void dev_tensor(const at::Tensor& x, at::ScalarType st, const char* name) {
  TORCH_CHECK(x.is_cuda(), name, " must be a HIP device tensor");
  TORCH_CHECK(x.scalar_type() == st, name, " has dtype ", x.scalar_type(), ", expected ", st);
  TORCH_CHECK(x.is_contiguous(), name, " must be contiguous");
}

void ring_state(const at::Tensor& nbr, const at::Tensor& eid, const at::Tensor& t) {
  dev_tensor(nbr, at::kLong, "nbr");
  dev_tensor(eid, at::kLong, "e_id");
  dev_tensor(t, at::kFloat, "t");
  TORCH_CHECK(nbr.dim() == 2 && eid.sizes() == nbr.sizes() && t.sizes() == nbr.sizes(),
              "ring tensors must be [num_nodes, size]");
}

void ring_reset(at::Tensor eid, at::Tensor t) {
  dev_tensor(eid, at::kLong, "e_id");
  dev_tensor(t, at::kFloat, "t");
  TORCH_CHECK(eid.dim() == 2 && t.sizes() == eid.sizes(), "ring tensors must be [num_nodes, size]");
  same_device(eid, {&t});
  const c10::OptionalDeviceGuard guard(eid.device());
  check_rc(tgnx_ring_reset(eid.data_ptr<int64_t>(), t.data_ptr<float>(), eid.size(0), (int32_t)eid.size(1),
                           cur_stream()),
           "tgnx_ring_reset");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> ring_sample(const at::Tensor& nbr, const at::Tensor& eid,
                                                                       const at::Tensor& t, at::Tensor assoc,
                                                                       const at::Tensor& n_id) {
  ring_state(nbr, eid, t);
  dev_tensor(assoc, at::kLong, "assoc");
  dev_tensor(n_id, at::kLong, "n_id");
  same_device(nbr, {&eid, &t, &assoc, &n_id});
  const c10::OptionalDeviceGuard guard(nbr.device());
  const int64_t N = nbr.size(0), K = nbr.size(1), q = n_id.numel();
  TORCH_CHECK(assoc.numel() == N, "assoc must have num_nodes entries");
  const int64_t cap_n = std::max<int64_t>(q * (1 + K), 1), cap_e = std::max<int64_t>(q * K, 1);
  auto lopt = n_id.options();
  at::Tensor out_nid = at::empty({cap_n}, lopt), out_ei = at::empty({2 * cap_e}, lopt);
  at::Tensor out_eid = at::empty({cap_e}, lopt), out_t = at::empty({cap_e}, t.options());
  at::Tensor counts = at::zeros({2}, lopt);
  const size_t nb = tgnx_ring_sample_ws_bytes(N, q);
  at::Tensor ws = at::zeros({(int64_t)std::max<size_t>(nb, 1)}, n_id.options().dtype(at::kByte));
  check_rc(tgnx_ring_sample(nbr.data_ptr<int64_t>(), eid.data_ptr<int64_t>(), t.data_ptr<float>(), N, (int32_t)K,
                            n_id.data_ptr<int64_t>(), q, assoc.data_ptr<int64_t>(), out_nid.data_ptr<int64_t>(),
                            out_ei.data_ptr<int64_t>(), out_eid.data_ptr<int64_t>(), out_t.data_ptr<float>(), cap_n,
                            cap_e, counts.data_ptr<int64_t>(), ws.data_ptr(), nb, cur_stream()),
           "tgnx_ring_sample");
  const at::Tensor c = counts.cpu();  // one device -> host sync, as the reference's unique()
  const int64_t M = c.data_ptr<int64_t>()[0], E = c.data_ptr<int64_t>()[1];
  return {out_nid.narrow(0, 0, M), out_ei.view({2, cap_e}).narrow(1, 0, E), out_eid.narrow(0, 0, E),
          out_t.narrow(0, 0, E)};
}

void ring_insert(at::Tensor nbr, at::Tensor eid, at::Tensor t, const at::Tensor& src, const at::Tensor& dst,
                 const at::Tensor& ev_t, int64_t cur_e_id, at::Tensor assoc) {
  ring_state(nbr, eid, t);
  dev_tensor(src, at::kLong, "src");
  dev_tensor(dst, at::kLong, "dst");
  dev_tensor(ev_t, at::kFloat, "ev_t");
  dev_tensor(assoc, at::kLong, "assoc");
  same_device(nbr, {&eid, &t, &src, &dst, &ev_t, &assoc});
  const c10::OptionalDeviceGuard guard(nbr.device());
  const int64_t B = src.numel();
  TORCH_CHECK(dst.numel() == B && ev_t.numel() == B, "src, dst, ev_t must have the same length");
  TORCH_CHECK(B <= tgnx_ring_insert_max_batch(), "batch ", B, " > ", tgnx_ring_insert_max_batch());
  check_rc(tgnx_ring_insert(nbr.data_ptr<int64_t>(), eid.data_ptr<int64_t>(), t.data_ptr<float>(), nbr.size(0),
                            (int32_t)nbr.size(1), src.data_ptr<int64_t>(), dst.data_ptr<int64_t>(),
                            ev_t.data_ptr<float>(), B, cur_e_id, assoc.data_ptr<int64_t>(), cur_stream()),
           "tgnx_ring_insert");
}

at::Tensor neg_sample(const at::Tensor& dst_nodes, const at::Tensor& pos, int64_t seed, int64_t offset) {
  dev_tensor(dst_nodes, at::kLong, "dst_nodes");
  dev_tensor(pos, at::kLong, "pos");
  TORCH_CHECK(dst_nodes.numel() > 0, "empty destination set");
  same_device(dst_nodes, {&pos});
  const c10::OptionalDeviceGuard guard(dst_nodes.device());
  at::Tensor out = at::empty_like(pos);
  check_rc(tgnx_neg_sample(dst_nodes.data_ptr<int64_t>(), dst_nodes.numel(), pos.data_ptr<int64_t>(), pos.numel(),
                           (uint64_t)seed, (uint64_t)offset, out.data_ptr<int64_t>(), cur_stream()),
           "tgnx_neg_sample");
  return out;
}

at::Tensor block_ids(const at::Tensor& src, const at::Tensor& dst, int64_t batch) {
  TORCH_CHECK(!src.is_cuda() && !dst.is_cuda(), "block_ids runs on host tensors (dependencyGraph.py is CPU code)");
  const at::Tensor s = src.to(at::kLong).contiguous(), d = dst.to(at::kLong).contiguous();
  TORCH_CHECK(s.numel() == d.numel(), "src and dst must have the same length");
  at::Tensor out = at::empty_like(s);
  check_rc(tgnx_block_ids_host(s.data_ptr<int64_t>(), d.data_ptr<int64_t>(), s.numel(), batch,
                               out.data_ptr<int64_t>()),
           "tgnx_block_ids_host");
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, bool> tcsr_build(const at::Tensor& src,
                                                                             const at::Tensor& dst,
                                                                             const at::Tensor& t, int64_t num_nodes,
                                                                             bool add_reverse) {
  dev_tensor(src, at::kLong, "src");
  dev_tensor(dst, at::kLong, "dst");
  dev_tensor(t, at::kFloat, "t");
  same_device(src, {&dst, &t});
  const c10::OptionalDeviceGuard guard(src.device());
  const int64_t E = src.numel(), nnz = add_reverse ? 2 * E : E;
  auto lopt = src.options();
  at::Tensor indptr = at::empty({num_nodes + 1}, lopt), indices = at::empty({std::max<int64_t>(nnz, 1)}, lopt);
  at::Tensor eid = at::empty({std::max<int64_t>(nnz, 1)}, lopt), ts = at::empty({std::max<int64_t>(nnz, 1)}, t.options());
  at::Tensor chrono = at::zeros({1}, lopt.dtype(at::kInt));
  const size_t nb = tgnx_tcsr_build_ws_bytes(E, add_reverse ? 1 : 0);
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, lopt.dtype(at::kByte));
  check_rc(tgnx_tcsr_build(src.data_ptr<int64_t>(), dst.data_ptr<int64_t>(), t.data_ptr<float>(), E, num_nodes,
                           add_reverse ? 1 : 0, indptr.data_ptr<int64_t>(), indices.data_ptr<int64_t>(),
                           eid.data_ptr<int64_t>(), ts.data_ptr<float>(), chrono.data_ptr<int32_t>(), ws.data_ptr(), nb,
                           cur_stream()),
           "tgnx_tcsr_build");
  const bool chr = chrono.cpu().data_ptr<int32_t>()[0] != 0;
  return {indptr, indices.narrow(0, 0, nnz), eid.narrow(0, 0, nnz), ts.narrow(0, 0, nnz), chr};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tcsr_sample(const at::Tensor& indptr,
                                                                       const at::Tensor& indices,
                                                                       const at::Tensor& eid, const at::Tensor& ts,
                                                                       int64_t K, const at::Tensor& roots,
                                                                       int64_t mode, const at::Tensor& cut) {
  dev_tensor(indptr, at::kLong, "indptr");
  dev_tensor(indices, at::kLong, "indices");
  dev_tensor(eid, at::kLong, "eid");
  dev_tensor(ts, at::kFloat, "ts");
  dev_tensor(roots, at::kLong, "roots");
  TORCH_CHECK(mode == 0 || mode == 1, "mode 0 (event-id cutoff) or 1 (time cutoff)");
  dev_tensor(cut, mode == 0 ? at::kLong : at::kFloat, "cut");
  same_device(indptr, {&indices, &eid, &ts, &roots, &cut});
  const c10::OptionalDeviceGuard guard(indptr.device());
  const int64_t Q = roots.numel();
  TORCH_CHECK(cut.numel() == Q, "one cutoff per root");
  auto lopt = roots.options();
  at::Tensor nbr = at::empty({Q, K}, lopt), oe = at::empty({Q, K}, lopt), ot = at::empty({Q, K}, ts.options());
  at::Tensor cnt = at::empty({Q}, lopt.dtype(at::kInt));
  check_rc(tgnx_tcsr_sample(indptr.data_ptr<int64_t>(), indices.data_ptr<int64_t>(), eid.data_ptr<int64_t>(),
                            ts.data_ptr<float>(), indptr.numel() - 1, (int32_t)K, roots.data_ptr<int64_t>(), Q,
                            (int32_t)mode, mode == 0 ? cut.data_ptr<int64_t>() : nullptr, 0,
                            mode == 1 ? cut.data_ptr<float>() : nullptr, nbr.data_ptr<int64_t>(), oe.data_ptr<int64_t>(),
                            ot.data_ptr<float>(), cnt.data_ptr<int32_t>(), cur_stream()),
           "tgnx_tcsr_sample");
  return {nbr, oe, ot, cnt};
}

at::Tensor gemm_f32(const at::Tensor& A, const at::Tensor& B, const c10::optional<at::Tensor>& bias, bool trans_a,
                    bool trans_b) {
  dev_tensor(A, at::kFloat, "A");
  dev_tensor(B, at::kFloat, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "A and B must be 2-D");
  same_device(A, {&B});
  const c10::OptionalDeviceGuard guard(A.device());
  const int64_t M = trans_a ? A.size(1) : A.size(0), K = trans_a ? A.size(0) : A.size(1);
  const int64_t KB = trans_b ? B.size(1) : B.size(0), N = trans_b ? B.size(0) : B.size(1);
  TORCH_CHECK(K == KB, "inner dimensions differ: ", K, " vs ", KB);
  const float* bp = nullptr;
  if (bias.has_value()) {
    dev_tensor(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "bias must have N entries");
    same_device(A, {&*bias});
    bp = bias->data_ptr<float>();
  }
  at::Tensor C = at::empty({M, N}, A.options());
  const size_t nb = tgnx_gemm_f32_ws_bytes(M, N, K);
  at::Tensor ws = at::empty({(int64_t)nb}, A.options().dtype(at::kByte));
  check_rc(tgnx_gemm_f32(M, N, K, A.data_ptr<float>(), A.size(1), trans_a ? 1 : 0, B.data_ptr<float>(), B.size(1),
                         trans_b ? 1 : 0, C.data_ptr<float>(), N, bp, 0, ws.data_ptr(), nb, cur_stream()),
           "tgnx_gemm_f32");
  return C;
}

const float* opt_ptr(const c10::optional<at::Tensor>& x, const at::Tensor& ref, int64_t numel, const char* name) {
  if (!x.has_value()) return nullptr;
  dev_tensor(*x, at::kFloat, name);
  TORCH_CHECK(x->numel() == numel, name, " must have ", numel, " entries");
  same_device(ref, {&*x});
  return x->data_ptr<float>();
}

// out-of-range index -> RuntimeError, as the reference's scatter (one device -> host read of the drop count)
std::tuple<at::Tensor, at::Tensor> msg_agg(int32_t mode, const at::Tensor& msg, const at::Tensor& index,
                                           const at::Tensor* t, int64_t dim_size) {
  dev_tensor(msg, at::kFloat, "msg");
  dev_tensor(index, at::kLong, "index");
  TORCH_CHECK(msg.dim() == 2, "msg must be [n_msg, dim]");
  TORCH_CHECK(index.dim() == 1 && index.numel() == msg.size(0), "index must be [n_msg]");
  TORCH_CHECK(dim_size >= 0, "dim_size must be non-negative");
  int32_t t_dtype = 0;
  if (t) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->numel() == msg.size(0), "t must be a contiguous [n_msg] device tensor");
    TORCH_CHECK(t->scalar_type() == at::kLong || t->scalar_type() == at::kFloat, "t must be int64 or float32");
    t_dtype = t->scalar_type() == at::kLong ? 0 : 1;
    same_device(msg, {t});
  }
  same_device(msg, {&index});
  const c10::OptionalDeviceGuard guard(msg.device());
  const int64_t n = msg.size(0), dim = msg.size(1);
  at::Tensor out = at::empty({dim_size, dim}, msg.options());
  at::Tensor arg = at::empty({dim_size}, index.options());
  at::Tensor bad = at::zeros({1}, index.options());
  const size_t nb = tgnx_msg_agg_ws_bytes(n, dim_size);
  at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, index.options().dtype(at::kByte));
  check_rc(tgnx_msg_agg(mode, msg.data_ptr<float>(), n, dim, index.data_ptr<int64_t>(), t ? t->data_ptr() : nullptr,
                        t_dtype, dim_size, out.data_ptr<float>(), arg.data_ptr<int64_t>(), bad.data_ptr<int64_t>(),
                        ws.data_ptr(), nb, cur_stream()),
           "tgnx_msg_agg");
  const int64_t nbad = bad.cpu().data_ptr<int64_t>()[0];
  TORCH_CHECK(nbad == 0, "msg_agg: ", nbad, " index entries outside [0, ", dim_size, ")");
  return {out, arg};
}

std::tuple<at::Tensor, at::Tensor> msg_agg_last(const at::Tensor& msg, const at::Tensor& index, const at::Tensor& t,
                                                int64_t dim_size) {
  return msg_agg(0, msg, index, &t, dim_size);
}

at::Tensor msg_agg_mean(const at::Tensor& msg, const at::Tensor& index, int64_t dim_size) {
  return std::get<0>(msg_agg(1, msg, index, nullptr, dim_size));
}

at::Tensor gru_update(const at::Tensor& x, const at::Tensor& h, const at::Tensor& w_ih, const at::Tensor& w_hh,
                      const c10::optional<at::Tensor>& b_ih, const c10::optional<at::Tensor>& b_hh, int64_t cell) {
  dev_tensor(x, at::kFloat, "x");
  dev_tensor(h, at::kFloat, "h");
  dev_tensor(w_ih, at::kFloat, "w_ih");
  dev_tensor(w_hh, at::kFloat, "w_hh");
  TORCH_CHECK(cell == 0 || cell == 1, "cell 0 (GRUCell) or 1 (RNNCell, tanh)");
  TORCH_CHECK(x.dim() == 2 && h.dim() == 2 && x.size(0) == h.size(0), "x [M, d_in] and h [M, D]");
  const int64_t M = x.size(0), d_in = x.size(1), D = h.size(1), G = (cell == 0 ? 3 : 1) * D;
  TORCH_CHECK(w_ih.dim() == 2 && w_ih.size(0) == G && w_ih.size(1) == d_in, "w_ih must be [", G, ", ", d_in, "]");
  TORCH_CHECK(w_hh.dim() == 2 && w_hh.size(0) == G && w_hh.size(1) == D, "w_hh must be [", G, ", ", D, "]");
  same_device(x, {&h, &w_ih, &w_hh});
  const float* bi = opt_ptr(b_ih, x, G, "b_ih");
  const float* bh = opt_ptr(b_hh, x, G, "b_hh");
  const c10::OptionalDeviceGuard guard(x.device());
  at::Tensor out = at::empty_like(h);
  const size_t nb = tgnx_memory_cell_ws_bytes(M, d_in, D);
  at::Tensor ws = at::empty({(int64_t)nb}, x.options().dtype(at::kByte));
  check_rc(tgnx_memory_cell((int32_t)cell, M, d_in, D, x.data_ptr<float>(), h.data_ptr<float>(), w_ih.data_ptr<float>(),
                            w_hh.data_ptr<float>(), bi, bh, out.data_ptr<float>(), ws.data_ptr(), nb, cur_stream()),
           "tgnx_memory_cell");
  return out;
}

at::Tensor predictor(const at::Tensor& z_src, const at::Tensor& z_dst, const at::Tensor& w_src,
                     const c10::optional<at::Tensor>& b_src, const at::Tensor& w_dst,
                     const c10::optional<at::Tensor>& b_dst, const at::Tensor& w_out, const at::Tensor& b_out,
                     bool sigmoid) {
  dev_tensor(z_src, at::kFloat, "z_src");
  dev_tensor(z_dst, at::kFloat, "z_dst");
  dev_tensor(w_src, at::kFloat, "w_src");
  dev_tensor(w_dst, at::kFloat, "w_dst");
  dev_tensor(w_out, at::kFloat, "w_out");
  dev_tensor(b_out, at::kFloat, "b_out");
  TORCH_CHECK(z_src.dim() == 2 && z_dst.dim() == 2 && z_src.size(1) == z_dst.size(1), "z_src [B, d] and z_dst [M, d]");
  const int64_t B = z_src.size(0), M = z_dst.size(0), d_in = z_src.size(1), D = w_src.size(0);
  TORCH_CHECK(M == 0 || (B > 0 && M % B == 0), "z_dst rows must be a multiple of z_src rows (tile pairing)");
  TORCH_CHECK(w_src.dim() == 2 && w_src.size(1) == d_in && w_dst.dim() == 2 && w_dst.size(0) == D &&
                  w_dst.size(1) == d_in,
              "w_src / w_dst must be [D, d]");
  TORCH_CHECK(w_out.numel() == D && b_out.numel() == 1, "w_out must have D entries and b_out one");
  same_device(z_src, {&z_dst, &w_src, &w_dst, &w_out, &b_out});
  const float* bs = opt_ptr(b_src, z_src, D, "b_src");
  const float* bd = opt_ptr(b_dst, z_src, D, "b_dst");
  const c10::OptionalDeviceGuard guard(z_src.device());
  at::Tensor out = at::empty({M, 1}, z_src.options());
  const size_t nb = tgnx_link_predictor_ws_bytes(B, M, d_in, D);
  at::Tensor ws = at::empty({(int64_t)nb}, z_src.options().dtype(at::kByte));
  check_rc(tgnx_link_predictor(B, M, d_in, D, z_src.data_ptr<float>(), z_dst.data_ptr<float>(), w_src.data_ptr<float>(),
                               bs, w_dst.data_ptr<float>(), bd, w_out.data_ptr<float>(), b_out.data_ptr<float>(),
                               sigmoid ? 1 : 0, out.data_ptr<float>(), ws.data_ptr(), nb, cur_stream()),
           "tgnx_link_predictor");
  return out;
}

void attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const c10::optional<at::Tensor>& e,
               const at::Tensor& indptr, int64_t heads) {
  dev_tensor(q, at::kFloat, "q");
  dev_tensor(k, at::kFloat, "k");
  dev_tensor(v, at::kFloat, "v");
  dev_tensor(indptr, at::kLong, "indptr");
  TORCH_CHECK(q.dim() == 2 && k.dim() == 2 && v.sizes() == k.sizes() && k.size(1) == q.size(1),
              "q [n_dst, H*C], k / v [E, H*C]");
  TORCH_CHECK(heads >= 1 && q.size(1) % heads == 0, "H*C must be a multiple of heads");
  TORCH_CHECK(indptr.numel() == q.size(0) + 1, "indptr must have n_dst + 1 entries");
  same_device(q, {&k, &v, &indptr});
  if (e.has_value()) {
    dev_tensor(*e, at::kFloat, "e");
    TORCH_CHECK(e->sizes() == k.sizes(), "e must be [E, H*C]");
    same_device(q, {&*e});
  }
}

std::tuple<at::Tensor, at::Tensor> edge_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                 const c10::optional<at::Tensor>& e, const at::Tensor& indptr,
                                                 int64_t heads) {
  attn_args(q, k, v, e, indptr, heads);
  const c10::OptionalDeviceGuard guard(q.device());
  const int64_t n = q.size(0), E = k.size(0), C = q.size(1) / heads;
  at::Tensor out = at::empty_like(q), alpha = at::empty({E, heads}, q.options());
  check_rc(tgnx_edge_attn_fwd(n, E, (int32_t)heads, (int32_t)C, q.data_ptr<float>(), k.data_ptr<float>(),
                              v.data_ptr<float>(), e.has_value() ? e->data_ptr<float>() : nullptr,
                              indptr.data_ptr<int64_t>(), out.data_ptr<float>(), alpha.data_ptr<float>(), cur_stream()),
           "tgnx_edge_attn_fwd");
  return {out, alpha};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> edge_attn_bwd(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
    const c10::optional<at::Tensor>& e, const at::Tensor& indptr, const at::Tensor& alpha, int64_t heads) {
  attn_args(q, k, v, e, indptr, heads);
  dev_tensor(dout, at::kFloat, "dout");
  dev_tensor(alpha, at::kFloat, "alpha");
  TORCH_CHECK(dout.sizes() == q.sizes(), "dout must be [n_dst, H*C]");
  TORCH_CHECK(alpha.dim() == 2 && alpha.size(0) == k.size(0) && alpha.size(1) == heads, "alpha must be [E, heads]");
  same_device(q, {&dout, &alpha});
  const c10::OptionalDeviceGuard guard(q.device());
  const int64_t n = q.size(0), E = k.size(0), C = q.size(1) / heads;
  at::Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  at::Tensor de = e.has_value() ? at::empty_like(k) : at::empty({0}, k.options());
  check_rc(tgnx_edge_attn_bwd(n, E, (int32_t)heads, (int32_t)C, dout.data_ptr<float>(), q.data_ptr<float>(),
                              k.data_ptr<float>(), v.data_ptr<float>(), e.has_value() ? e->data_ptr<float>() : nullptr,
                              indptr.data_ptr<int64_t>(), alpha.data_ptr<float>(), dq.data_ptr<float>(),
                              dk.data_ptr<float>(), dv.data_ptr<float>(), e.has_value() ? de.data_ptr<float>() : nullptr,
                              cur_stream()),
           "tgnx_edge_attn_bwd");
  return {dq, dk, dv, de};
}

}  // namespace

TORCH_LIBRARY(tgnx, m) {
  m.def("ring_reset(Tensor(a!) e_id, Tensor(b!) t) -> ()", &ring_reset);
  m.def("ring_sample(Tensor nbr, Tensor e_id, Tensor t, Tensor(a!) assoc, Tensor n_id) -> (Tensor, Tensor, Tensor, Tensor)",
        &ring_sample);
  m.def("ring_insert(Tensor(a!) nbr, Tensor(b!) e_id, Tensor(c!) t, Tensor src, Tensor dst, Tensor ev_t, int cur_e_id, "
        "Tensor(d!) assoc) -> ()",
        &ring_insert);
  m.def("neg_sample(Tensor dst_nodes, Tensor pos, int seed, int offset) -> Tensor", &neg_sample);
  m.def("block_ids(Tensor src, Tensor dst, int batch) -> Tensor", &block_ids);
  m.def("tcsr_build(Tensor src, Tensor dst, Tensor t, int num_nodes, bool add_reverse) -> "
        "(Tensor, Tensor, Tensor, Tensor, bool)",
        &tcsr_build);
  m.def("tcsr_sample(Tensor indptr, Tensor indices, Tensor eid, Tensor ts, int K, Tensor roots, int mode, Tensor cut) "
        "-> (Tensor, Tensor, Tensor, Tensor)",
        &tcsr_sample);
  m.def("gemm_f32(Tensor A, Tensor B, Tensor? bias=None, bool trans_a=False, bool trans_b=False) -> Tensor", &gemm_f32);
  // SURVEY §8b's names for the sampler ops (the same functions as ring_sample / ring_insert / ring_reset)
  m.def("sample_recent(Tensor nbr, Tensor e_id, Tensor t, Tensor(a!) assoc, Tensor n_id) -> "
        "(Tensor, Tensor, Tensor, Tensor)",
        &ring_sample);
  m.def("insert_recent(Tensor(a!) nbr, Tensor(b!) e_id, Tensor(c!) t, Tensor src, Tensor dst, Tensor ev_t, "
        "int cur_e_id, Tensor(d!) assoc) -> ()",
        &ring_insert);
  m.def("reset(Tensor(a!) e_id, Tensor(b!) t) -> ()", &ring_reset);
  m.def("msg_agg_last(Tensor msg, Tensor index, Tensor t, int dim_size) -> (Tensor, Tensor)", &msg_agg_last);
  m.def("msg_agg_mean(Tensor msg, Tensor index, int dim_size) -> Tensor", &msg_agg_mean);
  m.def("gru_update(Tensor x, Tensor h, Tensor w_ih, Tensor w_hh, Tensor? b_ih=None, Tensor? b_hh=None, int cell=0) "
        "-> Tensor",
        &gru_update);
  m.def("predictor(Tensor z_src, Tensor z_dst, Tensor w_src, Tensor? b_src, Tensor w_dst, Tensor? b_dst, Tensor w_out, "
        "Tensor b_out, bool sigmoid=True) -> Tensor",
        &predictor);
  m.def("edge_attn_fwd(Tensor q, Tensor k, Tensor v, Tensor? e, Tensor indptr, int heads) -> (Tensor, Tensor)",
        &edge_attn_fwd);
  m.def("edge_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor? e, Tensor indptr, Tensor alpha, int heads) "
        "-> (Tensor, Tensor, Tensor, Tensor)",
        &edge_attn_bwd);
}
