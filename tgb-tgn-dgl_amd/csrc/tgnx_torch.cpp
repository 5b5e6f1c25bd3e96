// torch.ops.tgnx — the C ABI of libtgnx (include/tgnx.h) registered as PyTorch operators (SURVEY §8b:
// "wrapped by TORCH_LIBRARY(tgnx, ...) ops").  Host code only: every op checks its tensors, allocates its
// outputs / workspace through PyTorch's caching allocator and calls the C entry point on the current HIP
// stream; errors raise RuntimeError with tgnx_last_error().  The fused TGN / TGNN steps keep their struct
// interface (tgnx_tgn_config / tgnx_tgn_buffers, driven by tgnx/tgn.py); these ops are the building blocks a
// torch caller composes directly:
//
//   ring_reset / ring_sample / ring_insert   LastNeighborLoader reset_state / __call__ / insert
//                                            (neighbor_loader.py:106-109, :26-50, :52-104)
//   neg_sample                               NegLinkSamplerDest.sample (neg_sampler.py:8-23)
//   block_ids                                get_block / dependecyAwareBatch (dependencyGraph.py:8-49), CPU
//   tcsr_build / tcsr_sample                 TGL's ext_full.npz + recent sampler (utils.py:73, README.md:2-5)
//   gemm_f32                                 the modules' Linear contractions on the MFMA GEMM
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
}
