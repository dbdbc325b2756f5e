// pybind11 bindings: torch tensors -> raw-pointer launchers of csrc/kernels/*.hip.
//
// Compiled by the host compiler against torch's headers; every op enqueues on the current HIP
// stream of the calling thread (at::hip::getCurrentHIPStream) and allocates its outputs with the
// torch caching allocator, so ops compose with torch streams and can be captured in a hipGraph.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "mlp_train.h"
#include "pde_kernels.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pde native op '", what, "' failed: ", hipGetErrorString(e));
}

#define CHECK_DEV(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be fp32")
#define CHECK_IN(x) \
  CHECK_DEV(x);     \
  CHECK_CONTIG(x)

inline uint16_t* u16(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
inline const uint16_t* cu16(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<const uint16_t*>(t->data_ptr()) : nullptr;
}
inline const float* cf32(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
inline float* f32(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

pde::Operand dense(const Tensor& t, long ld_r, long ld_k) {
  pde::Operand o{};
  o.ptr = t.data_ptr();
  o.kind = 0;
  o.ld_r = ld_r;
  o.ld_k = ld_k;
  return o;
}

pde::Operand gather(const Tensor& t, int kind, int N, int H, int W, int C, int R, int S, int stride, int pad,
                    int Ho, int Wo) {
  pde::Operand o{};
  o.ptr = t.data_ptr();
  o.kind = kind;
  o.g = pde::ConvGeom{N, H, W, C, R, S, stride, pad, Ho, Wo};
  return o;
}

// A 1x1 / stride-1 / pad-0 convolution is a plain GEMM over the NHWC activation: its operands are
// described densely, which skips the implicit-GEMM gather arithmetic entirely.
inline bool is_pointwise(int R, int S, int stride, int pad) { return R == 1 && S == 1 && stride == 1 && pad == 0; }

// Optional fp32 gradient sink: the op's weight gradient is written (or added) straight into it.
Tensor grad_sink(const optional<Tensor>& out, at::IntArrayRef shape, const Tensor& like) {
  if (out.has_value() && out->defined()) {
    CHECK_IN(*out); CHECK_F32(*out);
    TORCH_CHECK(out->sizes() == shape, "gradient sink has the wrong shape");
    return *out;
  }
  return at::empty(shape, like.options().dtype(at::kFloat));
}

// Split-K cap for a GEMM with reduction length K: at most 512 slabs, each >= 256 long, and the fp32
// slab workspace bounded to 128 MiB (the kernel picks the actual split from the tile count).
int split_cap(const pde::GemmArgs& a) {
  long cap = a.K / 128;
  const long by_mem = (128L << 20) / (4L * a.M * a.N);
  if (cap > by_mem) cap = by_mem;
  if (cap > 512) cap = 512;
  return cap < 1 ? 1 : static_cast<int>(cap);
}

// GEMM pairing (gemm_pair_begin / gemm_pair_end): while a pair is being collected, run_gemm records the
// GEMM (with its workspace) instead of launching it; gemm_pair_end launches the two recorded GEMMs as one
// pde::gemm_bf16_pair.  Used for a layer's dgrad + wgrad (ops/functional.py, models/mlp_fused.py).
struct PendingGemm {
  pde::GemmArgs args;
  Tensor ws;
  bool defer_out = false;  // problem 0 of a pair: leave its split-K slabs for the BatchNorm backward (conv_dgrad)
};
thread_local bool g_collect = false;
thread_local std::vector<PendingGemm> g_pending;

void run_gemm(pde::GemmArgs& a, const Tensor& like, int max_split) {
  Tensor ws;
  a.workspace = nullptr;
  a.splitk = 1;
  if (max_split < 0) max_split = split_cap(a);
  if (max_split > 1) {
    ws = at::empty({static_cast<long>(max_split) * a.M * a.N}, like.options().dtype(at::kFloat));
    a.workspace = ws.data_ptr<float>();
    a.splitk = max_split;
  }
  if (g_collect) {
    TORCH_CHECK(g_pending.size() < 2, "gemm pair: more than two GEMMs collected");
    g_pending.push_back({a, ws});
    return;
  }
  check(pde::gemm_bf16(a, cur_stream()), "gemm");
}

// ---- conv outputs left as unreduced split-K slabs for the BatchNorm that follows (conv_fwd(defer=true)) ----
// The one-launch BatchNorm sums the slabs itself (bn_fwd): the GEMM's reduce launch is gone.  Any other op
// that reads such an output first resolves it (resolve_pending: the plain reduce), so a deferred output is
// never read unreduced.  The entry keeps the slab workspace alive until it is consumed.
struct PendingConv {
  Tensor ws;
  int splits, M, N;
};
std::unordered_map<const void*, PendingConv> g_pending_conv;
std::mutex g_pending_mu;  // forward ops (main thread) and backward ops (autograd's device thread)

void resolve_pending(const Tensor& t) {
  if (!t.defined()) return;
  std::lock_guard<std::mutex> lk(g_pending_mu);
  if (g_pending_conv.empty()) return;
  auto it = g_pending_conv.find(t.data_ptr());
  if (it == g_pending_conv.end()) return;
  PendingConv pc = std::move(it->second);
  g_pending_conv.erase(it);
  check(pde::gemm_reduce_slabs_bf16(pc.ws.data_ptr<float>(), pc.splits, pc.M, pc.N,
                                    reinterpret_cast<uint16_t*>(t.data_ptr()), cur_stream()),
        "resolve_pending");
}
void resolve_pending(const optional<Tensor>& t) {
  if (t.has_value()) resolve_pending(*t);
}
int pending_conv_count() { return static_cast<int>(g_pending_conv.size()); }
std::atomic<long> g_bn_bwd_slab_uses{0};  // BatchNorm backwards that summed a deferred dgrad's slabs (tests)
long bn_bwd_slab_uses() { return g_bn_bwd_slab_uses.load(); }

void gemm_pair_begin() {
  TORCH_CHECK(!g_collect && g_pending.empty(), "gemm_pair_begin: a pair is already being collected");
  g_collect = true;
}

// Deferred weight-gradient reductions (gemm_pair_end(defer=true)): the second GEMM of a pair (a weight
// gradient accumulated into .grad, read only by the optimizer / all-reduce) leaves its split-K slabs for
// ONE batched reduce launch, gemm_flush_deferred(), at the end of backward (ops/functional.py).  The slabs
// stay alive here until then; the flush runs on the stream that produced them.
struct DeferredReduce {
  pde::ReduceJob job;
  Tensor ws;
};
std::vector<DeferredReduce> g_deferred;
// an optimiser segment waiting for the next paired GEMM launch (optim_attach)
bool g_seg_pending = false;
pde::OptimSeg g_seg{};
size_t g_deferred_bytes = 0;
int gemm_flush_deferred();

// Peak-memory bound for the deferred slabs: once the pending workspaces pass this many bytes (default
// 1 GiB, PDE_DEFER_CAP_MB) the list is flushed early, so a deep network's backward keeps O(cap) of slabs
// alive rather than one workspace per layer.  A full launch's worth of jobs flushes too.
size_t deferred_cap_bytes() {
  static const size_t cap = [] {
    const char* e = std::getenv("PDE_DEFER_CAP_MB");
    long mb = e ? std::atol(e) : 1024;
    return static_cast<size_t>(mb > 0 ? mb : 1024) << 20;
  }();
  return cap;
}

// Launch what was collected (2 GEMMs: one paired launch; fewer: ordinary launches).  abort=true drops it.
// defer=true: the second GEMM's slab reduction is deferred to gemm_flush_deferred (returns true if it was).
bool gemm_pair_end(bool abort, bool defer) {
  g_collect = false;
  std::vector<PendingGemm> q;
  q.swap(g_pending);
  const bool has_seg = g_seg_pending;
  const pde::OptimSeg seg = g_seg;
  g_seg_pending = false;
  if (abort) return false;
  if (q.size() == 2) {
    int sp1 = 0, sp0 = 0;
    check(pde::gemm_bf16_pair(q[0].args, q[1].args, cur_stream(), defer ? &sp1 : nullptr, has_seg ? &seg : nullptr,
                              q[0].defer_out ? &sp0 : nullptr),
          "gemm_pair");
    if (sp0 > 1) {  // the dgrad output stays unreduced: the BatchNorm backward sums its slabs (bn_bwd)
      std::lock_guard<std::mutex> lk(g_pending_mu);
      g_pending_conv[q[0].args.out] = PendingConv{q[0].ws, sp0, q[0].args.M, q[0].args.N};
    }
    if (sp1 > 1) {
      const pde::GemmArgs& a = q[1].args;
      pde::ReduceJob j{};
      j.workspace = a.workspace; j.out = a.out; j.bias_grad = a.bias_grad; j.ldo = a.ldo;
      j.M = a.M; j.N = a.N; j.splits = sp1; j.epi = a.epi;
      j.oihw_ci = a.oihw_ci; j.oihw_rs = a.oihw_rs; j.oihw_cp = a.oihw_cp; j.bias_col = a.bias_col;
      g_deferred.push_back({j, q[1].ws});
      g_deferred_bytes += q[1].ws.nbytes();
      if (g_deferred_bytes > deferred_cap_bytes() || static_cast<int>(g_deferred.size()) >= pde::kMaxReduceJobs)
        gemm_flush_deferred();
      return true;
    }
  } else {
    for (auto& p : q) check(pde::gemm_bf16(p.args, cur_stream()), "gemm");
    if (has_seg)
      check(pde::multi_tensor_optim_range(seg.mode, seg.tab, seg.chunks, seg.c0, seg.c1, seg.hp, seg.step,
                                          seg.publish, cur_stream()),
            "optim segment");
  }
  return false;
}

// One batched launch for every deferred reduction (no-op when none is pending).
int gemm_flush_deferred() {
  std::vector<DeferredReduce> d;
  d.swap(g_deferred);
  g_deferred_bytes = 0;
  if (d.empty()) return 0;
  std::vector<pde::ReduceJob> jobs;
  jobs.reserve(d.size());
  for (auto& x : d) jobs.push_back(x.job);
  check(pde::gemm_reduce_jobs(jobs.data(), static_cast<int>(jobs.size()), cur_stream()), "gemm_reduce_jobs");
  return static_cast<int>(d.size());  // the slabs are released after the launch (stream-ordered reuse)
}
int gemm_deferred_count() { return static_cast<int>(g_deferred.size()); }

// ------------------------------------------------------------------------------------------------
// Dense GEMMs (nn.Linear)
// ------------------------------------------------------------------------------------------------
Tensor linear_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, bool relu, bool out_f32) {
  resolve_pending(x);
  CHECK_IN(x); CHECK_IN(w); CHECK_BF16(x); CHECK_BF16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "linear_fwd: shape mismatch");
  Tensor out = at::empty({M, N}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  pde::GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.a = dense(x, K, 1);
  a.b = dense(w, K, 1);
  a.out = out.data_ptr(); a.ldo = N;
  a.bias = cf32(bias);
  a.nbias = a.bias ? static_cast<int>(bias->numel()) : 0;
  a.epi = (a.bias ? pde::EPI_BIAS : 0) | (relu ? pde::EPI_RELU : 0) | (out_f32 ? pde::EPI_OUT_F32 : 0);
  run_gemm(a, x, -1);
  return out;
}

// dx[M,K] = dy[M,N] . w[N,K]  (optionally * (aux > 0): fused ReLU backward of the producer)
Tensor linear_dgrad(const Tensor& dy, const Tensor& w, const optional<Tensor>& aux) {
  CHECK_IN(dy); CHECK_IN(w); CHECK_BF16(dy); CHECK_BF16(w);
  const int M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N, "linear_dgrad: shape mismatch");
  Tensor dx = at::empty({M, K}, dy.options());
  pde::GemmArgs a{};
  a.M = M; a.N = K; a.K = N;
  a.a = dense(dy, N, 1);
  a.b = dense(w, 1, K);
  a.out = dx.data_ptr(); a.ldo = K;
  a.aux = cu16(aux); a.ldaux = K;
  a.epi = a.aux ? pde::EPI_DRELU : 0;
  run_gemm(a, dy, -1);
  return dx;
}

// dW[N,K] = dy[M,N]^T . x[M,K]   (fp32, split-K over the batch when the tile grid is small); with ``out``
// the result is written (accumulate: added) into that tensor, e.g. the parameter's .grad.
Tensor linear_wgrad(const Tensor& dy, const Tensor& x, const optional<Tensor>& out, bool accumulate) {
  CHECK_IN(dy); CHECK_IN(x); CHECK_BF16(dy); CHECK_BF16(x);
  const int M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == M, "linear_wgrad: shape mismatch");
  Tensor dw = grad_sink(out, {N, K}, dy);
  pde::GemmArgs a{};
  a.M = N; a.N = K; a.K = M;
  a.a = dense(dy, 1, N);
  a.b = dense(x, 1, K);
  a.out = dw.data_ptr(); a.ldo = K;
  a.epi = pde::EPI_OUT_F32 | (accumulate ? pde::EPI_ACCUM : 0);
  run_gemm(a, dy, -1);
  return dw;
}

// ------------------------------------------------------------------------------------------------
// Linear ops on strided row views (the fused MLP step, models/mlp_fused.py): operands and outputs are 2-D
// views whose rows may be padded (stride(0) = ld >= cols, stride(1) = 1), e.g. activations that carry a
// trailing ones column for the bias gradient.
// ------------------------------------------------------------------------------------------------
#define CHECK_ROWS(x) \
  CHECK_DEV(x);       \
  TORCH_CHECK((x).dim() == 2 && (x).stride(1) == 1, #x " must be a 2-D row-major view")

// out = relu?(x W^T + b)
void linear_fwd_out(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, bool relu, Tensor& out) {
  CHECK_ROWS(x); CHECK_IN(w); CHECK_ROWS(out); CHECK_BF16(x); CHECK_BF16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "linear_fwd_out: shape mismatch");
  const bool f32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || out.scalar_type() == at::kBFloat16, "linear_fwd_out: out must be fp32 or bf16");
  pde::GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.a = dense(x, x.stride(0), 1);
  a.b = dense(w, K, 1);
  a.out = out.data_ptr(); a.ldo = out.stride(0);
  a.bias = cf32(bias);
  a.nbias = a.bias ? static_cast<int>(bias->numel()) : 0;
  a.epi = (a.bias ? pde::EPI_BIAS : 0) | (relu ? pde::EPI_RELU : 0) | (f32 ? pde::EPI_OUT_F32 : 0);
  run_gemm(a, x, -1);
}

// out = (dy . W) * (aux > 0 when aux is given)
void linear_dgrad_out(const Tensor& dy, const Tensor& w, const optional<Tensor>& aux, Tensor& out) {
  CHECK_ROWS(dy); CHECK_IN(w); CHECK_ROWS(out); CHECK_BF16(dy); CHECK_BF16(w); CHECK_BF16(out);
  const int M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N && out.size(0) == M && out.size(1) == K, "linear_dgrad_out: shape mismatch");
  pde::GemmArgs a{};
  a.M = M; a.N = K; a.K = N;
  a.a = dense(dy, dy.stride(0), 1);
  a.b = dense(w, 1, K);
  a.out = out.data_ptr(); a.ldo = out.stride(0);
  if (aux.has_value() && aux->defined()) {
    CHECK_ROWS(*aux); CHECK_BF16(*aux);
    TORCH_CHECK(aux->size(0) == M && aux->size(1) >= K, "linear_dgrad_out: aux shape");
    a.aux = cu16(aux); a.ldaux = aux->stride(0);
    a.epi = pde::EPI_DRELU;
  }
  run_gemm(a, dy, -1);
}

// out_w = dy^T . x_ext[:, :K],  out_b = dy^T . x_ext[:, K] (= column sums of dy: x_ext's last column is
// all ones) -- weight and bias gradients of a linear layer in ONE GEMM (fp32, written or accumulated).
void linear_wgrad_bias(const Tensor& dy, const Tensor& x_ext, Tensor& out_w, Tensor& out_b, bool accumulate) {
  CHECK_ROWS(dy); CHECK_ROWS(x_ext); CHECK_IN(out_w); CHECK_IN(out_b); CHECK_BF16(dy); CHECK_BF16(x_ext);
  CHECK_F32(out_w); CHECK_F32(out_b);
  const int M = dy.size(0), N = dy.size(1), K = x_ext.size(1) - 1;
  TORCH_CHECK(x_ext.size(0) == M && out_w.numel() == static_cast<long>(N) * K && out_b.numel() == N,
              "linear_wgrad_bias: shape mismatch");
  pde::GemmArgs a{};
  a.M = N; a.N = K + 1; a.K = M;
  a.a = dense(dy, 1, dy.stride(0));
  a.b = dense(x_ext, 1, x_ext.stride(0));
  a.out = out_w.data_ptr(); a.ldo = K;
  a.bias_grad = out_b.data_ptr<float>(); a.bias_col = K;
  a.epi = pde::EPI_OUT_F32 | (accumulate ? pde::EPI_ACCUM : 0);
  run_gemm(a, dy, -1);
}

// x [B, K] fp32 -> out[:, :K] bf16 and out[:, K] = 1 (out: a [B, >= K + 1] row view)
void cast_rows_ones(const Tensor& x, Tensor& out) {
  CHECK_IN(x); CHECK_F32(x); CHECK_ROWS(out); CHECK_BF16(out);
  const int B = x.size(0), K = x.numel() / std::max<int64_t>(1, x.size(0));
  TORCH_CHECK(out.size(0) == B && out.size(1) >= K + 1, "cast_rows_ones: out must be [B, >= K + 1]");
  check(pde::cast_rows_bf16(x.data_ptr<float>(), B, K, u16(out), out.stride(0), 1, cur_stream()), "cast_rows_ones");
}

// Device-counter batch gather (pde::gather_rows_counter): x_out [rows, ...] fp32 / y_out [rows] int64 <- rows
// counter[0] x rows ... of idx from src / labels; counter (int32 [2], device) advances by one per launch.
void gather_rows_counter(const Tensor& src, const Tensor& labels, const Tensor& idx, Tensor& counter, Tensor& x_out,
                         Tensor& y_out) {
  CHECK_IN(src); CHECK_F32(src); CHECK_IN(labels); CHECK_IN(idx); CHECK_IN(x_out); CHECK_F32(x_out); CHECK_IN(y_out);
  TORCH_CHECK(labels.scalar_type() == at::kLong && idx.scalar_type() == at::kLong && y_out.scalar_type() == at::kLong,
              "gather_rows_counter: int64 labels / indices");
  TORCH_CHECK(counter.is_cuda() && counter.scalar_type() == at::kInt && counter.numel() >= 2,
              "gather_rows_counter: counter must be a device int32[2]");
  const int64_t row_elems = src.numel() / std::max<int64_t>(1, src.size(0));
  const int rows = static_cast<int>(x_out.size(0));
  TORCH_CHECK(x_out.numel() == rows * row_elems && y_out.numel() == rows, "gather_rows_counter: x_out [rows, row]");
  TORCH_CHECK(row_elems % 4 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(x_out.data_ptr()) % 16 == 0, "gather_rows_counter: 16-byte rows");
  TORCH_CHECK(idx.numel() > 0 && labels.numel() == src.size(0), "gather_rows_counter: idx / labels");
  check(pde::gather_rows_counter(src.data_ptr<float>(), labels.data_ptr<int64_t>(), idx.data_ptr<int64_t>(),
                                 idx.numel(), reinterpret_cast<uint32_t*>(counter.data_ptr<int>()), rows,
                                 static_cast<int>(row_elems), x_out.data_ptr<float>(), y_out.data_ptr<int64_t>(),
                                 cur_stream()),
        "gather_rows_counter");
}

// (mean cross-entropy loss, d loss / d logits as bf16) in one launch.  dx_out: a [B, >= V] bf16 row view to
// write d logits into (its columns past V are left as they are, e.g. the zero padding of a K = 16 operand).
std::vector<Tensor> ce_fused(const Tensor& x, const Tensor& tgt, const optional<Tensor>& dx_out) {
  CHECK_IN(x); CHECK_IN(tgt);
  TORCH_CHECK(tgt.scalar_type() == at::kLong, "targets must be int64");
  const int B = x.size(0), V = x.size(1);
  Tensor loss = at::empty({}, x.options().dtype(at::kFloat));
  Tensor dx;
  if (dx_out.has_value() && dx_out->defined()) {
    dx = *dx_out;
    CHECK_ROWS(dx); CHECK_BF16(dx);
    TORCH_CHECK(dx.size(0) == B && dx.stride(0) >= V, "ce_fused: dx_out must be [B, >= V] rows");
  } else {
    dx = at::empty({B, V}, x.options().dtype(at::kBFloat16));
  }
  check(pde::ce_fused(x.data_ptr(), x.scalar_type() == at::kFloat, tgt.data_ptr<int64_t>(), B, V,
                      loss.data_ptr<float>(), u16(dx), static_cast<int>(dx.stride(0)), cur_stream()),
        "ce_fused");
  return {loss, dx};
}

// ------------------------------------------------------------------------------------------------
// NHWC implicit-GEMM convolution
// ------------------------------------------------------------------------------------------------
Tensor conv_fwd(const Tensor& x, const Tensor& wf, const optional<Tensor>& bias, int R, int S, int stride, int pad,
                bool relu, bool out_f32, bool defer) {
  CHECK_IN(x); CHECK_IN(wf); CHECK_BF16(x); CHECK_BF16(wf);
  resolve_pending(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0, "conv_fwd: input channels must be padded to a multiple of 8");
  const int Co = wf.size(0);
  TORCH_CHECK(wf.size(1) == R * S * C, "conv_fwd: weight must be [Co, R*S*C]");
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  Tensor y = at::empty({N, Ho, Wo, Co}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  pde::GemmArgs a{};
  a.M = N * Ho * Wo; a.N = Co; a.K = R * S * C;
  a.a = is_pointwise(R, S, stride, pad) ? dense(x, C, 1) : gather(x, 1, N, H, W, C, R, S, stride, pad, Ho, Wo);
  a.b = dense(wf, a.K, 1);
  a.out = y.data_ptr(); a.ldo = Co;
  a.bias = cf32(bias);
  a.nbias = a.bias ? static_cast<int>(bias->numel()) : 0;
  a.epi = (a.bias ? pde::EPI_BIAS : 0) | (relu ? pde::EPI_RELU : 0) | (out_f32 ? pde::EPI_OUT_F32 : 0);
  if (defer && a.epi == 0 && !g_collect) {
    // the BatchNorm that follows reduces the split-K slabs itself (bn_fwd): no reduce launch here
    const int max_split = split_cap(a);
    Tensor ws;
    if (max_split > 1) {
      ws = at::empty({static_cast<long>(max_split) * a.M * a.N}, x.options().dtype(at::kFloat));
      a.workspace = ws.data_ptr<float>();
      a.splitk = max_split;
    } else {
      a.workspace = nullptr;
      a.splitk = 1;
    }
    int used = 1;
    a.splits_out = &used;
    check(pde::gemm_bf16(a, cur_stream()), "conv_fwd");
    if (used > 1) {
      std::lock_guard<std::mutex> lk(g_pending_mu);
      g_pending_conv[y.data_ptr()] = PendingConv{ws, used, a.M, a.N};
    }
    return y;
  }
  run_gemm(a, x, -1);
  return y;
}

// ---- BatchNorm folded into the convolutions around it (pde_kernels.h BnStatsOut / BnFoldIn) ----
// conv_fwd_bn(x, wf, ...): the forward convolution of a Bottleneck with
//   stats_out (int64 [G, 2, Co] zero-initialised sums): its epilogue emits the statistics of the BatchNorm that
//     normalises its output (the producer side);
//   fold_sums / fold_ticket / gamma / beta / running stats: its A operand x is the RAW output of the previous
//     conv and the BatchNorm (+ ReLU) between the two is applied in the A loader (the consumer side).  Returns
//     {y, act, save_mean, save_invstd, scale_shift} -- act = relu(bn(x)) materialised for the backward.
// bn_fold_plan(...) answers, from the shapes alone, whether both sides can run folded (plan before the first
// launch, outside graph capture: it may allocate the split-K arrival tickets).
pde::GemmArgs conv_shape_args(int N, int H, int W, int C, int Co, int R, int S, int stride, int pad, const void* xp,
                              const void* wp, void* yp) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  pde::GemmArgs a{};
  a.M = N * Ho * Wo; a.N = Co; a.K = R * S * C;
  a.a.ptr = xp;
  if (is_pointwise(R, S, stride, pad)) {
    a.a.kind = 0; a.a.ld_r = C; a.a.ld_k = 1;
  } else {
    a.a.kind = 1; a.a.g = pde::ConvGeom{N, H, W, C, R, S, stride, pad, Ho, Wo};
  }
  a.b.ptr = wp; a.b.kind = 0; a.b.ld_r = a.K; a.b.ld_k = 1;
  a.out = yp; a.ldo = Co;
  a.epi = 0;
  return a;
}

bool bn_fold_plan(int N, int H, int W, int C, int Co1, int R1, int S1, int stride1, int pad1, int Co2, int R2, int S2,
                  int stride2, int pad2, int groups) {
  void* fake = reinterpret_cast<void*>(static_cast<uintptr_t>(1) << 20);  // any 16-B aligned address
  // producer: conv(x [N,H,W,C]) -> a [N,H1,W1,Co1] with statistics
  pde::GemmArgs p = conv_shape_args(N, H, W, C, Co1, R1, S1, stride1, pad1, fake, fake, fake);
  p.splitk = split_cap(p);
  p.workspace = p.splitk > 1 ? static_cast<float*>(fake) : nullptr;
  if (groups < 1 || p.M % groups != 0) return false;
  p.bn_out.sums = static_cast<long long*>(fake);
  p.bn_out.C = Co1; p.bn_out.G = groups; p.bn_out.rows_per_group = p.M / groups;
  if (!pde::gemm_bn_stats_ok(p, cur_stream())) return false;
  // consumer: conv(relu(bn(a))) with the BatchNorm in its A loader
  const int H1 = (H + 2 * pad1 - R1) / stride1 + 1, W1 = (W + 2 * pad1 - S1) / stride1 + 1;
  pde::GemmArgs c = conv_shape_args(N, H1, W1, Co1, Co2, R2, S2, stride2, pad2, fake, fake, fake);
  c.splitk = split_cap(c);
  c.workspace = c.splitk > 1 ? static_cast<float*>(fake) : nullptr;
  c.bn_in.ss = static_cast<const float*>(fake);
  c.bn_in.C = Co1; c.bn_in.G = groups; c.bn_in.rows_per_group = (N * H1 * W1) / groups;
  c.bn_in.center = is_pointwise(R2, S2, stride2, pad2) ? 0 : 1;
  return (N * H1 * W1) % groups == 0 && pde::gemm_bn_fold_ok(c);
}

// Returns {y, save_mean, save_invstd, scale_shift, act}: the last three-plus-one are defined when the conv
// produces statistics (stats_sums: the NEXT BatchNorm's finalize) / consumes a folded BatchNorm (fold_ss).
std::vector<Tensor> conv_fwd_bn(const Tensor& x, const Tensor& wf, int R, int S, int stride, int pad, int64_t groups,
                                const optional<Tensor>& stats_sums, const optional<Tensor>& stats_ticket,
                                const optional<Tensor>& gamma, const optional<Tensor>& beta,
                                const optional<Tensor>& running_mean, const optional<Tensor>& running_var, double eps,
                                double momentum, const optional<Tensor>& fold_ss, bool relu, bool defer) {
  CHECK_IN(x); CHECK_IN(wf); CHECK_BF16(x); CHECK_BF16(wf);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0, "conv_fwd_bn: input channels must be padded to a multiple of 8");
  const int Co = wf.size(0);
  TORCH_CHECK(wf.size(1) == R * S * C, "conv_fwd_bn: weight must be [Co, R*S*C]");
  const int G = static_cast<int>(groups);
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  Tensor y = at::empty({N, Ho, Wo, Co}, x.options());
  pde::GemmArgs a = conv_shape_args(N, H, W, C, Co, R, S, stride, pad, x.data_ptr(), wf.data_ptr(), y.data_ptr());
  auto fo = x.options().dtype(at::kFloat);
  std::vector<Tensor> out{y, Tensor(), Tensor(), Tensor(), Tensor()};
  const bool fold = fold_ss.has_value() && fold_ss->defined();
  const bool stats = stats_sums.has_value() && stats_sums->defined();
  static const int dbg = std::getenv("PDE_BN_FOLD_DEBUG") ? std::atoi(std::getenv("PDE_BN_FOLD_DEBUG")) : 0;
  a.bn_in.debug = dbg;
  a.bn_out.debug = dbg;
  if (!fold) resolve_pending(x);
  if (fold) {
    TORCH_CHECK(fold_ss->scalar_type() == at::kFloat && fold_ss->numel() == static_cast<long>(G) * 2 * C,
                "conv_fwd_bn: folded scale / shift must be fp32 [G, 2, C]");
    TORCH_CHECK((N * H * W) % G == 0, "conv_fwd_bn: rows not divisible by groups");
    Tensor act = at::empty_like(x);
    pde::BnFoldIn& f = a.bn_in;
    f.ss = fold_ss->data_ptr<float>();
    f.act = u16(act);
    f.C = C; f.G = G; f.rows_per_group = (N * H * W) / G;
    f.relu = relu ? 1 : 0;
    f.center = is_pointwise(R, S, stride, pad) ? 0 : 1;
    out[4] = act;
  }
  if (stats) {
    TORCH_CHECK(stats_ticket.has_value() && stats_ticket->defined(), "conv_fwd_bn: statistics need their ticket");
    TORCH_CHECK(stats_sums->scalar_type() == at::kLong &&
                    stats_sums->numel() == static_cast<long>(pde::kBnShards) * G * 2 * Co,
                "conv_fwd_bn: statistics sums must be int64 [bn_fold_shards, G, 2, Co]");
    TORCH_CHECK(a.M % G == 0, "conv_fwd_bn: output rows not divisible by groups");
    Tensor mean = at::empty({G * Co}, fo), invstd = at::empty({G * Co}, fo), ss = at::empty({G * 2 * Co}, fo);
    pde::BnStatsOut& f = a.bn_out;
    f.sums = static_cast<long long*>(stats_sums->data_ptr());
    f.ticket = stats_ticket->data_ptr<int>();
    f.C = Co; f.G = G; f.rows_per_group = a.M / G;
    f.gamma = cf32(gamma); f.beta = cf32(beta);
    f.running_mean = f32(running_mean); f.running_var = f32(running_var);
    f.save_mean = mean.data_ptr<float>(); f.save_invstd = invstd.data_ptr<float>(); f.ss = ss.data_ptr<float>();
    f.eps = static_cast<float>(eps); f.momentum = static_cast<float>(momentum);
    out[1] = mean; out[2] = invstd; out[3] = ss;
  }
  const int max_split = split_cap(a);
  Tensor ws;
  if (max_split > 1) {
    ws = at::empty({static_cast<long>(max_split) * a.M * a.N}, fo);
    a.workspace = ws.data_ptr<float>();
    a.splitk = max_split;
  } else {
    a.workspace = nullptr;
    a.splitk = 1;
  }
  if (stats) TORCH_CHECK(pde::gemm_bn_stats_ok(a, cur_stream()), "conv_fwd_bn: statistics epilogue not possible");
  if (fold) TORCH_CHECK(pde::gemm_bn_fold_ok(a), "conv_fwd_bn: folded BatchNorm not possible for this shape");
  int used = 1;
  if (defer && !stats) a.splits_out = &used;  // the one-launch BatchNorm after this conv reduces the slabs
  check(pde::gemm_bf16(a, cur_stream()), "conv_fwd_bn");
  if (used > 1) {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    g_pending_conv[y.data_ptr()] = PendingConv{ws, used, a.M, a.N};
  }
  return out;
}

// dx[N,H,W,Ci] from dy[N,Ho,Wo,Co] and wd = [Ci, R*S*Co]; or, for a 1x1 / stride-1 conv with
// w_fwd_layout, from the forward copy wd = [Co, Ci] read transposed (no separate dgrad layout).
// aux: with add_aux, a bf16 [N*H*W, Ci] gradient added in the epilogue (the other branch of a residual
// fork); otherwise the saved post-ReLU activation whose mask multiplies the result.
Tensor conv_dgrad(const Tensor& dy, const Tensor& wd, int H, int W, int R, int S, int stride, int pad,
                  const optional<Tensor>& aux, bool w_fwd_layout, bool add_aux, bool defer) {
  CHECK_IN(dy); CHECK_IN(wd); CHECK_BF16(dy); CHECK_BF16(wd);
  resolve_pending(aux);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  TORCH_CHECK(Co % 8 == 0, "conv_dgrad: Cout must be a multiple of 8");
  int Ci;
  if (w_fwd_layout) {
    // 1x1 (any stride): B[ci][co] = w[co][ci] is the forward copy read transposed; a strided conv gathers dy
    TORCH_CHECK(R == 1 && S == 1 && pad == 0, "conv_dgrad: the forward-layout weight needs an unpadded 1x1 conv");
    TORCH_CHECK(wd.dim() == 2 && wd.size(0) == Co && wd.size(1) % 8 == 0, "conv_dgrad: weight must be [Co, Ci]");
    Ci = wd.size(1);
  } else {
    Ci = wd.size(0);
    TORCH_CHECK(wd.size(1) == R * S * Co, "conv_dgrad: weight must be [Ci, R*S*Co]");
  }
  Tensor dx = at::empty({N, H, W, Ci}, dy.options());
  pde::GemmArgs a{};
  a.M = N * H * W; a.N = Ci; a.K = R * S * Co;
  a.a = is_pointwise(R, S, stride, pad) ? dense(dy, Co, 1) : gather(dy, 3, N, Ho, Wo, Co, R, S, stride, pad, H, W);
  a.b = w_fwd_layout ? dense(wd, 1, Ci) : dense(wd, a.K, 1);
  a.out = dx.data_ptr(); a.ldo = Ci;
  a.aux = cu16(aux); a.ldaux = Ci;
  if (a.aux) {
    CHECK_IN(*aux); CHECK_BF16(*aux);
    TORCH_CHECK(aux->numel() == dx.numel(), "conv_dgrad: aux must match dx");
  }
  a.epi = a.aux ? (add_aux ? pde::EPI_ADD_AUX : pde::EPI_DRELU) : 0;
  run_gemm(a, dy, -1);
  // defer (a dgrad collected as problem 0 of a pair, plain epilogue): its split-K slabs are left for the
  // BatchNorm backward that consumes dx (registered as pending by gemm_pair_end if it did split)
  if (defer && g_collect && a.epi == 0 && g_pending.size() == 1) g_pending.back().defer_out = true;
  return dx;
}

// dW[Co, Ci, R, S] fp32 (the parameter's layout) from dy[N,Ho,Wo,Cop] and x[N,H,W,Cp]: the GEMM
// dW[co][(r,s,c)] = sum_pixels dy[pixel][co] * x-gather[pixel][(r,s,c)] stores through the OIHW epilogue
// remap, so no layout kernel runs; with ``out`` (accumulate: +=) it lands directly in the .grad tensor.
Tensor conv_wgrad(const Tensor& dy, const Tensor& x, int R, int S, int stride, int pad, int Co, int Ci,
                  const optional<Tensor>& out, bool accumulate) {
  resolve_pending(x);
  CHECK_IN(dy); CHECK_IN(x); CHECK_BF16(dy); CHECK_BF16(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2), Cop = dy.size(3);
  TORCH_CHECK(C % 8 == 0, "conv_wgrad: input channels must be a multiple of 8");
  TORCH_CHECK(Co <= Cop && Ci <= C, "conv_wgrad: real channels exceed the padded activations");
  Tensor dw = grad_sink(out, {Co, Ci, R, S}, dy);
  pde::GemmArgs a{};
  a.M = Co; a.N = R * S * C; a.K = N * Ho * Wo;
  a.a = dense(dy, 1, Cop);
  a.b = is_pointwise(R, S, stride, pad) ? dense(x, 1, C) : gather(x, 2, N, H, W, C, R, S, stride, pad, Ho, Wo);
  a.out = dw.data_ptr(); a.ldo = a.N;
  a.epi = pde::EPI_OUT_F32 | pde::EPI_OIHW | (accumulate ? pde::EPI_ACCUM : 0);
  a.oihw_ci = Ci; a.oihw_rs = R * S; a.oihw_cp = C;
  run_gemm(a, dy, -1);
  return dw;
}

// ------------------------------------------------------------------------------------------------
// Elementwise / layout
// ------------------------------------------------------------------------------------------------
Tensor cast_bf16(const Tensor& x) {
  CHECK_IN(x); CHECK_F32(x);
  Tensor y = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  check(pde::cast_f32_bf16(x.data_ptr<float>(), u16(y), x.numel(), cur_stream()), "cast_bf16");
  return y;
}
void cast_bf16_into(const Tensor& x, Tensor& y) {
  CHECK_IN(x); CHECK_F32(x); CHECK_IN(y); CHECK_BF16(y);
  TORCH_CHECK(x.numel() == y.numel(), "cast_bf16_into: size mismatch");
  check(pde::cast_f32_bf16(x.data_ptr<float>(), u16(y), x.numel(), cur_stream()), "cast_bf16_into");
}
Tensor cast_f32(const Tensor& x) {
  CHECK_IN(x); CHECK_BF16(x);
  Tensor y = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  check(pde::cast_bf16_f32(u16(x), y.data_ptr<float>(), x.numel(), cur_stream()), "cast_f32");
  return y;
}
void cast_f32_into(const Tensor& x, Tensor& y) {
  CHECK_IN(x); CHECK_BF16(x); CHECK_IN(y); CHECK_F32(y);
  TORCH_CHECK(x.numel() == y.numel(), "cast_f32_into: size mismatch");
  check(pde::cast_bf16_f32(u16(x), y.data_ptr<float>(), x.numel(), cur_stream()), "cast_f32_into");
}
Tensor nchw_to_nhwc(const Tensor& x, int Cp) {
  CHECK_IN(x); CHECK_F32(x);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(Cp % 8 == 0 && Cp >= C, "nchw_to_nhwc: bad channel padding");
  Tensor y = at::empty({N, H, W, Cp}, x.options().dtype(at::kBFloat16));
  check(pde::nchw_f32_to_nhwc_bf16(x.data_ptr<float>(), u16(y), N, C, H, W, Cp, cur_stream()), "nchw_to_nhwc");
  return y;
}
// [Co, Ci, R, S] fp32 -> [Cop, R*S*Cp] bf16 (zero padded channels)
Tensor conv_w_fwd(const Tensor& w, int Cp, int Cop, const optional<Tensor>& out) {
  CHECK_IN(w); CHECK_F32(w);
  const int Co = w.size(0), Ci = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(Cp >= Ci && Cop >= Co, "conv_w_fwd: padding smaller than channels");
  Tensor y = out.has_value() && out->defined() ? *out : at::empty({Cop, R * S * Cp}, w.options().dtype(at::kBFloat16));
  CHECK_IN(y); CHECK_BF16(y);
  TORCH_CHECK(y.numel() == static_cast<long>(Cop) * R * S * Cp, "conv_w_fwd: out size");
  check(pde::conv_weight_fwd_layout(w.data_ptr<float>(), u16(y), Co, Ci, R, S, Cp, Cop, cur_stream()), "conv_w_fwd");
  return y;
}
// [Co, Ci, R, S] fp32 -> [Cip, R*S*Cop] bf16
Tensor conv_w_dgrad(const Tensor& w, int Cip, int Cop, const optional<Tensor>& out) {
  CHECK_IN(w); CHECK_F32(w);
  const int Co = w.size(0), Ci = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(Cip >= Ci && Cop >= Co, "conv_w_dgrad: padding smaller than channels");
  Tensor y = out.has_value() && out->defined() ? *out : at::empty({Cip, R * S * Cop}, w.options().dtype(at::kBFloat16));
  CHECK_IN(y); CHECK_BF16(y);
  TORCH_CHECK(y.numel() == static_cast<long>(Cip) * R * S * Cop, "conv_w_dgrad: out size");
  check(pde::conv_weight_dgrad_layout(w.data_ptr<float>(), u16(y), Co, Ci, R, S, Cip, Cop, cur_stream()),
        "conv_w_dgrad");
  return y;
}
// [Cop, R*S*Cp] fp32 (wgrad GEMM output) -> [Co, Ci, R, S] fp32
Tensor conv_wgrad_oihw(const Tensor& g, int Co, int Ci, int R, int S) {
  CHECK_IN(g); CHECK_F32(g);
  TORCH_CHECK(g.size(0) >= Co, "conv_wgrad_oihw: rows");
  const int Cp = g.size(1) / (R * S);
  Tensor y = at::empty({Co, Ci, R, S}, g.options());
  check(pde::conv_wgrad_to_oihw(g.data_ptr<float>(), y.data_ptr<float>(), Co, Ci, R, S, Cp, 0, cur_stream()),
        "conv_wgrad_oihw");
  return y;
}
// Column sums (bias gradient) of the first ``ncols`` columns (-1: all); ``out``/accumulate as linear_wgrad.
Tensor colsum(const Tensor& x, int64_t ncols, const optional<Tensor>& out, bool accumulate) {
  CHECK_IN(x); CHECK_BF16(x);
  const int N = x.size(-1);
  const int M = x.numel() / N;
  const int nc = ncols < 0 ? N : static_cast<int>(ncols);
  TORCH_CHECK(nc <= N, "colsum: ncols");
  const int ws_blocks = 512;
  Tensor ws = at::empty({static_cast<long>(ws_blocks) * N}, x.options().dtype(at::kFloat));
  if (nc == N && out.has_value() && out->defined()) {  // straight into the sink (bias .grad)
    Tensor o = *out;
    CHECK_IN(o); CHECK_F32(o);
    TORCH_CHECK(o.numel() == N, "colsum: out");
    check(pde::colsum_bf16_ws(u16(x), o.data_ptr<float>(), M, N, accumulate ? 1 : 0, ws.data_ptr<float>(),
                              ws_blocks, cur_stream()),
          "colsum");
    return o;
  }
  if (nc != N) {
    // padded channels: full sums into a scratch row, then copy / add the real columns
    Tensor full = colsum(x, -1, c10::nullopt, false);
    Tensor res = full.narrow(0, 0, nc);
    if (out.has_value() && out->defined()) {
      Tensor o = *out;
      TORCH_CHECK(o.numel() == nc && o.scalar_type() == at::kFloat, "colsum: out");
      if (accumulate) o.add_(res.view(o.sizes())); else o.copy_(res.view(o.sizes()));
      return o;
    }
    return res.contiguous();
  }
  Tensor y = at::empty({N}, x.options().dtype(at::kFloat));
  check(pde::colsum_bf16_ws(u16(x), y.data_ptr<float>(), M, N, 0, ws.data_ptr<float>(), ws_blocks, cur_stream()),
        "colsum");
  return y;
}
Tensor relu_bwd(const Tensor& dy, const Tensor& y) {
  resolve_pending(y);
  CHECK_IN(dy); CHECK_IN(y); CHECK_BF16(dy); CHECK_BF16(y);
  Tensor dx = at::empty_like(dy);
  check(pde::relu_bwd_bf16(u16(dy), u16(y), u16(dx), dy.numel(), cur_stream()), "relu_bwd");
  return dx;
}

// ------------------------------------------------------------------------------------------------
// Losses
// ------------------------------------------------------------------------------------------------
std::vector<Tensor> ce_fwd(const Tensor& x, const Tensor& tgt, int mode) {
  CHECK_IN(x); CHECK_IN(tgt);
  TORCH_CHECK(tgt.scalar_type() == at::kLong, "targets must be int64");
  const int B = x.size(0), V = x.size(1);
  TORCH_CHECK(B <= 1 << 20, "batch too large for the single-block reduction");
  const bool f = x.scalar_type() == at::kFloat;
  Tensor loss = at::empty({}, x.options().dtype(at::kFloat));
  Tensor lse = at::empty({B}, x.options().dtype(at::kFloat));
  check(pde::ce_fwd(x.data_ptr(), f, tgt.data_ptr<int64_t>(), B, V, mode, loss.data_ptr<float>(),
                    mode == 0 ? lse.data_ptr<float>() : nullptr, cur_stream()),
        "ce_fwd");
  return {loss, lse};
}
Tensor ce_bwd(const Tensor& x, const Tensor& tgt, const Tensor& lse, const Tensor& gout, int mode, bool dx_f32) {
  CHECK_IN(x); CHECK_IN(tgt); CHECK_IN(gout);
  const int B = x.size(0), V = x.size(1);
  const bool f = x.scalar_type() == at::kFloat;
  Tensor dx = at::empty({B, V}, x.options().dtype(dx_f32 ? at::kFloat : at::kBFloat16));
  check(pde::ce_bwd(x.data_ptr(), f, tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), gout.data_ptr<float>(), B, V,
                    mode, dx.data_ptr(), dx_f32, cur_stream()),
        "ce_bwd");
  return dx;
}
Tensor log_softmax_fwd(const Tensor& x) {
  CHECK_IN(x);
  const int B = x.size(0), V = x.size(1);
  Tensor y = at::empty({B, V}, x.options().dtype(at::kFloat));
  check(pde::log_softmax_fwd(x.data_ptr(), x.scalar_type() == at::kFloat, B, V, y.data_ptr<float>(), cur_stream()),
        "log_softmax_fwd");
  return y;
}
Tensor log_softmax_bwd(const Tensor& dy, const Tensor& y, bool dx_f32) {
  CHECK_IN(dy); CHECK_IN(y); CHECK_F32(dy); CHECK_F32(y);
  const int B = y.size(0), V = y.size(1);
  Tensor dx = at::empty({B, V}, y.options().dtype(dx_f32 ? at::kFloat : at::kBFloat16));
  check(pde::log_softmax_bwd(dy.data_ptr<float>(), y.data_ptr<float>(), B, V, dx.data_ptr(), dx_f32, cur_stream()),
        "log_softmax_bwd");
  return dx;
}
Tensor mse_fwd(const Tensor& p, const Tensor& t) {
  CHECK_IN(p); CHECK_IN(t); CHECK_F32(t);
  Tensor loss = at::empty({}, p.options().dtype(at::kFloat));
  check(pde::mse_fwd(p.data_ptr(), p.scalar_type() == at::kFloat, t.data_ptr<float>(), p.numel(),
                     loss.data_ptr<float>(), cur_stream()),
        "mse_fwd");
  return loss;
}
Tensor mse_bwd(const Tensor& p, const Tensor& t, const Tensor& gout, bool dx_f32) {
  CHECK_IN(p); CHECK_IN(t); CHECK_IN(gout);
  Tensor dx = at::empty(p.sizes(), p.options().dtype(dx_f32 ? at::kFloat : at::kBFloat16));
  check(pde::mse_bwd(p.data_ptr(), p.scalar_type() == at::kFloat, t.data_ptr<float>(), gout.data_ptr<float>(),
                     p.numel(), dx.data_ptr(), dx_f32, cur_stream()),
        "mse_bwd");
  return dx;
}

// ------------------------------------------------------------------------------------------------
// Fused multi-tensor optimiser
// ------------------------------------------------------------------------------------------------
// Build the device tables for a parameter set: per-tensor entries and the chunk list (tensors cut into
// chunks of optim_chunk_elems(), a chunk never straddles two tensors).  Returns (table, chunks, nchunks).
// bf16_copies: compute copies refreshed by the update (an empty tensor in any optional list = none).
Tensor to_device_bytes(const void* src, long bytes, const at::TensorOptions& dev_opts) {
  Tensor host = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  std::memcpy(host.data_ptr(), src, bytes);
  Tensor dev = at::empty({bytes}, dev_opts.dtype(at::kByte));
  dev.copy_(host, /*non_blocking=*/true);
  return dev;
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

std::tuple<Tensor, Tensor, int64_t> optim_table(const std::vector<Tensor>& params, const std::vector<Tensor>& grads,
                                                const std::vector<Tensor>& exp_avg,
                                                const std::vector<Tensor>& exp_avg_sq,
                                                const std::vector<Tensor>& bf16_copies) {
  const size_t n = params.size();
  TORCH_CHECK(n > 0, "optim_table: no parameters");
  TORCH_CHECK(grads.size() == n, "optim_table: grads size");
  std::vector<pde::OptimEntry> tab(n);
  std::vector<pde::OptimChunk> chunks;
  const int chunk = pde::optim_chunk_elems();
  auto get = [&](const std::vector<Tensor>& v, size_t i) -> const Tensor* {
    return i < v.size() && v[i].defined() && v[i].numel() > 0 ? &v[i] : nullptr;  // empty tensor = none
  };
  for (size_t i = 0; i < n; ++i) {
    const Tensor& p = params[i];
    CHECK_IN(p); CHECK_F32(p);
    TORCH_CHECK(p.numel() < (1L << 31), "optim_table: tensor too large");
    pde::OptimEntry e{};
    e.param = p.data_ptr<float>();
    if (grads[i].defined()) {
      CHECK_CONTIG(grads[i]); TORCH_CHECK(grads[i].numel() == p.numel(), "grad size");
      e.grad = grads[i].data_ptr<float>();
    }
    if (auto t = get(exp_avg, i)) e.exp_avg = t->data_ptr<float>();
    if (auto t = get(exp_avg_sq, i)) e.exp_avg_sq = t->data_ptr<float>();
    if (auto t = get(bf16_copies, i)) {
      CHECK_IN(*t);
      TORCH_CHECK(t->numel() == p.numel() && t->scalar_type() == at::kBFloat16, "bf16 copy");
      e.bf16_copy = u16(*t);
    }
    e.size = p.numel();
    e.vec = al16(e.param) && (!e.grad || al16(e.grad)) && (!e.exp_avg || al16(e.exp_avg)) &&
            (!e.exp_avg_sq || al16(e.exp_avg_sq)) && (!e.bf16_copy || (reinterpret_cast<uintptr_t>(e.bf16_copy) & 7) == 0);
    tab[i] = e;
    for (long s0 = 0; s0 < e.size; s0 += chunk)
      chunks.push_back(pde::OptimChunk{static_cast<int>(i), static_cast<int>(s0),
                                       static_cast<int>(std::min<long>(chunk, e.size - s0)), 0});
  }
  auto opts = params[0].options();
  Tensor dtab = to_device_bytes(tab.data(), static_cast<long>(n * sizeof(pde::OptimEntry)), opts);
  Tensor dchunks = to_device_bytes(chunks.data(), static_cast<long>(chunks.size() * sizeof(pde::OptimChunk)), opts);
  return {dtab, dchunks, static_cast<int64_t>(chunks.size())};
}

// Device table for conv_layouts_step: weights w[i] [Co,Ci,R,S] fp32 with their bf16 forward ([Cop, R*S*Cp])
// and dgrad ([Cp, R*S*Cop]) layout tensors.
Tensor conv_layout_table(const std::vector<Tensor>& ws, const std::vector<Tensor>& fwds,
                         const std::vector<Tensor>& dgrads, const std::vector<int64_t>& cps,
                         const std::vector<int64_t>& cops) {
  const size_t n = ws.size();
  TORCH_CHECK(n > 0 && fwds.size() == n && dgrads.size() == n && cps.size() == n && cops.size() == n,
              "conv_layout_table: list sizes");
  std::vector<pde::ConvLayoutEntry> tab(n);
  for (size_t i = 0; i < n; ++i) {
    const Tensor& w = ws[i];
    CHECK_IN(w); CHECK_F32(w); CHECK_IN(fwds[i]); CHECK_BF16(fwds[i]); CHECK_IN(dgrads[i]); CHECK_BF16(dgrads[i]);
    TORCH_CHECK(w.dim() == 4, "conv_layout_table: 4-D weight");
    pde::ConvLayoutEntry e{};
    e.w = w.data_ptr<float>();
    e.fwd = u16(fwds[i]);
    e.dgrad = u16(dgrads[i]);
    e.Co = w.size(0); e.Ci = w.size(1); e.R = w.size(2); e.S = w.size(3);
    e.Cp = static_cast<int>(cps[i]); e.Cop = static_cast<int>(cops[i]);
    TORCH_CHECK(e.Cp >= e.Ci && e.Cop >= e.Co, "conv_layout_table: padding smaller than channels");
    const long total = static_cast<long>(e.Cop) * e.R * e.S * e.Cp;
    TORCH_CHECK(fwds[i].numel() == total && dgrads[i].numel() == total, "conv_layout_table: layout sizes");
    tab[i] = e;
  }
  return to_device_bytes(tab.data(), static_cast<long>(n * sizeof(pde::ConvLayoutEntry)), ws[0].options());
}

// blocks_x: x blocks per entry (size it for the largest weight; smaller entries' extra blocks exit).
void conv_layouts_step(const Tensor& table, int64_t n, int64_t blocks_x) {
  CHECK_IN(table);
  TORCH_CHECK(table.numel() == static_cast<long>(n * sizeof(pde::ConvLayoutEntry)), "conv_layouts_step: table");
  check(pde::conv_weight_layouts_multi(reinterpret_cast<const pde::ConvLayoutEntry*>(table.data_ptr()),
                                       static_cast<int>(n), static_cast<int>(blocks_x), cur_stream()),
        "conv_layouts_step");
}

void optim_step(const Tensor& table, const Tensor& chunks, int64_t nchunks, int mode, const Tensor& hparams,
                Tensor& step) {
  CHECK_IN(table); CHECK_IN(chunks); CHECK_IN(hparams); CHECK_IN(step);
  TORCH_CHECK(hparams.numel() >= pde::HP_COUNT, "hparams size");
  TORCH_CHECK(step.scalar_type() == at::kInt && step.numel() >= 2, "step must be int32[2]");
  check(pde::multi_tensor_optim(mode, reinterpret_cast<const pde::OptimEntry*>(table.data_ptr()),
                                reinterpret_cast<const pde::OptimChunk*>(chunks.data_ptr()),
                                static_cast<int>(nchunks), hparams.data_ptr<float>(), step.data_ptr<int>(),
                                cur_stream()),
        "optim_step");
}

// Chunk range [c0, c1) of an optimiser table: its own launch (publish: the step's last segment advances the
// device step counter), or -- optim_attach -- appended as extra blocks to the NEXT paired GEMM launch
// (gemm_pair_end), so the HBM-bound update of one layer overlaps the latency-bound backward GEMMs of the next.
pde::OptimSeg make_seg(const Tensor& table, const Tensor& chunks, int64_t c0, int64_t c1, int mode,
                       const Tensor& hparams, Tensor& step, bool publish) {
  CHECK_IN(table); CHECK_IN(chunks); CHECK_IN(hparams); CHECK_IN(step);
  TORCH_CHECK(hparams.numel() >= pde::HP_COUNT, "hparams size");
  TORCH_CHECK(step.scalar_type() == at::kInt && step.numel() >= 2, "step must be int32[2]");
  TORCH_CHECK(0 <= c0 && c0 <= c1 && c1 * static_cast<long>(sizeof(pde::OptimChunk)) <= chunks.nbytes(),
              "optimiser chunk range out of bounds");
  pde::OptimSeg g{};
  g.tab = reinterpret_cast<const pde::OptimEntry*>(table.data_ptr());
  g.chunks = reinterpret_cast<const pde::OptimChunk*>(chunks.data_ptr());
  g.hp = hparams.data_ptr<float>();
  g.step = step.data_ptr<int>();
  g.c0 = static_cast<int>(c0);
  g.c1 = static_cast<int>(c1);
  g.mode = mode;
  g.publish = publish ? 1 : 0;
  g.blocks = std::min(static_cast<int>(c1 - c0), 1024);
  return g;
}
void optim_step_range(const Tensor& table, const Tensor& chunks, int64_t c0, int64_t c1, int mode,
                      const Tensor& hparams, Tensor& step, bool publish) {
  const pde::OptimSeg g = make_seg(table, chunks, c0, c1, mode, hparams, step, publish);
  if (!g_deferred.empty()) gemm_flush_deferred();  // the gradients it reads must be final
  check(pde::multi_tensor_optim_range(mode, g.tab, g.chunks, g.c0, g.c1, g.hp, g.step, g.publish, cur_stream()),
        "optim_step_range");
}
void optim_attach(const Tensor& table, const Tensor& chunks, int64_t c0, int64_t c1, int mode, const Tensor& hparams,
                  Tensor& step, bool publish) {
  TORCH_CHECK(!g_seg_pending, "optim_attach: a segment is already waiting for a GEMM pair");
  // its gradients must be final: deferred split-K reductions are flushed first
  if (!g_deferred.empty()) gemm_flush_deferred();
  g_seg = make_seg(table, chunks, c0, c1, mode, hparams, step, publish);
  g_seg_pending = true;
}

// ------------------------------------------------------------------------------------------------
// BatchNorm / pooling / dropout / EmbeddingBag
// ------------------------------------------------------------------------------------------------
// Returns y, save_mean, save_invstd, scale_shift ([2C] fp32: y = relu?(x*scale + shift + res)).
std::vector<Tensor> bn_fwd(const Tensor& x, const optional<Tensor>& gamma, const optional<Tensor>& beta,
                           const optional<Tensor>& running_mean, const optional<Tensor>& running_var, double eps,
                           double momentum, const optional<Tensor>& res, bool relu, int64_t groups) {
  CHECK_IN(x); CHECK_BF16(x);
  const int C = x.size(-1);
  const int P = x.numel() / C;
  const int G = static_cast<int>(groups);
  TORCH_CHECK(C % 8 == 0, "bn_fwd: C must be a multiple of 8");
  TORCH_CHECK(G >= 1 && x.size(0) % G == 0, "bn_fwd: batch ", x.size(0), " is not a multiple of groups ", G);
  auto fo = x.options().dtype(at::kFloat);
  Tensor y = at::empty_like(x);
  // grouped: per-group statistics [G][C], scale/shift [G][2C] (groups = micro-batches of one launch)
  Tensor mean = at::empty({G * C}, fo), invstd = at::empty({G * C}, fo), ss = at::empty({G * 2 * C}, fo);
  Tensor ws = at::empty({static_cast<long>(pde::bn_workspace_blocks(P, C, G)) * 2 * C}, fo);
  Tensor gs = G > 1 ? at::empty({G * 2 * C}, fo) : Tensor();
  resolve_pending(res);
  PendingConv pc{};
  {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    auto it = g_pending_conv.find(x.data_ptr());
    if (it != g_pending_conv.end()) {  // x = a deferred split-K conv output: the BatchNorm reduces its slabs
      pc = std::move(it->second);
      g_pending_conv.erase(it);
    }
  }
  TORCH_CHECK(!pc.ws.defined() || (pc.M == P && pc.N == C), "bn_fwd: deferred conv output shape mismatch");
  check(pde::bn_fwd_train(u16(x), P, C, cf32(gamma), cf32(beta), static_cast<float>(eps),
                          static_cast<float>(momentum), f32(running_mean), f32(running_var), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), ss.data_ptr<float>(), ws.data_ptr<float>(), cu16(res), relu,
                          u16(y), cur_stream(), pc.ws.defined() ? pc.ws.data_ptr<float>() : nullptr,
                          pc.ws.defined() ? pc.splits : 1, G, G > 1 ? gs.data_ptr<float>() : nullptr),
        "bn_fwd");
  return {y, mean, invstd, ss};
}
// Inference / eval mode: y = x*scale + shift with scale/shift from running stats (computed in torch).
Tensor bn_apply(const Tensor& x, const Tensor& scale, const Tensor& shift, const optional<Tensor>& res, bool relu) {
  CHECK_IN(x); CHECK_BF16(x);
  resolve_pending(x);
  resolve_pending(res);
  const int C = x.size(-1);
  const int P = x.numel() / C;
  Tensor y = at::empty_like(x);
  check(pde::bn_apply(u16(x), P, C, scale.data_ptr<float>(), shift.data_ptr<float>(), cu16(res), relu, u16(y),
                      cur_stream()),
        "bn_apply");
  return y;
}
// Returns dx, dgamma, dbeta, dres (dres undefined unless want_dres).  With dg_out / db_out (both, [C] fp32)
// the parameter gradients are ADDED into those tensors (direct accumulation into .grad).  scale_shift (the
// forward's, only for a BatchNorm without residual): the ReLU mask comes from x instead of y.
std::vector<Tensor> bn_bwd(const Tensor& dy, const Tensor& x, const Tensor& y, const Tensor& mean,
                           const Tensor& invstd, const optional<Tensor>& gamma, bool relu, bool want_dres,
                           const optional<Tensor>& dg_out, const optional<Tensor>& db_out,
                           const optional<Tensor>& scale_shift, int64_t groups, bool accum) {
  CHECK_IN(dy); CHECK_IN(x); CHECK_IN(y); CHECK_BF16(dy);
  resolve_pending(x);
  resolve_pending(y);
  const int C = x.size(-1);
  const int P = x.numel() / C;
  // dy left as split-K slabs by the conv dgrad that produced it (conv_dgrad(defer=true)): summed by the kernel
  Tensor dyws;
  int dysp = 1;
  {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    auto it = g_pending_conv.find(dy.data_ptr());
    if (it != g_pending_conv.end() && it->second.M == P && it->second.N == C && dy.numel() == x.numel()) {
      dyws = it->second.ws;
      dysp = it->second.splits;
      g_pending_conv.erase(it);
    }
  }
  if (!dyws.defined()) resolve_pending(dy);
  else ++g_bn_bwd_slab_uses;
  const int G = static_cast<int>(groups);
  TORCH_CHECK(G >= 1 && x.size(0) % G == 0 && mean.numel() == static_cast<long>(G) * C,
              "bn_bwd: groups / statistics shape mismatch");
  auto fo = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x);
  const bool direct = dg_out.has_value() && dg_out->defined() && db_out.has_value() && db_out->defined();
  Tensor dg = direct ? grad_sink(dg_out, {C}, x) : at::empty({C}, fo);
  Tensor db = direct ? grad_sink(db_out, {C}, x) : at::empty({C}, fo);
  Tensor coef = at::empty({G * 3 * C}, fo);
  Tensor ws = at::empty({static_cast<long>(pde::bn_workspace_blocks(P, C, G)) * 2 * C}, fo);
  Tensor gs = G > 1 ? at::empty({G * 2 * C}, fo) : Tensor();
  Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  check(pde::bn_bwd(u16(dy), u16(x), u16(y), mean.data_ptr<float>(), invstd.data_ptr<float>(), cf32(gamma), P, C,
                    relu, dg.data_ptr<float>(), db.data_ptr<float>(), direct && accum ? 1 : 0, ws.data_ptr<float>(),
                    coef.data_ptr<float>(), u16(dx), want_dres ? u16(dres) : nullptr, cur_stream(),
                    want_dres ? nullptr : cf32(scale_shift), G, G > 1 ? gs.data_ptr<float>() : nullptr,
                    dyws.defined() ? dyws.data_ptr<float>() : nullptr, dysp),
        "bn_bwd");
  return {dx, dg, db, dres};
}
std::vector<Tensor> maxpool_fwd(const Tensor& x, int k, int s, int p, bool relu) {
  CHECK_IN(x); CHECK_BF16(x);
  resolve_pending(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  Tensor y = at::empty({N, Ho, Wo, C}, x.options());
  Tensor idx = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  check(pde::maxpool_fwd(u16(x), u16(y), idx.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, k, s, p, relu, cur_stream()),
        "maxpool_fwd");
  return {y, idx};
}
Tensor maxpool_bwd(const Tensor& dy, const Tensor& y, const Tensor& idx, int H, int W, int k, int s, int p,
                   bool relu) {
  CHECK_IN(dy); CHECK_IN(y); CHECK_IN(idx); CHECK_BF16(dy);
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  check(pde::maxpool_bwd(u16(dy), u16(y), idx.data_ptr<uint8_t>(), u16(dx), N, H, W, C, Ho, Wo, k, s, p, relu,
                         cur_stream()),
        "maxpool_bwd");
  return dx;
}
Tensor avgpool_fwd(const Tensor& x) {
  resolve_pending(x);
  CHECK_IN(x); CHECK_BF16(x);
  const int N = x.size(0), C = x.size(-1);
  const int HW = x.numel() / (static_cast<long>(N) * C);
  TORCH_CHECK(C % 8 == 0, "avgpool: C % 8");
  Tensor y = at::empty({N, C}, x.options());
  check(pde::avgpool_fwd(u16(x), u16(y), N, HW, C, cur_stream()), "avgpool_fwd");
  return y;
}
Tensor avgpool_bwd(const Tensor& dy, int H, int W) {
  CHECK_IN(dy); CHECK_BF16(dy);
  const int N = dy.size(0), C = dy.size(1);
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  check(pde::avgpool_bwd(u16(dy), u16(dx), N, H * W, C, cur_stream()), "avgpool_bwd");
  return dx;
}
// counter: device int64[1] RNG counter (advanced on device after the draw); salt: per-call constant.
std::vector<Tensor> dropout_fwd(const Tensor& x, double p, Tensor& counter, int64_t salt, bool channel) {
  CHECK_IN(x); CHECK_BF16(x); CHECK_IN(counter);
  TORCH_CHECK(counter.scalar_type() == at::kLong && counter.numel() >= 1, "counter must be int64[1]");
  Tensor y = at::empty_like(x);
  Tensor mask = at::empty(x.sizes(), x.options().dtype(at::kByte));
  int HW = 1, C = 1;
  if (channel) {
    C = x.size(-1);
    HW = x.numel() / (x.size(0) * C);
  }
  check(pde::dropout_fwd(u16(x), u16(y), mask.data_ptr<uint8_t>(), x.numel(), channel ? 1 : 0, HW, C,
                         static_cast<float>(p), reinterpret_cast<unsigned long long*>(counter.data_ptr()),
                         static_cast<unsigned long long>(salt), cur_stream()),
        "dropout_fwd");
  return {y, mask};
}
Tensor dropout_bwd(const Tensor& dy, const Tensor& mask, double p) {
  CHECK_IN(dy); CHECK_IN(mask);
  Tensor dx = at::empty_like(dy);
  check(pde::dropout_bwd(u16(dy), mask.data_ptr<uint8_t>(), u16(dx), dy.numel(), static_cast<float>(p), cur_stream()),
        "dropout_bwd");
  return dx;
}
Tensor embbag_fwd(const Tensor& w, const Tensor& idx, const Tensor& off) {
  CHECK_IN(w); CHECK_IN(idx); CHECK_IN(off); CHECK_F32(w);
  const int B = off.size(0), D = w.size(1);
  Tensor out = at::empty({B, D}, w.options());
  check(pde::embbag_fwd(w.data_ptr<float>(), idx.data_ptr<int64_t>(), off.data_ptr<int64_t>(), B, idx.numel(), D,
                        out.data_ptr<float>(), cur_stream()),
        "embbag_fwd");
  return out;
}
Tensor embbag_bwd(const Tensor& dy, const Tensor& idx, const Tensor& off, int64_t num) {
  CHECK_IN(dy); CHECK_IN(idx); CHECK_IN(off); CHECK_F32(dy);
  const int B = off.size(0), D = dy.size(1);
  Tensor dw = at::zeros({num, D}, dy.options());
  check(pde::embbag_bwd(dy.data_ptr<float>(), idx.data_ptr<int64_t>(), off.data_ptr<int64_t>(), B, idx.numel(), D,
                        dw.data_ptr<float>(), num, cur_stream()),
        "embbag_bwd");
  return dw;
}

// ------------------------------------------------------------------------------------------------
// Fused MNIST CNN training step
// ------------------------------------------------------------------------------------------------
// Launches forward+loss+backward for the whole batch; returns (loss scalar, slabs).  The caller reduces
// the slabs into a gradient buffer with cnn_reduce (possibly the DDP flat gradient).
Tensor cnn_train(const Tensor& images, const Tensor& tgt, const Tensor& params, Tensor& rng, double p_drop2,
                 double p_drop1, bool training, Tensor& grads, bool accumulate, const optional<Tensor>& gscale,
                 const optional<Tensor>& stamps, const optional<Tensor>& frag_buf, bool prep,
                 const optional<Tensor>& sgd_hp, int64_t stop_after, const optional<Tensor>& sgd_step,
                 const optional<std::vector<int64_t>>& xgmi_view, double xscale) {
  CHECK_IN(images); CHECK_IN(tgt); CHECK_IN(params); CHECK_IN(rng); CHECK_IN(grads);
  pde::XgmiView xv{};
  const bool have_xv = xgmi_view.has_value();
  if (have_xv) {  // XgmiAllreduce.view(): base[8], state, timeout_ticks, flag_bytes, slot_bytes, rank, size, blocks,
                  // read_delay_ticks, host
    const auto& w = *xgmi_view;
    TORCH_CHECK(w.size() == pde::kXgmiMaxRanks + 9, "cnn_train: malformed xgmi view");
    for (int r = 0; r < pde::kXgmiMaxRanks; ++r) xv.base[r] = reinterpret_cast<char*>(w[r]);
    xv.state = reinterpret_cast<uint32_t*>(w[8]);
    xv.timeout_ticks = static_cast<uint64_t>(w[9]);
    xv.flag_bytes = w[10];
    xv.slot_bytes = w[11];
    xv.rank = static_cast<int>(w[12]);
    xv.size = static_cast<int>(w[13]);
    xv.blocks = static_cast<int>(w[14]);
    xv.read_delay_ticks = static_cast<uint64_t>(w[15]);
    xv.host = reinterpret_cast<uint32_t*>(w[16]);
    TORCH_CHECK(!accumulate, "cnn_train: the xGMI gradient exchange replaces accumulation");
  }
  CHECK_F32(images); CHECK_F32(params); CHECK_F32(grads);
  TORCH_CHECK(params.numel() == pde::cnn_num_params(), "cnn_train: params must be the flat Net parameters");
  TORCH_CHECK(grads.numel() == pde::cnn_num_params(), "cnn_train: grads size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(grads.data_ptr()) % 16 == 0, "cnn_train: grads must be 16-B aligned");
  TORCH_CHECK(images.numel() == tgt.numel() * 28 * 28, "cnn_train: images must be [B,1,28,28]");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && rng.scalar_type() == at::kLong, "cnn_train: dtypes");
  const int B = tgt.numel();
  const int ni = pde::cnn_images_per_workgroup();
  const int n = (B + ni - 1) / ni;
  if (stamps.has_value() && stamps->defined())
    TORCH_CHECK(stamps->numel() >= static_cast<long>(n) * 16 && stamps->scalar_type() == at::kLong,
                "cnn_train: stamps must be int64[nwg*16]");
  auto fo = images.options();
  Tensor slabs = at::empty({static_cast<long>(n) * pde::cnn_slab_floats()}, fo);
  Tensor part = at::empty({n}, fo);
  Tensor acts = at::empty({static_cast<long>(pde::cnn_act_rows()) * pde::cnn_act_pitch(n)}, fo.dtype(at::kBFloat16));
  Tensor loss = at::empty({}, fo);
  Tensor frag;
  if (frag_buf.has_value() && frag_buf->defined()) {
    frag = *frag_buf;
    CHECK_IN(frag);
    TORCH_CHECK(frag.nbytes() >= pde::cnn_frag_bytes() && reinterpret_cast<uintptr_t>(frag.data_ptr()) % 16 == 0,
                "cnn_train: frag must be a 16-B aligned buffer of cnn_frag_bytes()");
  } else {
    TORCH_CHECK(prep, "cnn_train: prep=False needs a persistent frag buffer");
    frag = at::empty({static_cast<long>(pde::cnn_frag_bytes())}, fo.dtype(at::kByte));
  }
  if (sgd_hp.has_value() && sgd_hp->defined()) {
    CHECK_IN(*sgd_hp); CHECK_F32(*sgd_hp);
    TORCH_CHECK(sgd_hp->numel() >= pde::HP_COUNT, "cnn_train: sgd_hp must hold the optimiser hyper-parameters");
  }
  check(pde::cnn_train_fused(images.data_ptr<float>(), tgt.data_ptr<int64_t>(), B, params.data_ptr<float>(),
                             frag.data_ptr(),
                             reinterpret_cast<unsigned long long*>(rng.data_ptr()), static_cast<float>(p_drop2),
                             static_cast<float>(p_drop1), training ? 1 : 0, slabs.data_ptr<float>(),
                             part.data_ptr<float>(), reinterpret_cast<uint16_t*>(acts.data_ptr()), n, loss.data_ptr<float>(), grads.data_ptr<float>(), cf32(gscale),
                             accumulate ? 1 : 0, cur_stream(),
                             stamps.has_value() && stamps->defined()
                                 ? reinterpret_cast<unsigned long long*>(stamps->data_ptr())
                                 : nullptr,
                             prep ? 1 : 0, sgd_hp.has_value() && sgd_hp->defined() ? sgd_hp->data_ptr<float>() : nullptr,
                             static_cast<int>(stop_after),
                             sgd_step.has_value() && sgd_step->defined() ? sgd_step->data_ptr<int>() : nullptr,
                             have_xv ? &xv : nullptr, static_cast<float>(xscale)),
        "cnn_train");
  return loss;
}


// Whole MLP training step in one persistent launch (mlp_fused.hip).  Per-layer lists (index l = layer); empty
// tensors stand for absent state (mw / vw / mb / vb by mode, wtbf of layer 0, act / d of index 0).
int mlp_train_grid_py() {
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  return pde::mlp_train_grid(dev);
}

void mlp_train(const Tensor& x, const Tensor& y, const std::vector<Tensor>& w, const std::vector<Tensor>& b,
               const std::vector<Tensor>& gw, const std::vector<Tensor>& gb, const std::vector<Tensor>& mw,
               const std::vector<Tensor>& vw, const std::vector<Tensor>& mb, const std::vector<Tensor>& vb,
               const std::vector<Tensor>& wbf, const std::vector<Tensor>& wtbf, const std::vector<Tensor>& act,
               const std::vector<Tensor>& actT, const std::vector<Tensor>& d, const std::vector<Tensor>& dT,
               Tensor& dlog, Tensor& dlogT, Tensor& loss_part, Tensor& loss, const Tensor& hp, Tensor& step, int mode,
               Tensor& bar, Tensor& err, int grid, const optional<Tensor>& stamps,
               const optional<std::vector<int64_t>>& xgmi_view, double xscale) {
  const int nl = static_cast<int>(w.size());
  TORCH_CHECK(nl >= 1 && nl <= pde::kMlpMaxLayers, "mlp_train: 1..8 layers");
  for (const auto* v : {&b, &gw, &gb, &mw, &vw, &mb, &vb, &wbf, &wtbf, &act, &actT, &d, &dT})
    TORCH_CHECK(static_cast<int>(v->size()) == nl, "mlp_train: every per-layer list has one entry per layer");
  CHECK_IN(x); CHECK_F32(x); CHECK_IN(y);
  TORCH_CHECK(y.scalar_type() == at::kLong && x.dim() == 2, "mlp_train: x [B, in] fp32, y int64");
  const int B = static_cast<int>(x.size(0));
  TORCH_CHECK(B % 32 == 0 && B > 0 && y.numel() == B, "mlp_train: batch must be a multiple of 32");
  TORCH_CHECK(grid > 0, "mlp_train: no resident grid (mlp_train_grid() == 0)");
  auto ptr = [](const Tensor& t) -> void* { return t.defined() && t.numel() > 0 ? t.data_ptr() : nullptr; };
  auto aligned = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  pde::MlpTrainArgs a{};
  a.nl = nl; a.B = B; a.mode = mode;
  TORCH_CHECK(mode >= 0 && mode <= 2, "mlp_train: mode 0 SGD, 1 Adam, 2 AdamW");
  a.x = x.data_ptr<float>(); a.y = y.data_ptr<int64_t>();
  for (int l = 0; l < nl; ++l) {
    const bool last = l == nl - 1;
    CHECK_IN(w[l]); CHECK_F32(w[l]);
    TORCH_CHECK(w[l].dim() == 2, "mlp_train: weights [out, in]");
    const int out = static_cast<int>(w[l].size(0)), in = static_cast<int>(w[l].size(1));
    TORCH_CHECK(in % 8 == 0 && in <= 1024 && (last ? out <= 16 : (out % 8 == 0 && out <= 1024)),
                "mlp_train: in % 8 == 0, in <= 1024, hidden out % 8 == 0 (<= 1024), last out <= 16");
    TORCH_CHECK(l == 0 ? in == x.size(1) : in == w[l - 1].size(0), "mlp_train: layer sizes do not chain");
    auto f32n = [&](const Tensor& t, long n, const char* what) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.numel() == n, "mlp_train: ",
                  what, " of layer ", l);
      return t.data_ptr<float>();
    };
    pde::MlpLayerArgs& L = a.L[l];
    L.in = in; L.out = out;
    L.w = w[l].data_ptr<float>();
    L.b = f32n(b[l], out, "bias");
    L.gw = f32n(gw[l], static_cast<long>(out) * in, "weight grad");
    L.gb = f32n(gb[l], out, "bias grad");
    const bool need_m = mode != 0 || (mw[l].defined() && mw[l].numel() > 0);
    L.mw = need_m ? f32n(mw[l], static_cast<long>(out) * in, "exp_avg / momentum") : nullptr;
    L.mb = need_m ? f32n(mb[l], out, "bias exp_avg / momentum") : nullptr;
    L.vw = mode != 0 ? f32n(vw[l], static_cast<long>(out) * in, "exp_avg_sq") : nullptr;
    L.vb = mode != 0 ? f32n(vb[l], out, "bias exp_avg_sq") : nullptr;
    TORCH_CHECK(wbf[l].is_cuda() && wbf[l].scalar_type() == at::kBFloat16 && wbf[l].is_contiguous() &&
                    wbf[l].numel() == static_cast<long>(out) * in && aligned(wbf[l].data_ptr()),
                "mlp_train: bf16 weight copy of layer ", l);
    L.wbf = u16(wbf[l]);
    L.ldt = last ? 32 : out;
    if (l == 0) {
      L.wtbf = nullptr;
    } else {
      TORCH_CHECK(wtbf[l].is_cuda() && wtbf[l].scalar_type() == at::kBFloat16 && wtbf[l].is_contiguous() &&
                      wtbf[l].dim() == 2 && wtbf[l].size(0) == in && wtbf[l].size(1) == L.ldt,
                  "mlp_train: transposed bf16 copy of layer ", l, " must be [in, ", L.ldt, "]");
      L.wtbf = u16(wtbf[l]);
    }
    auto bfbuf = [&](const Tensor& t, long r, long c, const char* what) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 &&
                      t.size(0) == r && t.size(1) == c && aligned(t.data_ptr()),
                  "mlp_train: ", what, " ", l, " must be bf16 [", r, ", ", c, "]");
      return u16(t);
    };
    a.actT[l] = bfbuf(actT[l], in, B, "actT");
    if (l >= 1) {
      a.act[l] = bfbuf(act[l], B, in, "act");
      a.d[l] = bfbuf(d[l], B, in, "d");
      a.dT[l] = bfbuf(dT[l], in, B, "dT");
    }
    for (void* p : {ptr(w[l]), ptr(gw[l]), ptr(mw[l]), ptr(vw[l])}) TORCH_CHECK(aligned(p), "mlp_train: alignment");
  }
  const int nout = static_cast<int>(w[nl - 1].size(0));
  (void)nout;
  a.dlog = [&] { TORCH_CHECK(dlog.numel() == static_cast<long>(B) * 32 && dlog.scalar_type() == at::kBFloat16,
                             "mlp_train: dlog [B, 32] bf16"); return u16(dlog); }();
  a.dlogT = [&] { TORCH_CHECK(dlogT.numel() == static_cast<long>(B) * 32 && dlogT.scalar_type() == at::kBFloat16,
                              "mlp_train: dlogT [32, B] bf16"); return u16(dlogT); }();
  TORCH_CHECK(loss_part.numel() >= B / 32 && loss_part.scalar_type() == at::kFloat, "mlp_train: loss_part");
  TORCH_CHECK(loss.numel() == 1 && loss.scalar_type() == at::kFloat, "mlp_train: loss");
  CHECK_IN(hp); CHECK_F32(hp);
  TORCH_CHECK(hp.numel() >= pde::HP_COUNT, "mlp_train: hp");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kInt && step.numel() >= 1, "mlp_train: step int32");
  TORCH_CHECK(bar.is_cuda() && bar.scalar_type() == at::kInt && bar.numel() >= 320 && reinterpret_cast<uintptr_t>(bar.data_ptr()) % 16 == 0, "mlp_train: bar int32[320] (zeroed once), 16-B aligned");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 1, "mlp_train: err int32");
  a.loss_part = loss_part.data_ptr<float>(); a.loss = loss.data_ptr<float>();
  a.hp = hp.data_ptr<float>(); a.step = step.data_ptr<int>();
  a.bar = reinterpret_cast<unsigned*>(bar.data_ptr()); a.err = err.data_ptr<int>();
  a.stamps = nullptr;
  // bit 0: the update state is loaded after the weight-gradient tiles instead of behind their operands
  // (PDE_MLP_PRELOAD=0, A/B)
  a.flags = (std::getenv("PDE_MLP_PRELOAD") != nullptr && std::getenv("PDE_MLP_PRELOAD")[0] == '0') ? 1 : 0;
  // (PDE_MLP_FUSE=0: the update of layer j one window after its weight gradient, read back from gw -- A/B)
  if (std::getenv("PDE_MLP_FUSE") != nullptr && std::getenv("PDE_MLP_FUSE")[0] == '0') a.flags |= 2;
  if (stamps.has_value() && stamps->defined()) {
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == at::kLong && stamps->numel() >= 128, "mlp_train: stamps int64[128]");
    a.stamps = reinterpret_cast<long long*>(stamps->data_ptr());
  }
  a.xchg = 0;
  a.xscale = 1.f;
  if (xgmi_view.has_value()) {  // XgmiAllreduce.view(): the in-launch gradient exchange (world > 1, one node)
    const auto& v = *xgmi_view;
    TORCH_CHECK(v.size() == pde::kXgmiMaxRanks + 9, "mlp_train: malformed xgmi view");
    for (int r = 0; r < pde::kXgmiMaxRanks; ++r) a.xv.base[r] = reinterpret_cast<char*>(v[r]);
    a.xv.state = reinterpret_cast<uint32_t*>(v[8]);
    a.xv.timeout_ticks = static_cast<uint64_t>(v[9]);
    a.xv.flag_bytes = v[10];
    a.xv.slot_bytes = v[11];
    a.xv.rank = static_cast<int>(v[12]);
    a.xv.size = static_cast<int>(v[13]);
    a.xv.blocks = static_cast<int>(v[14]);
    a.xv.read_delay_ticks = static_cast<uint64_t>(v[15]);
    a.xv.host = reinterpret_cast<uint32_t*>(v[16]);
    a.xchg = 1;
    a.xscale = static_cast<float>(xscale);
    int ins[pde::kMlpMaxLayers], outs[pde::kMlpMaxLayers];
    for (int l = 0; l < nl; ++l) {
      ins[l] = a.L[l].in; outs[l] = a.L[l].out;
      a.xoff[l] = pde::mlp_xchg_floats(ins, outs, l);  // the tiles of layers 0 .. l-1 come first
    }
    TORCH_CHECK(pde::mlp_xchg_floats(ins, outs, nl) * 4 <= a.xv.slot_bytes,
                "mlp_train: the xGMI instance's slot is smaller than the exchanged gradient tiles (",
                pde::mlp_xchg_floats(ins, outs, nl) * 4, " B)");
    TORCH_CHECK(a.xv.blocks >= grid, "mlp_train: the xGMI instance needs >= ", grid, " flag blocks");
    TORCH_CHECK(mode != 0 && (a.flags & 2) == 0, "mlp_train: the exchange needs the fused Adam / AdamW form");
  }
  check(pde::mlp_train_step(a, grid, cur_stream()), "mlp_train");
}

// Plain SGD on the flat CNN parameters + fragment-image refresh (after the gradient all-reduce).
}  // namespace
namespace pde {
// (declared here, not in pde_kernels.h: cnn_fused.hip is the only definition, bindings.cpp the only caller)
hipError_t cnn_adamw_fused(float* params, const float* grads, float* m, float* v, const float* hp, void* frag,
                           int* step, hipStream_t s);
}  // namespace pde
namespace {

// AdamW over the flat CNN parameters + fragment refresh, one launch (FusedCNN.adamw_step)
void cnn_adamw(Tensor& params, const Tensor& grads, Tensor& m, Tensor& v, const Tensor& hp, Tensor& frag,
               Tensor& step) {
  CHECK_IN(params); CHECK_IN(grads); CHECK_IN(m); CHECK_IN(v); CHECK_IN(hp); CHECK_IN(frag);
  CHECK_F32(params); CHECK_F32(grads); CHECK_F32(m); CHECK_F32(v); CHECK_F32(hp);
  const long n = pde::cnn_num_params();
  TORCH_CHECK(params.numel() == n && grads.numel() == n && m.numel() == n && v.numel() == n, "cnn_adamw: sizes");
  TORCH_CHECK(hp.numel() >= pde::HP_COUNT, "cnn_adamw: hp");
  TORCH_CHECK(frag.nbytes() >= pde::cnn_frag_bytes(), "cnn_adamw: frag size");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kInt && step.numel() >= 2, "cnn_adamw: step int32[2]");
  check(pde::cnn_adamw_fused(params.data_ptr<float>(), grads.data_ptr<float>(), m.data_ptr<float>(),
                             v.data_ptr<float>(), hp.data_ptr<float>(), frag.data_ptr(), step.data_ptr<int>(),
                             cur_stream()),
        "cnn_adamw");
}

void cnn_sgd(Tensor& params, const Tensor& grads, const Tensor& hp, Tensor& frag, const optional<Tensor>& step) {
  CHECK_IN(params); CHECK_IN(grads); CHECK_IN(hp); CHECK_IN(frag);
  CHECK_F32(params); CHECK_F32(grads); CHECK_F32(hp);
  TORCH_CHECK(params.numel() == pde::cnn_num_params() && grads.numel() == pde::cnn_num_params(), "cnn_sgd: sizes");
  TORCH_CHECK(hp.numel() >= pde::HP_COUNT, "cnn_sgd: hp");
  TORCH_CHECK(frag.nbytes() >= pde::cnn_frag_bytes(), "cnn_sgd: frag size");
  if (step.has_value() && step->defined())
    TORCH_CHECK(step->is_cuda() && step->scalar_type() == at::kInt, "cnn_sgd: step must be a device int32 tensor");
  check(pde::cnn_sgd_fused(params.data_ptr<float>(), grads.data_ptr<float>(), hp.data_ptr<float>(), frag.data_ptr(),
                           cur_stream(), step.has_value() && step->defined() ? step->data_ptr<int>() : nullptr),
        "cnn_sgd");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("cnn_train", &cnn_train, py::arg("images"), py::arg("tgt"), py::arg("params"), py::arg("rng"),
        py::arg("p_drop2"), py::arg("p_drop1"), py::arg("training"), py::arg("grads"), py::arg("accumulate"),
        py::arg("gscale") = py::none(), py::arg("stamps") = py::none(), py::arg("frag") = py::none(),
        py::arg("prep") = true, py::arg("sgd_hp") = py::none(), py::arg("stop_after") = -1,
        py::arg("sgd_step") = py::none(), py::arg("xgmi_view") = py::none(), py::arg("xscale") = 1.0);
  m.def("mlp_train_grid", &mlp_train_grid_py);
  m.def("mlp_train", &mlp_train, py::arg("x"), py::arg("y"), py::arg("w"), py::arg("b"), py::arg("gw"), py::arg("gb"),
        py::arg("mw"), py::arg("vw"), py::arg("mb"), py::arg("vb"), py::arg("wbf"), py::arg("wtbf"), py::arg("act"),
        py::arg("actT"), py::arg("d"), py::arg("dT"), py::arg("dlog"), py::arg("dlogT"), py::arg("loss_part"),
        py::arg("loss"), py::arg("hp"), py::arg("step"), py::arg("mode"), py::arg("bar"), py::arg("err"),
        py::arg("grid"), py::arg("stamps") = py::none(), py::arg("xgmi_view") = py::none(),
        py::arg("xscale") = 1.0);
  m.def("cnn_adamw", &cnn_adamw, py::arg("params"), py::arg("grads"), py::arg("m"), py::arg("v"), py::arg("hp"),
        py::arg("frag"), py::arg("step"));
  m.def("cnn_sgd", &cnn_sgd, py::arg("params"), py::arg("grads"), py::arg("hp"), py::arg("frag"),
        py::arg("step") = py::none());
  m.def("clear_last_error", []() { return static_cast<int>(hipGetLastError()); },
        "Read and reset the HIP last-error state (after an aborted stream capture).");
  m.def("bn_reserve_headroom", &pde::bn_reserve_headroom, py::arg("blocks"),
        "Reserve (> 0) / release (< 0) CUs for spinning side-stream kernels; returns the one-launch BatchNorm's "
        "resident cap");
  m.def("bn_headroom_reserved", &pde::bn_headroom_reserved,
        "CUs currently reserved (bn_reserve_headroom) for kernels spinning on other streams");
  m.def("bn_launch_stats", []() {
    long one = 0, multi = 0;
    int last = 0, cap = 0;
    pde::bn_launch_stats(&one, &multi, &last, &cap);
    py::dict d;
    d["one_launch"] = one;
    d["multi_launch"] = multi;
    d["last_grid"] = last;
    d["cap"] = cap;
    return d;
  });
  m.def("graph_upload",
        [](int64_t exec) {  // torch.cuda.CUDAGraph.raw_cuda_graph_exec(): upload the executable graph's launch
                            // resources NOW (current stream), not inside the first timed replay
          const hipError_t e = hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec),
                                              cur_stream());
          return static_cast<int>(e);
        },
        py::arg("exec"));
  m.def("cnn_frag_bytes", &pde::cnn_frag_bytes);
  m.def("cnn_num_params", &pde::cnn_num_params);
  m.def("cnn_smem_bytes", &pde::cnn_smem_bytes);
  m.doc() = "MI355X (gfx950) native kernels for pytorch_distributed_examples_amd";
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_dgrad", &linear_dgrad);
  m.def("linear_wgrad", &linear_wgrad, py::arg("dy"), py::arg("x"), py::arg("out") = py::none(),
        py::arg("accumulate") = false);
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("wf"), py::arg("bias"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("relu"), py::arg("out_f32"), py::arg("defer") = false);
  m.def("pending_conv_count", &pending_conv_count);
  m.def("bn_fold_shards", []() { return pde::kBnShards; });
  m.def("bn_fold_plan", &bn_fold_plan, py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Co1"),
        py::arg("R1"), py::arg("S1"), py::arg("stride1"), py::arg("pad1"), py::arg("Co2"), py::arg("R2"),
        py::arg("S2"), py::arg("stride2"), py::arg("pad2"), py::arg("groups"));
  m.def("conv_fwd_bn", &conv_fwd_bn, py::arg("x"), py::arg("wf"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("groups"), py::arg("stats_sums"), py::arg("stats_ticket"), py::arg("gamma"),
        py::arg("beta"), py::arg("running_mean"), py::arg("running_var"), py::arg("eps"), py::arg("momentum"),
        py::arg("fold_ss"), py::arg("relu"), py::arg("defer") = false);
  m.def("bn_bwd_slab_uses", &bn_bwd_slab_uses);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("wd"), py::arg("H"), py::arg("W"), py::arg("R"),
        py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("aux") = py::none(), py::arg("w_fwd_layout") = false,
        py::arg("add_aux") = false, py::arg("defer") = false);
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("Co"), py::arg("Ci"), py::arg("out") = py::none(), py::arg("accumulate") = false);
  m.def("cast_bf16", &cast_bf16);
  m.def("cast_bf16_into", &cast_bf16_into);
  m.def("cast_f32", &cast_f32);
  m.def("cast_f32_into", &cast_f32_into);
  m.def("nchw_to_nhwc", &nchw_to_nhwc);
  m.def("conv_layout_table", &conv_layout_table, py::arg("ws"), py::arg("fwds"), py::arg("dgrads"),
        py::arg("cps"), py::arg("cops"));
  m.def("conv_layouts_step", &conv_layouts_step, py::arg("table"), py::arg("n"), py::arg("blocks_x"));
  m.def("conv_w_fwd", &conv_w_fwd, py::arg("w"), py::arg("Cp"), py::arg("Cop"), py::arg("out") = py::none());
  m.def("conv_w_dgrad", &conv_w_dgrad, py::arg("w"), py::arg("Cip"), py::arg("Cop"), py::arg("out") = py::none());
  m.def("conv_wgrad_oihw", &conv_wgrad_oihw);
  m.def("colsum", &colsum, py::arg("x"), py::arg("ncols") = -1, py::arg("out") = py::none(),
        py::arg("accumulate") = false);
  m.def("relu_bwd", &relu_bwd);
  m.def("time_stamp",
        [](Tensor& stamps, int slot) {
          TORCH_CHECK(stamps.is_cuda() && stamps.scalar_type() == at::kLong && slot >= 0 && slot < stamps.numel(),
                      "time_stamp: int64 GPU tensor and a slot inside it");
          check(pde::time_stamp(reinterpret_cast<unsigned long long*>(stamps.data_ptr()), slot, cur_stream()),
                "time_stamp");
        },
        py::arg("stamps"), py::arg("slot"));
  m.def("wall_clock_hz", []() {
    int dev = 0, khz = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    return static_cast<double>(khz) * 1e3;
  });
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_fused", &ce_fused, py::arg("x"), py::arg("tgt"), py::arg("dx_out") = py::none());
  m.def("linear_fwd_out", &linear_fwd_out);
  m.def("linear_dgrad_out", &linear_dgrad_out);
  m.def("linear_wgrad_bias", &linear_wgrad_bias);
  m.def("gemm_pair_begin", &gemm_pair_begin);
  m.def("gemm_pair_end", &gemm_pair_end, py::arg("abort") = false, py::arg("defer") = false);
  m.def("gemm_flush_deferred", &gemm_flush_deferred);
  m.def("gemm_deferred_count", &gemm_deferred_count);
  m.def("cast_rows_ones", &cast_rows_ones);
  m.def("gather_rows_counter", &gather_rows_counter, py::arg("src"), py::arg("labels"), py::arg("idx"),
        py::arg("counter"), py::arg("x_out"), py::arg("y_out"));
  m.def("ce_bwd", &ce_bwd);
  m.def("log_softmax_fwd", &log_softmax_fwd);
  m.def("log_softmax_bwd", &log_softmax_bwd);
  m.def("mse_fwd", &mse_fwd);
  m.def("mse_bwd", &mse_bwd);
  m.def("optim_table", &optim_table);
  m.def("optim_step", &optim_step);
  m.def("optim_step_range", &optim_step_range);
  m.def("optim_chunk_elems", &pde::optim_chunk_elems);
  m.def("optim_attach", &optim_attach);
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("eps"), py::arg("momentum"), py::arg("res"), py::arg("relu"),
        py::arg("groups") = 1);
  // 1 if a one-launch BatchNorm wait timed out since the last reset (synchronises the device)
  m.def("bn_error", [](bool reset) { return pde::bn_error(reset ? 1 : 0); }, py::arg("reset") = true);
  m.def("cnn_tail_error", [](bool reset) { return pde::cnn_tail_error(reset ? 1 : 0); }, py::arg("reset") = true);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("mean"), py::arg("invstd"),
        py::arg("gamma"), py::arg("relu"), py::arg("want_dres"), py::arg("dg_out") = py::none(),
        py::arg("db_out") = py::none(), py::arg("scale_shift") = py::none(), py::arg("groups") = 1,
        py::arg("accum") = true);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("embbag_fwd", &embbag_fwd);
  m.def("embbag_bwd", &embbag_bwd);
}
