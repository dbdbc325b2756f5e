// Host-side launcher declarations for the CDNA4 (gfx950) kernels in csrc/kernels/*.hip.
//
// Every launcher takes raw device pointers plus the hipStream_t it must enqueue on, does no
// allocation and no synchronisation (so the caller may capture it into a hipGraph), and returns
// a hipError_t from hipGetLastError() after the launch.  bindings.cpp wraps them for torch.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "xgmi_view.h"

namespace pde {

// ---------------------------------------------------------------------------------------------
// GEMM / implicit-GEMM convolution (gemm.hip)
// ---------------------------------------------------------------------------------------------
// Epilogue flags (bitwise OR).
enum EpiFlags : int {
  EPI_NONE = 0,
  EPI_BIAS = 1,       // + bias[n] (fp32)
  EPI_RELU = 2,       // max(0, .)
  EPI_DRELU = 4,      // * (aux[m, n] > 0)   aux: bf16 [M, ldaux] (saved post-ReLU activation)
  EPI_OUT_F32 = 8,    // output fp32 (else bf16)
  EPI_ACCUM = 16,     // out += result (fp32 output only)
  EPI_OIHW = 32,      // conv weight gradient: m = co, n = (r*S + s)*Cp + ci written to out[co][ci][r][s]
  EPI_ADD_AUX = 64,   // + aux[m, n] (bf16): a second gradient branch summed in the epilogue
                      // (ci >= oihw_ci skipped; fp32 output)
};

// Operand description.  The GEMM computes  C[m, n] = sum_k A[m, k] * B[n, k].
//   kind 0 (dense):   element (r, k) at ptr[r * ld_r + k * ld_k]; one of ld_r / ld_k must be 1.
//   kind 1 (im2col):  NHWC activation gather.  r indexes output pixels (n, ho, wo), k indexes
//                     (kh, kw, c) with c fastest.  Requires C % 8 == 0.
//   kind 2 (im2col^T): same gather but r indexes (kh, kw, c) and k indexes output pixels
//                     (the weight-gradient "B" operand).
//   kind 3 (dgrad):   transposed-conv gather from dy (NHWC, C = Cout of the forward conv):
//                     r indexes input pixels (n, h, w), k indexes (kh, kw, co); element is
//                     dy[n, (h + pad - kh) / s, (w + pad - kw) / s, co] when divisible & in range.
struct ConvGeom {
  int N, H, W, C;      // gathered tensor dims (NHWC)
  int R, S;            // kernel
  int stride, pad;
  int Ho, Wo;          // output spatial dims of the gather (kind 1/2: conv output; kind 3: H, W of dx)
};

struct Operand {
  const void* ptr;
  int kind;            // 0 dense, 1 im2col, 2 im2col^T, 3 dgrad gather
  long ld_r, ld_k;     // dense strides (elements)
  ConvGeom g;          // gather geometry
};

// BatchNorm folded into the convolutions around it (forward, training mode; VERDICT r3 ask 1).
//   producer (the conv whose output x the BatchNorm normalises): its epilogue adds per-tile column sums of the
//     stored bf16 outputs into `sums` -- fixed point (S1 = sum x * 2^32, S2 = sum x^2 * 2^20, int64 atomics:
//     exact, so the statistics do not depend on arrival order), SHARDED by row tile (kBnShards copies, tile tm
//     adds into shard tm % kBnShards: hundreds of row tiles adding into the same 2C words would serialise at
//     the memory side).  Every block then arrives on `ticket`; the LAST one reads-and-zeroes the shards
//     (atomic exchange), derives mean / invstd / scale / shift per (group, channel), writes them and the
//     running statistics (group order), and resets the ticket -- the BatchNorm's whole finalize, once;
//   consumer (the next conv): every block copies its group's scale / shift [2][C] into LDS (overlapping its
//     first operand loads) and its A loader applies relu(x * scale + shift) to every in-range element while
//     staging the tile (padding taps stay zero).  Blocks of the first N-tile also write the activation `act`
//     (the backward's operand): a 1x1 consumer every A element, a 3x3 stride-1 consumer the centre tap.
constexpr int kBnShards = 16;
struct BnStatsOut {
  long long* sums;        // [kBnShards][G][2][C] zero-initialised; nullptr: off
  int* ticket;            // zero-initialised arrival counter
  int nblocks;            // blocks of the producing launch (set by the launcher)
  int C;                  // real channels (the output may be padded)
  int G, rows_per_group;  // micro-batch groups; rows per group (a multiple of the 64-row tile)
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float* save_mean;       // [G][C]
  float* save_invstd;     // [G][C]
  float* ss;              // [G][2][C]: scale, shift (the consumer's coefficients, the backward's ReLU mask)
  float eps, momentum;
  int debug;              // PDE_BN_FOLD_DEBUG cost attribution (timing only, results invalid): 1 skip the
                          // finalize tail, 2 skip the statistics epilogue
};
constexpr int kBnFoldMaxC = 512;  // 4 KB of scale / shift: 4 blocks of 36 KB still fit a CU
struct BnFoldIn {
  const float* ss;        // [G][2][C] from the producer's finalize; nullptr: off
  uint16_t* act;          // [rows][C] bf16 activation written by the first N-tile's blocks
  int C, G, rows_per_group;
  int relu;
  int center;             // 1: 3x3 stride-1 pad-1 gather, act from the centre tap; 0: 1x1 (every element)
  int debug;              // PDE_BN_FOLD_DEBUG & 4: skip the A transform (timing only)
};

struct GemmArgs {
  int M, N, K;
  Operand a, b;
  void* out; long ldo;             // out[m * ldo + n]
  const float* bias;               // EPI_BIAS (bias[n] for n < nbias, 0 beyond: padded channels)
  int nbias;
  const uint16_t* aux; long ldaux; // EPI_DRELU / EPI_ADD_AUX (bf16 bits)
  int epi;
  int splitk;                      // >1: fp32 partial slabs in workspace, then reduce + epilogue
  float* workspace;                // splitk * M * N fp32
  int oihw_ci, oihw_rs, oihw_cp;   // EPI_OIHW: real Cin, R*S, padded Cin of the gathered activation
  int* tickets;                    // set by gemm_bf16: per-tile arrival counters of the in-kernel split-K reduce
  float* bias_grad;                // EPI_OUT_F32: output column bias_col goes to bias_grad[m] instead (the
  int bias_col;                    //   "ones column" bias gradient of a linear wgrad), columns beyond are dropped
  int* splits_out;                 // != nullptr: a split-K GEMM leaves its slabs UNREDUCED for a consumer that
                                   //   sums them itself (the one-launch BatchNorm); the split count used is stored
                                   //   here (1: the output was written directly)
  BnStatsOut bn_out;               // producer side of a folded BatchNorm (bn_out.sums != nullptr)
  BnFoldIn bn_in;                  // consumer side (bn_in.ss != nullptr): A = relu(x * scale + shift)
  int wt;                          // vector output / slab stores write-through (set by gemm_bf16*: PDE_GEMM_WT)
};
// Whether gemm_bf16 would run `a` on a path whose epilogue emits BatchNorm statistics (bn_out): the 64x64
// FAST tile, bf16 output without epilogue ops, and no split-K (or one reduced inside the launch).
bool gemm_bn_stats_ok(const GemmArgs& a, hipStream_t s);
// Whether gemm_bf16 can apply a folded BatchNorm in `a`'s A loader (bn_in): the 64x64 FAST tile with a dense
// (1x1) or 3x3 stride-1 gathered A, K-contiguous dense B, rows_per_group a multiple of 64, C <= kBnFoldMaxC.
bool gemm_bn_fold_ok(const GemmArgs& a);
// Sum `splits` fp32 slabs [splits][M][N] in z order into bf16 out[M][N] (the plain split-K reduction of a
// GEMM with no epilogue) -- the fallback when a deferred conv output is read by something else.
hipError_t gemm_reduce_slabs_bf16(float* ws, int splits, int M, int N, uint16_t* out, hipStream_t s);

hipError_t gemm_bf16(const GemmArgs& args, hipStream_t stream);
// Two independent GEMMs (a layer's dgrad and wgrad) in one launch when both run on the 64x64 FAST tile, their
// split-K slab reductions in one more; otherwise two ordinary gemm_bf16 launches (problem 0 first).
// defer_split1 != nullptr: problem 1's split-K slab reduction is NOT launched; its split count is returned
// there (0 / 1: nothing deferred) and the caller reduces it later with gemm_reduce_jobs.
struct OptimSeg;
// seg (optional): optimiser blocks appended to the launch (their own chunk range; run as a separate launch when
// the two problems cannot be paired)
// defer_split0 != nullptr: problem 0's split-K slab reduction is NOT launched either; its split count is returned
// there (0 / 1: nothing deferred, the output is written) and a consumer sums the slabs itself (bn_bwd's dys).
hipError_t gemm_bf16_pair(const GemmArgs& a0, const GemmArgs& a1, hipStream_t stream, int* defer_split1 = nullptr,
                          const OptimSeg* seg = nullptr, int* defer_split0 = nullptr);
bool gemm_pair_enabled();
// A deferred split-K slab reduction (vector form: N % 4 == 0, 16-B aligned slabs) with the fp32 epilogue of
// its GEMM (accumulate, OIHW remap, ones-column bias gradient).
struct ReduceJob {
  float* workspace;
  void* out;
  float* bias_grad;
  long ldo;
  int M, N, splits, epi, oihw_ci, oihw_rs, oihw_cp, bias_col;
};
constexpr int kMaxReduceJobs = 24;
hipError_t gemm_reduce_jobs(const ReduceJob* jobs, int n, hipStream_t stream);

// ---------------------------------------------------------------------------------------------
// Elementwise / layout (elementwise.hip)
// ---------------------------------------------------------------------------------------------
hipError_t cast_f32_bf16(const float* in, uint16_t* out, long n, hipStream_t s);
// stamps[slot] = the 100 MHz wall clock when this node runs (phase attribution inside captured graphs)
hipError_t time_stamp(unsigned long long* stamps, int slot, hipStream_t s);
// in [rows][cols] fp32 -> out [rows][ldo] bf16, plus out[r][cols] = 1 when ones != 0 (the ones column a
// linear wgrad GEMM turns into the bias gradient)
hipError_t cast_rows_bf16(const float* in, int rows, int cols, uint16_t* out, int ldo, int ones, hipStream_t s);
hipError_t cast_bf16_f32(const uint16_t* in, float* out, long n, hipStream_t s);
// NCHW fp32 -> NHWC bf16 with channel padding to Cp (zero fill)
hipError_t nchw_f32_to_nhwc_bf16(const float* in, uint16_t* out, int N, int C, int H, int W, int Cp,
                                 hipStream_t s);
// [Cout, Cin, R, S] fp32 -> [Cop, R, S, Cp] bf16 (forward igemm B operand, K-contiguous, zero padded)
hipError_t conv_weight_fwd_layout(const float* w, uint16_t* out, int Co, int Ci, int R, int S, int Cp, int Cop,
                                  hipStream_t s);
// [Cout, Cin, R, S] fp32 -> [Cip, R, S, Cop] bf16 (dgrad B operand: n = ci, k = (r, s, co), zero padded)
hipError_t conv_weight_dgrad_layout(const float* w, uint16_t* out, int Co, int Ci, int R, int S, int Cip, int Cop,
                                    hipStream_t s);
// Both bf16 GEMM layouts of several KxK conv weights in one launch (run after the optimizer update: the
// optimizer-maintained compute copies of the convs whose layout is not the parameter's own order).
struct ConvLayoutEntry {
  const float* w;    // [Co][Ci][R][S] fp32
  uint16_t* fwd;     // [Cop][R][S][Cp]
  uint16_t* dgrad;   // [Cp][R][S][Cop]
  int Co, Ci, R, S, Cp, Cop;
};
hipError_t conv_weight_layouts_multi(const ConvLayoutEntry* dev_table, int n, int blocks_x, hipStream_t s);
// dW gemm output [Cout, R*S*Cp] fp32 -> [Cout, Cin, R, S] fp32 (optionally accumulate)
hipError_t conv_wgrad_to_oihw(const float* in, float* out, int Co, int Ci, int R, int S, int Cp, int accum,
                              hipStream_t s);
// column sums of a bf16 [M, N] matrix into fp32 [N] (bias gradient); accum adds to out
hipError_t colsum_bf16(const uint16_t* x, float* out, int M, int N, int accum, hipStream_t s);
// Vectorised deterministic variant for N % 8 == 0; ws holds ws_blocks * N floats (falls back otherwise).
hipError_t colsum_bf16_ws(const uint16_t* x, float* out, int M, int N, int accum, float* ws, int ws_blocks,
                          hipStream_t s);
hipError_t relu_bwd_bf16(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Losses (loss.hip).  mode 0 = cross-entropy on logits, mode 1 = NLL on log-probabilities.
// ---------------------------------------------------------------------------------------------
hipError_t ce_fwd(const void* x, int x_f32, const int64_t* tgt, int B, int V, int mode, float* loss, float* lse,
                  hipStream_t s);
hipError_t ce_bwd(const void* x, int x_f32, const int64_t* tgt, const float* lse, const float* gout, int B, int V,
                  int mode, void* dx, int dx_f32, hipStream_t s);
// Mean cross-entropy and its input gradient in one launch (mode 0 of ce_fwd/ce_bwd with d loss = 1):
// loss[0] = mean_b (lse_b - x[b, t_b]),  dx[b, v] = (softmax(x_b)_v - [v == t_b]) / B  (bf16).
hipError_t ce_fused(const void* x, int x_f32, const int64_t* tgt, int B, int V, float* loss, uint16_t* dx, int ldx,
                    hipStream_t s);
hipError_t log_softmax_fwd(const void* x, int x_f32, int B, int V, float* y, hipStream_t s);
hipError_t log_softmax_bwd(const float* dy, const float* y, int B, int V, void* dx, int dx_f32, hipStream_t s);
hipError_t mse_fwd(const void* p, int p_f32, const float* t, long n, float* loss, hipStream_t s);
hipError_t mse_bwd(const void* p, int p_f32, const float* t, const float* gout, long n, void* dx, int dx_f32,
                   hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Optimisers (optim.hip): one launch over every tensor of a parameter set.
// ---------------------------------------------------------------------------------------------
struct OptimEntry {
  float* param;          // fp32 master weight
  const float* grad;     // fp32 gradient (nullptr: treated as zero)
  float* exp_avg;        // Adam/AdamW m, SGD momentum buffer
  float* exp_avg_sq;     // Adam/AdamW v
  uint16_t* bf16_copy;   // optional bf16 compute copy (same element order) written after the update
  long size;
  int vec;               // every pointer 16-byte aligned: 16-byte loads / stores
  int pad;
};
struct OptimChunk {      // elements [start, start + count) of tensor `tensor`
  int tensor, start, count, pad;
};
enum HParam { HP_LR = 0, HP_BETA1, HP_BETA2, HP_EPS, HP_WD, HP_MOMENTUM, HP_GRAD_SCALE, HP_COUNT };
int optim_chunk_elems();  // chunk size the host must cut tensors into
// A range of optimiser chunks [c0, c1) run by `blocks` extra blocks appended to a GEMM pair launch
// (gemm_bf16_pair) -- or by its own launch (multi_tensor_optim_range).  publish: this segment is the step's
// last one (its last block stores the new device step count).
struct OptimSeg {
  const OptimEntry* tab;
  const OptimChunk* chunks;
  const float* hp;
  int* step;
  int c0, c1, mode, publish, blocks, pad;
};
int optim_segment_blocks(int nchunks);
hipError_t multi_tensor_optim_range(int mode, const OptimEntry* dev_table, const OptimChunk* dev_chunks, int c_begin,
                                    int c_end, const float* dev_hparams, int* dev_step, int publish, hipStream_t s);
// mode 0 SGD, 1 Adam, 2 AdamW.  dev_hparams: float[HP_COUNT]; dev_step: int[2] = {steps taken so far,
// arrival counter (0 between launches)}; the step is advanced on device by the update itself.
hipError_t multi_tensor_optim(int mode, const OptimEntry* dev_table, const OptimChunk* dev_chunks, int nchunks,
                              const float* dev_hparams, int* dev_step, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// BatchNorm / pooling / dropout / EmbeddingBag (norm_pool.hip).  Activations NHWC bf16, [P = N*H*W][C].
// ---------------------------------------------------------------------------------------------
// ws needs bn_workspace_blocks * 2 * C floats.  groups > 1: P rows = `groups` equal micro-batches, each
// normalised with its own statistics (mean / invstd [groups][C], scale_shift [groups][2C], coef [groups][3C]);
// gscratch: 2 * groups * C floats.
int bn_workspace_blocks(int P, int C, int groups = 1);
// slabs != nullptr (splits > 1): x is the UNREDUCED output of a split-K conv GEMM (GemmArgs::splits_out):
// the BatchNorm sums the fp32 slabs [splits][P][C] in z order, rounds to bf16, WRITES x and normalizes it --
// the GEMM's separate slab-reduction launch is gone.
// Co-residency budget of the one-launch BatchNorm: reserve (blocks > 0) / release (< 0) CUs that kernels on
// other streams of this process may hold while it runs (spinning side-stream ring sends / receives, an
// overlapped RCCL all-reduce); returns the resulting resident cap.  Grids shrink to the cap; a BatchNorm whose
// minimal grid exceeds it is refused up front and runs multi-launch.
int bn_reserve_headroom(int blocks);
// rows [c x rows, (c+1) x rows) of idx (c = counter[0], advanced by the launch) gathered from src [N, row_elems]
// fp32 / labels [N] into dst / ydst (elastic/rewire.py: the per-replay batch gather inside the captured graph)
hipError_t gather_rows_counter(const float* src, const int64_t* labels, const int64_t* idx, int64_t n_idx,
                               uint32_t* counter, int rows, int row_elems, float* dst, int64_t* ydst, hipStream_t s);
int bn_headroom_reserved();  // CUs currently reserved for spinning side-stream kernels
void bn_launch_stats(long* one_launch, long* multi_launch, int* last_grid, int* cap);
hipError_t bn_fwd_train(const uint16_t* x, int P, int C, const float* gamma, const float* beta, float eps,
                        float momentum, float* running_mean, float* running_var, float* save_mean,
                        float* save_invstd, float* scale_shift, float* ws, const uint16_t* res, int relu,
                        uint16_t* y, hipStream_t s, const float* slabs = nullptr, int splits = 1, int groups = 1,
                        float* gscratch = nullptr);
// 1 when a one-launch BatchNorm wait timed out (a block of the grid was never resident); reset clears it
int bn_error(int reset);
hipError_t bn_apply(const uint16_t* x, int P, int C, const float* scale, const float* shift, const uint16_t* res,
                    int relu, uint16_t* y, hipStream_t s);
// dgamma / dbeta are written, or added to when accum_params != 0 (direct accumulation into .grad).
// ss (optional, the forward's fp32 scale/shift [2C] of a BatchNorm WITHOUT residual): the ReLU mask is
// recomputed from x (y is not read by the one-launch kernel)
hipError_t bn_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean, const float* invstd,
                  const float* gamma, int P, int C, int relu, float* dgamma, float* dbeta, int accum_params, float* ws,
                  float* coef, uint16_t* dx, uint16_t* dres, hipStream_t s, const float* ss = nullptr, int groups = 1,
                  float* gscratch = nullptr, const float* dys = nullptr, int dysplits = 1);
// (dys / dysplits > 1: dy's values are still the unreduced split-K slabs [dysplits][P][C] fp32 of the conv dgrad
// that produced it -- summed by the BatchNorm itself, or reduced into dy first where its kernel cannot)
hipError_t maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                       int k, int st, int p, int relu, hipStream_t s);
hipError_t maxpool_bwd(const uint16_t* dy, const uint16_t* y, const uint8_t* idx, uint16_t* dx, int N, int H, int W,
                       int C, int Ho, int Wo, int k, int st, int p, int relu, hipStream_t s);
hipError_t avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s);
hipError_t avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s);
hipError_t dropout_fwd(const uint16_t* x, uint16_t* y, uint8_t* mask, long n, int mode, int HW, int C, float p,
                       unsigned long long* counter, unsigned long long salt, hipStream_t s);
hipError_t dropout_bwd(const uint16_t* dy, const uint8_t* mask, uint16_t* dx, long n, float p, hipStream_t s);
hipError_t embbag_fwd(const float* w, const int64_t* idx, const int64_t* off, int B, long L, int D, float* out,
                      hipStream_t s);
// ---------------------------------------------------------------------------------------------
// Fused MNIST-CNN training step (cnn_fused.hip): forward + NLL + backward of horovod/mnist_horovod.py's
// Net per image in LDS.  params: flat fp32 in torch parameter order (cnn_num_params() floats).
// slabs: nwg * cnn_slab_floats() floats; loss_part: nwg floats; acts: cnn_act_rows() x cnn_act_pitch(nwg) bf16.
// ---------------------------------------------------------------------------------------------
int cnn_num_params();
size_t cnn_smem_bytes();
int cnn_images_per_workgroup();
// Three launches: the weight-fragment prep, the fused training kernel (per-workgroup gradient slabs +
// loss partials), then the deterministic slab reduction into `grads` (16-B aligned; (+)= gscale * sum)
// which also finalises the loss and advances the dropout counter.
size_t cnn_frag_bytes();  // workspace for the per-step bf16 weight-fragment image (16-B aligned)
// prep = 0 skips the fragment prep (the image is already current: the previous step's fused SGD wrote it).
// sgd_hp != nullptr fuses plain SGD (lr = sgd_hp[HP_LR], grad scale sgd_hp[HP_GRAD_SCALE]) and the
// fragment refresh into the slab reduction.  xv (world > 1, an XgmiAllreduce's view): the reduction
// first exchanges each workgroup's gradient chunk with every peer over xGMI and sums all ranks' chunks in
// rank order (x xscale), so the update stays fused at any world size -- 2 launches per step.
int cnn_slab_floats();  // per-workgroup slab (every gradient except fc1's weight)
int cnn_act_rows();     // rows of the per-batch activation image feeding the fc1 weight-gradient GEMM
int cnn_act_pitch(int nwg);  // its row pitch (bf16 elements)
hipError_t cnn_train_fused(const float* images, const int64_t* tgt, int B, float* params, void* frag,
                           unsigned long long* rng, float p_drop2, float p_drop1, int training, float* slabs,
                           float* loss_part, uint16_t* acts, int nwg, float* loss, float* grads, const float* gscale,
                           int accumulate, hipStream_t s, unsigned long long* stamps = nullptr, int prep = 1,
                           const float* sgd_hp = nullptr, int stop_after = -1, int* sgd_step = nullptr,
                           const XgmiView* xv = nullptr, float xscale = 1.f);
// params -= lr * gscale * grads (plain SGD) and the matching fragment-image refresh, one launch (used
// after the gradient all-reduce when world > 1).
// 1 when the single-process fused tail's grid barrier timed out (PDE_CNN_FUSED_TAIL); reset clears it
int cnn_tail_error(int reset);
hipError_t cnn_sgd_fused(float* params, const float* grads, const float* hp, void* frag, hipStream_t s,
                         int* step = nullptr);  // step: the optimiser's device step counter (+1 per call)

// dw (+)= EmbeddingBag-sum gradient; deterministic (row-owner scan) for tables with rows * L <= 2^26 and
// D <= 256, fp32 atomics beyond
hipError_t embbag_bwd(const float* dy, const int64_t* idx, const int64_t* off, int B, long L, int D, float* dw,
                      long rows, hipStream_t s);



}  // namespace pde
