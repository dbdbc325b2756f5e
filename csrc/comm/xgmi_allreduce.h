// One-shot peer all-reduce over xGMI for latency-bound buckets.
//
// An MI355X node is a full mesh: every GPU reaches each of its 7 peers over a direct xGMI link.  For a
// small gradient bucket (the MNIST CNN's 87 KB, the hybrid fc's 544 B) a ring all-reduce is a chain of
// 2(N-1) latency-bound hops; here each rank instead
//   1. copies its bucket into its own IPC-exported, uncached staging slot,
//   2. raises one flag per (workgroup, rank) in EVERY peer's flag array (system-scope release),
//   3. waits for the N flags of its workgroup (one polling lane per peer, bounded spin),
//   4. reads the same chunk from all N slots over xGMI (7 links in parallel) and sums them in rank order.
// Every rank sums identical values in the same order, so the result is bit-identical on all ranks.
//
// Synchronisation is epoch based and needs no reset between calls: every call has ONE epoch, kept in
// device memory and advanced by the call's last finishing workgroup (so the kernel is hipGraph-capturable
// and replays advance it; calls of different sizes keep every workgroup on the same epoch), flags are
// written with the epoch value, staging alternates between two slots (a peer can be at most one call
// ahead: it cannot pass the next call's flag wait without this rank).  Spins are
// bounded by s_memrealtime; a timeout sets an error word and the workgroup drains (never a hung grid).
//
// Memory: one hipExtMallocWithFlags(hipDeviceMallocUncached) allocation per rank = [flags | slot0 | slot1],
// exported with hipIpcGetMemHandle; peers map it with hipIpcOpenMemHandle.  Uncached memory keeps the
// staged bytes and flags coherent between GPUs (and between processes sharing one GPU in rehearsals).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "xgmi_view.h"

namespace pde {

class XgmiAllreduce {
 public:
  XgmiAllreduce(int rank, int size, int device, int64_t max_bytes, int blocks, double timeout_s);
  ~XgmiAllreduce();
  XgmiAllreduce(const XgmiAllreduce&) = delete;
  XgmiAllreduce& operator=(const XgmiAllreduce&) = delete;

  std::string ipc_handle() const;                   // this rank's exported allocation
  void open(const std::vector<std::string>& handles);  // all ranks' handles, in rank order
  // dst[i] = scale * sum_r src_r[i]; fp32; src may alias dst; n * 4 <= max_bytes; stream-ordered.
  // wire_bf16: the exchanged copies are bf16 (cast fused into the staging; fp32 sum and output)
  void allreduce(const float* src, float* dst, int64_t n, float scale, hipStream_t s, bool wire_bf16 = false);
  // Two-shot form for bandwidth-bound buckets (reduce-scatter + all-gather through the same slots: each link
  // carries 2/N of the bucket instead of all of it); same contract as allreduce.  An instance runs either form
  // only (their flag values differ), and a kernel folding the exchange in (view()) uses a one-shot instance.
  void allreduce_twoshot(const float* src, float* dst, int64_t n, float scale, hipStream_t s, bool wire_bf16 = false);
  XgmiView view() const;  // device view for kernels that fold the exchange in (xgmi_device.h)
  // test hook: every workgroup of this rank stalls `us` microseconds between its flag wait and its peer reads
  void set_read_delay_us(double us) { read_delay_ticks_ = static_cast<uint64_t>(us * 100.0); }
  // 0, or 1 when some workgroup timed out waiting for a peer (or gave up on the host's abort word).
  // sync: wait for the device first (every queued call has run); otherwise a plain read of the host-mapped
  // status word -- cheap enough for a per-step check or a watchdog thread.
  int error(bool sync = true);
  // reset the error words after the host has handled a failure (synchronises the device: no call is in
  // flight while the device-side fail-fast word is cleared)
  void clear_error();
  // host-side abort: every current and later peer wait gives up within ~0.1 ms (its result is dropped and
  // the error word set) until reset_abort(); safe from any thread while kernels spin
  void abort();
  void reset_abort();
  bool aborted() const;
  void close();
  int rank() const { return rank_; }
  int size() const { return size_; }
  int64_t max_bytes() const { return max_bytes_; }
  int64_t calls() const { return calls_; }

 private:
  int rank_, size_, device_, blocks_;
  int64_t max_bytes_, slot_bytes_, flag_bytes_;
  uint64_t timeout_ticks_;
  uint64_t read_delay_ticks_ = 0;
  char* local_ = nullptr;       // my exported allocation
  uint32_t* state_ = nullptr;   // kXgmiStateWords: call epoch, done count, error word (device-local)
  uint32_t* host_ = nullptr;    // kXgmiHostWords, pinned host memory mapped into the device (status / abort)
  uint32_t* host_dev_ = nullptr;  // its device-side address
  std::vector<char*> peers_;    // mapped bases, peers_[rank_] == local_
  bool opened_ = false;
  int mode_ = 0;  // 0 unused, 1 one-shot, 2 two-shot
  int64_t calls_ = 0;
};

}  // namespace pde
