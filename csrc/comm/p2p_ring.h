// Stage-to-stage point-to-point channel over xGMI: a receive ring in the receiver's HBM that the sender
// writes directly (the reference moves every activation through
// rpc/model_parallel_ResNet50.py:173-174's RRef.to_here() as a CPU tensor).
//
// One P2PRing object per (rank, peer) pair, on both sides.  Each rank exports ONE uncached allocation
// (hipExtMallocWithFlags(hipDeviceMallocUncached), IPC handle through the c10d store):
//
//   [ctrl 4 KB: word 0 = ACK, written by the peer's receiver for MY sends]
//   [flags: kSlots x kMaxWg words, written by the peer's sender for MY receives]
//   [kSlots ring slots of slot_bytes, written by the peer's sender]
//
// send(src, bytes) -- one kernel, `g` workgroups (g from the byte count, the same formula on both sides):
//   message number seq = my device send counter, slot = seq % kSlots; wait (bounded) until the peer's ACK
//   shows message seq - kSlots consumed; every workgroup copies its chunk of src straight into the peer's
//   slot over xGMI, drains, releases at system scope and raises flag[slot][wg] = seq + 1 in the peer's
//   memory; the last workgroup to finish advances the send counter.
// recv(dst, bytes) -- one kernel, same grid: message seq = my receive counter; workgroup wg waits for
//   flag[slot][wg] == seq + 1 in MY memory, acquires, copies its chunk from my slot to dst; the last
//   workgroup advances the counter and writes ACK = seq + 1 into the PEER's ctrl word.
//
// Both kernels are stream-ordered and keep all state on the device, so a pipeline step that sends and
// receives records into a hipGraph and every replay moves the next messages.  Spins are bounded by
// s_memrealtime; a timeout sets the error word (error()) and the kernel drains -- never a hung grid.
// Two processes sharing ONE GPU map each other's rings exactly like two GPUs of a node (the rehearsal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace pde {

class P2PRing {
 public:
  static constexpr int kSlots = 4;     // messages in flight per direction
  static constexpr int kMaxWg = 128;   // workgroups per message (flag words per slot)

  P2PRing(int device, int64_t slot_bytes, double timeout_s);
  ~P2PRing();
  P2PRing(const P2PRing&) = delete;
  P2PRing& operator=(const P2PRing&) = delete;

  std::string ipc_handle() const;
  void open(const std::string& peer_handle);
  // loopback: the peer ring lives in THIS process on the same device (no IPC; single-process rehearsals)
  void open_local(P2PRing& peer);
  static int max_wg();  // workgroups a send / recv kernel may keep spinning (PDE_P2P_MAX_WG)
  // stream-ordered; 16-B aligned buffers; a message larger than a slot goes as slot-sized pieces
  void send(const void* src, int64_t bytes, hipStream_t s);
  void recv(void* dst, int64_t bytes, hipStream_t s);
  int error();  // 0, or 1 when a wait timed out (synchronises the device)
  void close();
  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t sent() const { return sent_; }          // ring messages (pieces) enqueued
  int64_t received() const { return received_; }

 private:
  int device_;
  int64_t slot_bytes_, flag_bytes_;
  uint64_t timeout_ticks_;
  char* local_ = nullptr;      // my exported allocation
  char* peer_ = nullptr;       // the peer's, mapped
  uint32_t* state_ = nullptr;  // device-local: send seq, recv seq, send done, recv done, error
  bool opened_ = false;
  bool peer_ipc_ = false;      // peer_ was mapped with hipIpcOpenMemHandle (else: a local ring's memory)
  int64_t sent_ = 0, received_ = 0;
};

}  // namespace pde
