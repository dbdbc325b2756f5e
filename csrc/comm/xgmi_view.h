// Plain-data view of an XgmiAllreduce's buffers (xgmi_allreduce.h), filled on the host and passed by value
// to kernels that fold the peer exchange into their own epilogue (device helpers: xgmi_device.h).
#pragma once

#include <cstdint>

namespace pde {

constexpr int kXgmiMaxRanks = 8;
// device-local state words (XgmiView::state)
constexpr int kXgmiStateEpoch = 0;  // epoch of the last completed call (one epoch per call, all workgroups)
constexpr int kXgmiStateDone = 1;   // workgroups of the running call that have finished
constexpr int kXgmiStateError = 2;  // 1 once a workgroup timed out waiting for a peer
constexpr int kXgmiStateWords = 4;
// host-mapped status words (XgmiView::host: pinned, coherent host memory both sides touch without a copy)
constexpr int kXgmiHostError = 0;  // 1 + epoch of the first timed-out wait (0: none); read by the host, no sync
constexpr int kXgmiHostAbort = 1;  // the host sets it (elastic round changed, engine failed): spins give up
constexpr int kXgmiHostWords = 16;

struct XgmiView {
  char* base[kXgmiMaxRanks];  // every rank's mapped [flags | slot0 | slot1] allocation (base[rank] = mine)
  uint32_t* state;            // kXgmiStateWords words, device-local
  uint32_t* host;             // kXgmiHostWords words, host-mapped (device pointer of pinned host memory)
  uint64_t timeout_ticks;     // s_memrealtime ticks (100 MHz) before a waiting workgroup gives up
  uint64_t read_delay_ticks;  // test hook (set_read_delay_us): stall before the peer reads
  int64_t flag_bytes, slot_bytes;
  int rank, size, blocks;     // a kernel using the view may run at most `blocks` workgroups
};

}  // namespace pde
