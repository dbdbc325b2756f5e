// Plain-data view of an XgmiAllreduce's buffers (xgmi_allreduce.h), filled on the host and passed by value
// to kernels that fold the peer exchange into their own epilogue (device helpers: xgmi_device.h).
#pragma once

#include <cstdint>

namespace pde {

constexpr int kXgmiMaxRanks = 8;

struct XgmiView {
  char* base[kXgmiMaxRanks];  // every rank's mapped [flags | slot0 | slot1] allocation (base[rank] = mine)
  uint32_t* state;            // [blocks] per-workgroup epochs + [1] error word, device-local
  uint64_t timeout_ticks;     // s_memrealtime ticks (100 MHz) before a waiting workgroup gives up
  int64_t flag_bytes, slot_bytes;
  int rank, size, blocks;     // a kernel using the view may run at most `blocks` workgroups
};

}  // namespace pde
