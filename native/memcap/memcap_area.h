// Layout of the HBM-cap shim's shared accounting file, shared by the shim
// (libadp_memcap.so, libc-only: this header needs nothing but <atomic> and
// <stdint.h>) and the daemon, which reads the header to report each
// container's HBM use (native/src/memcap/usage.h).
//
// One file per grant: every process of the container maps it, claims a slot
// and adds what it allocates to used[]. With --enforce-memory-units and
// --metrics-addr the daemon creates the file for each Allocate() (grant and
// device IDs filled in) under <plugin dir>/amdgpu-dp/usage/ and bind-mounts it
// into the container (ADP_MEMCAP_FILE); otherwise the shim creates one in the
// pod's /dev/shm.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <atomic>

namespace adp_memcap {

constexpr uint32_t kMagic = 0x434d4441;  // "ADMC"
constexpr uint32_t kVersion = 2;
constexpr int kMaxDevices = 64;
constexpr int kSlots = 256;
constexpr int kIdsBytes = 4096;

// The grant itself, daemon-owned and read-only in the container: one file per
// device of the grant, named by the device's HIP ordinal ("0", "1", ...), each
// holding the MiB granted on it ("36000\n"). The daemon bind-mounts them
// read-only from files it wrote before registering (<plugin dir>/amdgpu-dp/
// grants/<mib>.mib), so a pod can neither rewrite nor drop its grant; the
// AMD_GPU_MEMORY_LIMIT_MIB variable can only lower it.
constexpr const char* kGrantDir = "/run/amdgpu-dp/grant";

struct Slot {
  std::atomic<int32_t> pid;     // 0 free, > 0 owner, -1 being reclaimed
  std::atomic<uint64_t> start;  // owner's start time (/proc/<pid>/stat field 22): pid reuse guard
  std::atomic<uint64_t> bytes[kMaxDevices];
};

struct Area {
  std::atomic<uint32_t> magic;
  uint32_t version;
  uint32_t devices;  // entries of cap[] in the grant
  uint32_t ids_len;  // bytes of ids[]
  std::atomic<uint32_t> processes;  // slots held: processes of the container that use the shim
  uint32_t reserved;
  std::atomic<uint64_t> used[kMaxDevices];     // bytes held by the container, per HIP device
  std::atomic<uint64_t> cap[kMaxDevices];      // bytes granted (0 = not capped)
  std::atomic<uint64_t> peak[kMaxDevices];     // high-water mark of used[]
  std::atomic<uint64_t> refused[kMaxDevices];  // allocations refused at the cap
  char ids[kIdsBytes];                         // the grant's device IDs, comma-joined (daemon-written)
  Slot slots[kSlots];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared counters must be address-free");
static_assert(sizeof(std::atomic<uint64_t>) == 8 && sizeof(std::atomic<uint32_t>) == 4, "plain layout");

// What the daemon reads: everything before the slots.
constexpr size_t kHeaderBytes = offsetof(Area, slots);

}  // namespace adp_memcap
