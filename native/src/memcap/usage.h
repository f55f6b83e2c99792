// The daemon's side of the HBM-cap shim's accounting files: per-container HBM
// use of memory-unit grants, for /metrics.
//
// With --enforce-memory-units and --metrics-addr, Allocate() creates one file
// per grant under <plugin dir>/amdgpu-dp/usage/ -- the grant (bytes per
// device, in the container's HIP order) and its device IDs in the header of
// native/memcap/memcap_area.h -- and bind-mounts it into the container; the
// shim in the container counts what its processes hold into it. The metrics
// endpoint reads the headers back and matches them to pods through the
// kubelet's PodResources API (the file is named after the grant's device IDs,
// which PodResources lists per container). The reference counts memory units
// and never sees what a pod uses (server.go:99-111).
//
// The files are writable by the container: every read is bounded, follows no
// symlink, validates the header and treats the numbers as the container's
// claim.
#pragma once

#include <stdint.h>

#include <set>
#include <string>
#include <string_view>
#include <vector>

#include "common/status.h"

namespace adp::memcap {

// File name of a grant: FNV-1a of its device IDs, sorted and comma-joined.
std::string AllocationKey(std::vector<std::string_view> ids);
// The same for IDs already sorted.
std::string AllocationKeySorted(const std::vector<std::string_view>& sorted_ids);

// Creates <dir>/<key>.memcap for a grant of `cap_bytes` (one per device, in HIP
// order) to `ids` (comma-joined), atomically replacing any earlier file of the
// key (a new container gets fresh counters). Creates `dir` when missing.
Status CreateGrantFile(const std::string& dir, const std::string& key, const std::vector<uint64_t>& cap_bytes,
                       std::string_view ids_joined);

// CreateGrantFile on a background thread, so Allocate() -- on a gRPC loop --
// never waits for the filesystem (the container starts milliseconds later,
// after the kubelet has the response). Jobs run in order; a failure is logged
// once per process. Flush() waits (at most `timeout_ms`) until every job
// queued before it is done; false on timeout.
// With `wake` false the writer thread is not woken here but by the next
// WakeWriter() -- which the gRPC loops call after writing their responses, so
// the futex wake of a sleeping writer is off the Allocate() round trip -- or
// at the latest 20 ms later.
void CreateGrantFileAsync(std::string dir, std::string key, std::vector<uint64_t> cap_bytes, std::string ids_joined,
                          bool wake = true);
// Wakes the writer if a job is waiting for it; one atomic load otherwise.
void WakeWriter();
bool Flush(int timeout_ms = 5000);

struct Usage {
  std::string key;
  std::string ids;  // the IDs the file names, "" unless they hash to its key
  std::vector<uint64_t> used, cap, peak, refused;  // per HIP device of the container
  uint32_t processes = 0;                          // the container's processes holding a slot
  int64_t mtime_s = 0;
};

// One grant's file; NotFound if absent, InvalidArgument if not a valid file.
Result<Usage> ReadGrant(const std::string& dir, const std::string& key);

// Every grant file in `dir` (invalid ones skipped).
std::vector<Usage> ReadAll(const std::string& dir);

// Removes grant files whose key is not in `live` and that are older than
// `min_age_s` (a just-allocated container may not be listed by the kubelet
// yet); with `live` == nullptr (no PodResources) only keeps the newest
// `max_files`. Returns the number removed.
size_t Collect(const std::string& dir, const std::set<std::string>* live, int64_t min_age_s, size_t max_files);

}  // namespace adp::memcap
