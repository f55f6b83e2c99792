// xGMI/NUMA/partition-aware preferred allocation.
//
// Parity: the reference's best-effort policy
// (vendor/github.com/NVIDIA/go-gpuallocator/gpuallocator/besteffort_policy.go:34-89,
// pair scores :298-356). Its objective: among all ways to split the available
// GPUs into groups of the requested size, take the split with the highest total
// intra-group link score (so the GPUs left behind also group well), then return
// the best-scoring group of that split that holds every required GPU. It
// enumerates set partitions explicitly, which is fine for 8 GPUs and infeasible
// for the 64 compute partitions of an 8xMI355X node in CPX mode.
//
// MI355X-native design:
//  * Pair score between devices of different GPUs = PCIe/NUMA level (same NUMA
//    20, cross NUMA 10, as the reference's SameCPU/CrossCPU levels) + 100 per
//    direct xGMI hop (the NVLink analogue), minus 10 per xGMI link the GPU
//    reports down. On a healthy 8xMI355X mesh every pair is one xGMI hop, so
//    NUMA locality and link health are what separate candidates.
//  * Devices on the same physical GPU (compute partitions) score 1000: a
//    multi-partition request should stay on one die.
//  * Whole-GPU sets (<= 12 devices): exact search of the same objective with a
//    bitmask DP instead of explicit partition enumeration.
//  * Larger sets or partitions: hierarchical -- group by physical GPU, best-fit
//    the request onto the fewest GPUs (fragmentation), then grow by affinity.
//  * The graph is built once per snapshot; no SMI call happens on the RPC path.
#pragma once

#include <vector>

#include "inventory/inventory.h"

namespace adp::alloc {

struct DeviceRef {
  int gpu = 0;        // index into Snapshot::gpus
  int partition = -1; // index into PhysicalGpu::partitions, -1 = whole GPU
};

class DeviceGraph {
 public:
  DeviceGraph() = default;
  DeviceGraph(const inventory::Snapshot& snap, const std::vector<DeviceRef>& devices);
  // Explicit construction for tests.
  DeviceGraph(std::vector<int> parent, std::vector<int> scores);

  int size() const { return n_; }
  int parent(int i) const { return parent_[i]; }
  int Score(int a, int b) const { return score_[a * n_ + b]; }

 private:
  int n_ = 0;
  std::vector<int> parent_;
  std::vector<int> score_;
};

int PairScore(const inventory::Snapshot& snap, int gpu_a, int gpu_b);

// Preferred `size` devices out of `available` that include every `required`
// device. Returns sorted device indices, or empty when the request cannot be
// satisfied (same contract as the reference's Allocate).
std::vector<int> BestEffortAllocate(const DeviceGraph& g, const std::vector<int>& available,
                                    const std::vector<int>& required, int size);

}  // namespace adp::alloc
