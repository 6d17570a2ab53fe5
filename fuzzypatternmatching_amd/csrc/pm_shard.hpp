// Comm factories and the in-process shard group (pm_shard.hip).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <vector>

#include "../../include/pm_abi.h"
#include "pm_internal.hpp"

namespace pm {

// Shards of one search driven by threads of one process on one device.
struct ThreadGroup {
  explicit ThreadGroup(int n_) : n(n_), ptrs(n_, nullptr), hvec(n_, nullptr), counts(n_) {}
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<const void*> ptrs;
  std::vector<std::vector<uint64_t>*> hvec;
  std::vector<std::vector<uint64_t>> counts;  // alltoallv send sizes per shard
  std::mutex device;  // held by the shard that is computing (released inside collectives)
  void barrier();     // throws when another shard failed
  void abort();
};

Comm* make_rccl_comm(const void* unique_id, int nranks, int rank);
size_t rccl_unique_id(void* out, size_t len);
int rccl_selftest(int device, uint64_t bytes, int op);
Comm* make_thread_comm(ThreadGroup* g, int rank);
Comm* make_host_comm(const pm_host_comm& h);  // host-staged collectives of the caller (pm_abi.h)

}  // namespace pm
