// Device helpers shared by the HIP translation units (pm_kernels.hip,
// pm_lines.hip).  Header-only: every function is forceinline.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "pm_internal.hpp"

namespace pm {

static constexpr int kWave = 64;
static constexpr int kBlock = 256;
static constexpr int kWpb = kBlock / kWave;
static constexpr uint32_t kNone = 0xFFFFFFFFu;
static constexpr unsigned kMaxGrid = 1024;  // persistent-style grids: 4 blocks per CU
static constexpr int kU = 8;                // K2 strip unroll: independent loads in flight per lane

struct PopcOp {
  __host__ __device__ uint64_t operator()(unsigned long long m) const {
    return static_cast<uint64_t>(__builtin_popcountll(m));
  }
};

// u32 -> u64 scan input (64-bit accumulation of 32-bit counts)
struct Widen {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return static_cast<uint64_t>(x); }
};

// ---------------------------------------------------------------------------
// helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Template adjacency is read from an LDS copy (s_adj): a kernel-argument
// array indexed at run time compiles to a scalar memory load per access.
__device__ __forceinline__ void load_adj(uint16_t* s_adj, const PatArgs& pa) {
  if (threadIdx.x < 16) s_adj[threadIdx.x] = pa.adj[threadIdx.x];
}

__device__ __forceinline__ uint16_t nbr_mask(uint16_t T, const uint16_t* adj) {
  uint16_t m = 0;
  while (T) {
    const int t = __ffs(static_cast<int>(T)) - 1;
    m |= adj[t];
    T &= static_cast<uint16_t>(T - 1);
  }
  return m;
}

// global verify_and_update_vertex_state bit test (nonunique_ee.hpp:901-939):
// keep bit t iff adj[t] != 0 and adj[t] is a subset of TN.
__device__ __forceinline__ uint16_t keep_bits(uint16_t T, uint16_t TN, const uint16_t* adj) {
  uint16_t out = T, x = T;
  while (x) {
    const int t = __ffs(static_cast<int>(x)) - 1;
    x &= static_cast<uint16_t>(x - 1);
    const uint16_t a = adj[t];
    if (a == 0 || (a & static_cast<uint16_t>(~TN))) out &= static_cast<uint16_t>(~(1u << t));
  }
  return out;
}

// Owner rank of the vertex at position p.
__device__ __forceinline__ uint32_t owner_of(uint64_t p, const OwnerArgs& oa) {
  if (oa.nranks <= 1) return 0;
  const uint64_t v = oa.perm[p];
  if (oa.nhubs) {
    uint32_t lo = 0, hi = oa.nhubs;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (oa.hubs[mid] < v) lo = mid + 1; else hi = mid;
    }
    if (lo < oa.nhubs && oa.hubs[lo] == v) return lo % oa.nranks;
  }
  return static_cast<uint32_t>(v % oa.nranks);
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) x += __shfl_xor(x, d, kWave);
  return x;
}

// Per-block counters: each block sums its waves in LDS, then adds its
// nonzero totals to the counter slot with one atomic per word (a few thousand
// same-address atomics per launch at most; per-wave atomics would serialise
// at one L2 channel).  Layout of the W = 2P + 4 words: [vertices per rank |
// edges per rank | traversed | matching rows | removed flag | asymmetry flag];
// the slot is zeroed before the launch.
static constexpr int kMaxRanks = 64;
struct BlockAcc {
  uint64_t trav = 0, match = 0, vs = 0, es = 0;
  uint32_t removed = 0, asym = 0;
};

__device__ __forceinline__ void acc_owner(unsigned long long* s_hist, const OwnerArgs& oa, uint64_t v,
                                          uint64_t edges) {
  const uint32_t r = owner_of(v, oa);
  atomicAdd(&s_hist[r], 1ull);
  atomicAdd(&s_hist[oa.nranks + r], static_cast<unsigned long long>(edges));
}

struct Partials {
  unsigned long long* part;  // unused (kept for the launch signatures)
  unsigned long long* slot;
};

// All threads of the block must call this (after their loops).
__device__ __forceinline__ void flush_block(BlockAcc a, const OwnerArgs& oa, unsigned long long* s_hist,
                                            unsigned long long* s_red, const Partials& pp) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t v[6] = {wave_sum(a.trav), wave_sum(a.match), wave_sum(a.vs), wave_sum(a.es),
                         wave_sum(a.removed), wave_sum(a.asym)};
  if (lane == 0)
    for (int i = 0; i < 6; ++i) s_red[w * 6 + i] = v[i];
  __syncthreads();
  const uint32_t P = oa.nranks <= 1 ? 1 : oa.nranks;
  unsigned long long* out = pp.slot;
  if (threadIdx.x < 6) {
    unsigned long long t = 0;
    for (int i = 0; i < kWpb; ++i) t += s_red[i * 6 + threadIdx.x];
    const int j = threadIdx.x;
    int dst = -1;
    if (j == 0) dst = 2 * P;
    if (j == 1) dst = 2 * P + 1;
    if (j == 4) dst = 2 * P + 2;
    if (j == 5) dst = 2 * P + 3;
    if (oa.nranks <= 1) {
      if (j == 2) dst = 0;
      if (j == 3) dst = 1;
    }
    if (dst >= 0 && t) atomicAdd(out + dst, t);
  }
  if (oa.nranks > 1)
    for (uint32_t i = threadIdx.x; i < 2 * P; i += blockDim.x)
      if (s_hist[i]) atomicAdd(out + i, s_hist[i]);
}

// Wave-aggregated reservation of n slots on a global counter; returns the
// lane's first slot.  All lanes of the wave must call it.
__device__ __forceinline__ uint64_t wave_reserve(unsigned long long* ctr, uint32_t n) {
  const uint64_t incl = wave_incl_scan(n);
  const uint64_t total = __shfl(incl, kWave - 1, kWave);
  unsigned long long base = 0;
  if (lane_id() == 0 && total) base = atomicAdd(ctr, static_cast<unsigned long long>(total));
  base = __shfl(base, 0, kWave);
  return base + incl - n;
}

// The same on a 32-bit counter.
__device__ __forceinline__ uint32_t wave_reserve32(uint32_t* ctr, uint32_t n) {
  const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(n));
  const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
  uint32_t base = 0;
  if (lane_id() == 0 && total) base = atomicAdd(ctr, total);
  base = static_cast<uint32_t>(__shfl(static_cast<int>(base), 0, kWave));
  return base + incl - n;
}

// Block-aggregated global add: one atomic per block (all threads must call).
__device__ __forceinline__ void block_atomic_add(unsigned long long* dst, uint64_t v) {
  __shared__ unsigned long long s_b[kWpb];
  v = wave_sum(v);
  if (lane_id() == 0) s_b[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < kWpb; ++i) t += s_b[i];
    if (t) atomicAdd(dst, t);
  }
  __syncthreads();
}


__device__ __forceinline__ bool pos_ok(uint16_t T, int k, const LineArgs& la) {
  return la.lok[k] && ((T >> la.I[k]) & 1u);
}

// Walk storage: stride = C+2 u32 per walk, position p at w[i*stride + p].
__device__ __forceinline__ bool enum_ok(const uint32_t* w, int pos, uint32_t v, const LineArgs& la) {
  // tds_batch_1.hpp:284-302 / :622-639 / :821-839 / :864-882
  const uint16_t E = la.E[pos];
  if (E == pos) {
    for (int i = 0; i < pos; ++i)
      if (w[i] == v) return false;
    return true;
  }
  if (E < pos) return w[E] == v;
  return false;
}


}  // namespace pm
