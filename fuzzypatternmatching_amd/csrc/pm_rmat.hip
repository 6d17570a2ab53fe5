// GPU R-MAT generator and CSR builder.
//
// Bit-identical to the reference's generate_rmat stream (and to the host
// restatement host/rmat.hpp): generator rank r draws every edge from ONE
// boost::mt19937 (seed 5489 + 3r, src/generate_rmat.cpp:202-205), 5*S draws
// per edge (rmat_edge_generator.hpp:218-246), hash_nbits scramble (detail/
// hash.hpp:115-145) and emits (u,v) then (v,u) (rmat_edge_generator.hpp:127-139).
//
// MI355X design:
//   1. each rank's stream is cut into K substreams of esub edges (5*S*esub
//      draws); their start windows come from a jump tree: level L jumps the
//      2^L known windows by (K / 2^(L+1)) * 5*S*esub draws at once, applying
//      the GF(2) polynomial x^J mod phi computed on the host (host/mt_jump.hpp).
//      k_mt_jump: one block per jump, the 20560-word stretch of the sequence in
//      LDS, 624 lanes each XOR-ing the words the polynomial selects.
//   2. k_rmat_gen: one block per substream.  The MT19937 twist runs on the
//      block (three 227-wide phases into a second buffer, tempered draws
//      appended to an LDS ring); each round 128 lanes turn 128 * 5*S draws into
//      128 edges with the reference's double arithmetic (IEEE, no contraction:
//      the library is built with -ffp-contract=off) and store the two directed
//      64-bit keys (src << S | dst).
//   3. rocPRIM radix sort of the keys on 2*S bits, then k_csr_from_keys writes
//      the row offsets (one pass, no atomics) and the sorted columns: the
//      row-sorted CSR with multiplicity the device layout expects.
// The result is deterministic (no atomics anywhere) and independent of K.

#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "host/mt_jump.hpp"
#include "host/rmat.hpp"
#include "pm_internal.hpp"
#include "pm_rmat.hpp"

namespace pm {

namespace {

constexpr int kMtN = mtj::kN;          // 624
constexpr int kMtShift = kMtN - mtj::kM;  // 227
constexpr int kSeqLen = mtj::kDeg + kMtN - 1;  // x_k .. x_{k+19936+623}
constexpr int kJumpThreads = 640;
constexpr int kGenThreads = 256;
constexpr int kEdgesPerRound = 128;

__device__ __forceinline__ uint32_t mt_twist(uint32_t a, uint32_t b) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// hash.hpp:65-145 (same arithmetic as host/rmat.hpp)
__device__ __forceinline__ uint32_t d_hash32(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}

__device__ __forceinline__ uint32_t d_hash16(uint32_t a) {  // 16-bit arithmetic, truncated after each step
  a = ((a + 0x5d16u) + (a << 6)) & 0xFFFFu;
  a = ((a ^ 0xc23cu) ^ (a >> 9)) & 0xFFFFu;
  a = ((a + 0x67b1u) + (a << 5)) & 0xFFFFu;
  a = ((a + 0x646cu) ^ (a << 7)) & 0xFFFFu;
  a = ((a + 0x46c5u) + (a << 3)) & 0xFFFFu;
  a = ((a ^ 0x4f09u) ^ (a >> 8)) & 0xFFFFu;
  return a;
}

__device__ __forceinline__ uint64_t d_hash_nbits(uint64_t x, int n) {
  if (n == 32) return d_hash32(static_cast<uint32_t>(x));
  if (n > 32) {
    n -= 32;
    for (int i = 0; i <= n; ++i) {
      const uint64_t t = d_hash32(static_cast<uint32_t>((x >> i) & 0xFFFFFFFFull));
      x = (x & ~(0xFFFFFFFFull << i)) | (t << i);
    }
    for (int i = n; i >= 0; --i) {
      const uint64_t t = d_hash32(static_cast<uint32_t>((x >> i) & 0xFFFFFFFFull));
      x = (x & ~(0xFFFFFFFFull << i)) | (t << i);
    }
    return x;
  }
  n -= 16;
  for (int i = 0; i <= n; ++i) {
    const uint64_t t = d_hash16(static_cast<uint32_t>((x >> i) & 0xFFFFull));
    x = (x & ~(0xFFFFull << i)) | (t << i);
  }
  for (int i = n; i >= 0; --i) {
    const uint64_t t = d_hash16(static_cast<uint32_t>((x >> i) & 0xFFFFull));
    x = (x & ~(0xFFFFull << i)) | (t << i);
  }
  return x;
}

// One jump per block: win[dst] = p(T) win[src], p = x^J mod phi (bits 0..19936).
// Block b of the launch: rank group b / nsrc, source ordinal b % nsrc; the
// source window sits at (group * K + ordinal * stride) and the destination
// stride / 2 windows further.
__global__ __launch_bounds__(kJumpThreads) void k_mt_jump(uint32_t* __restrict__ win, uint32_t K, uint32_t nsrc,
                                                          uint32_t stride, const uint64_t* __restrict__ poly) {
  __shared__ uint32_t seq[kSeqLen];
  const uint32_t g = blockIdx.x / nsrc, o = blockIdx.x % nsrc;
  const uint64_t src = uint64_t(g) * K + uint64_t(o) * stride, dst = src + stride / 2;
  const uint32_t* w = win + src * kMtN;
  for (int i = threadIdx.x; i < kMtN; i += blockDim.x) seq[i] = w[i];
  __syncthreads();
  // x_t = x_{t-227} ^ twist(x_{t-624}, x_{t-623}): 227 independent words per phase
  for (int t0 = kMtN; t0 < kSeqLen; t0 += kMtShift) {
    const int t = t0 + static_cast<int>(threadIdx.x);
    if (threadIdx.x < static_cast<unsigned>(kMtShift) && t < kSeqLen)
      seq[t] = seq[t - kMtShift] ^ mt_twist(seq[t - kMtN], seq[t - kMtN + 1]);
    __syncthreads();
  }
  if (threadIdx.x < static_cast<unsigned>(kMtN)) {
    const int j = threadIdx.x;
    uint32_t acc = 0;
    for (int wi = 0; wi < mtj::kWords; ++wi) {
      uint64_t bits = poly[wi];  // wave-uniform (scalar loads)
      while (bits) {
        const int b = __ffsll(static_cast<long long>(bits)) - 1;
        bits &= bits - 1;
        acc ^= seq[wi * 64 + b + j];
      }
    }
    win[dst * kMtN + j] = acc;
  }
}

// One substream per block.  ring: tempered draws not consumed yet.
__global__ __launch_bounds__(kGenThreads) void k_rmat_gen(const uint32_t* __restrict__ win, uint32_t K,
                                                          uint64_t per_rank, uint64_t esub, int S, uint32_t ring_cap,
                                                          uint64_t* __restrict__ keys) {
  extern __shared__ uint32_t smem[];
  uint32_t* ma = smem;
  uint32_t* mb = smem + kMtN;
  uint32_t* ring = smem + 2 * kMtN;
  const uint32_t g = blockIdx.x / K, sub = blockIdx.x % K;
  const uint64_t e0 = uint64_t(sub) * esub;
  if (e0 >= per_rank) return;
  const uint64_t ne = min(esub, per_rank - e0);
  const uint32_t tid = threadIdx.x;
  for (int i = tid; i < kMtN; i += blockDim.x) ma[i] = win[uint64_t(blockIdx.x) * kMtN + i];
  __syncthreads();
  const uint32_t dpe = 5u * static_cast<uint32_t>(S);  // draws per edge
  uint32_t head = 0, tail = 0, avail = 0;              // ring positions (mod ring_cap)
  uint64_t* out = keys + 2 * (uint64_t(g) * per_rank + e0);
  const uint64_t mask = (S >= 64) ? ~0ull : ((1ull << S) - 1);
  for (uint64_t e = 0; e < ne; e += kEdgesPerRound) {
    const uint32_t n = static_cast<uint32_t>(min<uint64_t>(kEdgesPerRound, ne - e));
    const uint32_t need = n * dpe;
    while (avail < need) {  // block-uniform
      // std::mt19937 twist of ma into mb, each new word tempered into the ring
      auto put = [&](uint32_t t, uint32_t x) {
        mb[t] = x;
        uint32_t r = tail + t;
        if (r >= ring_cap) r -= ring_cap;
        ring[r] = mt_temper(x);
      };
      if (tid < static_cast<uint32_t>(kMtShift)) put(tid, ma[tid + mtj::kM] ^ mt_twist(ma[tid], ma[tid + 1]));
      __syncthreads();
      if (tid < static_cast<uint32_t>(kMtShift)) {
        const uint32_t t = kMtShift + tid;
        put(t, mb[t - kMtShift] ^ mt_twist(ma[t], ma[t + 1]));
      }
      __syncthreads();
      if (tid < static_cast<uint32_t>(kMtN - 2 * kMtShift)) {
        const uint32_t t = 2 * kMtShift + tid;
        put(t, mb[t - kMtShift] ^ mt_twist(ma[t], t + 1 < static_cast<uint32_t>(kMtN) ? ma[t + 1] : mb[0]));
      }
      __syncthreads();
      uint32_t* sw = ma;
      ma = mb;
      mb = sw;
      tail += kMtN;
      if (tail >= ring_cap) tail -= ring_cap;
      avail += kMtN;
    }
    if (tid < n) {
      uint32_t r = head + tid * dpe;
      if (r >= ring_cap) r -= ring_cap;
      auto u01 = [&]() {
        const double x = static_cast<double>(ring[r]) * (1.0 / 4294967296.0);
        if (++r == ring_cap) r = 0;
        return x;
      };
      // rmat_edge_generator.hpp:218-261, statement for statement
      double ra = 0.57, rb = 0.19, rc = 0.19, rd = 0.05;
      uint64_t u = 0, v = 0;
      uint64_t step = (uint64_t(1) << S) / 2;
      for (int j = 0; j < S; ++j) {
        const double p = u01();
        if (p < ra) {
        } else if (p >= ra && p < ra + rb) {
          v += step;
        } else if (p >= ra + rb && p < ra + rb + rc) {
          u += step;
        } else {
          u += step;
          v += step;
        }
        step /= 2;
        ra *= 0.9 + 0.2 * u01();
        rb *= 0.9 + 0.2 * u01();
        rc *= 0.9 + 0.2 * u01();
        rd *= 0.9 + 0.2 * u01();
        const double s = ra + rb + rc + rd;
        ra /= s;
        rb /= s;
        rc /= s;
        rd = 1. - ra - rb - rc;
      }
      u = d_hash_nbits(u, S) & mask;
      v = d_hash_nbits(v, S) & mask;
      out[2 * (e + tid)] = (u << S) | v;
      out[2 * (e + tid) + 1] = (v << S) | u;
    }
    head += need;
    while (head >= ring_cap) head -= ring_cap;
    avail -= need;
    __syncthreads();  // the next twists overwrite consumed ring words
  }
}

// Sorted keys -> row offsets (n + 1) and columns.  Entry i starts the rows
// prev_src + 1 .. src (empty rows in between); the last entry closes the rest.
__global__ void k_csr_from_keys(const uint64_t* __restrict__ keys, uint64_t nkeys, int S, uint64_t n,
                                uint64_t* __restrict__ off, uint32_t* __restrict__ col) {
  const uint64_t mask = (1ull << S) - 1;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nkeys; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = keys[i];
    const uint64_t s = k >> S;
    col[i] = static_cast<uint32_t>(k & mask);
    const uint64_t first = i ? (keys[i - 1] >> S) + 1 : 0;
    for (uint64_t w = first; w <= s; ++w) off[w] = i;
    if (i == nkeys - 1)
      for (uint64_t w = s + 1; w <= n; ++w) off[w] = nkeys;
  }
}

__global__ void k_fill_u64(uint64_t* p, uint64_t n, uint64_t x) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) p[i] = x;
}

unsigned grid_of(uint64_t items, unsigned per, unsigned cap) {
  uint64_t g = (items + per - 1) / per;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, cap)));
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* alloc(uint64_t n) {
    PM_HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(n, 1) * sizeof(T)));
    return static_cast<T*>(p);
  }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
  }
};

// Sharded build: out-degree of every source (the keys hold both directions of every pair).
__global__ void k_key_degrees(const uint64_t* __restrict__ keys, uint64_t n, int S, uint32_t* __restrict__ deg) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    atomicAdd(&deg[keys[i] >> S], 1u);
}

// Owner of a directed entry (delegate_partitioned_graph.ipp:818-969 low-degree rows by source,
// :1402-1648 delegate rows by target).
__device__ __forceinline__ uint32_t entry_owner(uint64_t key, int S, const uint32_t* deg, uint64_t thr, uint32_t G) {
  const uint64_t u = key >> S, v = key & ((1ull << S) - 1);
  return static_cast<uint32_t>((deg[u] >= thr ? v : u) % G);
}

__global__ void k_owner_count(const uint64_t* __restrict__ keys, uint64_t n, int S, const uint32_t* __restrict__ deg,
                              uint64_t thr, uint32_t G, unsigned long long* __restrict__ cnt) {
  __shared__ unsigned long long s_cnt[64];
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) s_cnt[g] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    atomicAdd(&s_cnt[entry_owner(keys[i], S, deg, thr, G)], 1ull);
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
    if (s_cnt[g]) atomicAdd(&cnt[g], s_cnt[g]);
}

// Entries into their owner's block (order inside a block is free: the receiver sorts).
__global__ void k_owner_scatter(const uint64_t* __restrict__ keys, uint64_t n, int S, const uint32_t* __restrict__ deg,
                                uint64_t thr, uint32_t G, unsigned long long* __restrict__ cursor,
                                uint64_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t k = keys[i];
    out[atomicAdd(&cursor[entry_owner(k, S, deg, thr, G)], 1ull)] = k;
  }
}

}  // namespace

RmatPlan rmat_plan(uint64_t scale, uint64_t p_gen) {
  if (scale < 1 || scale > 31) throw std::runtime_error("GPU R-MAT: scale must be in 1..31 (u32 ids, 2*S key bits)");
  if (p_gen == 0) throw std::runtime_error("P_gen must be positive");
  RmatPlan p;
  p.scale = scale;
  p.per_rank = rmat_edges_per_rank(scale, p_gen);
  // substreams per rank: at least 2048 edges each, at most 1024 of them
  uint32_t K = 1;
  while (K < 1024 && p.per_rank / (2ull * K) >= 2048) K *= 2;
  p.K = K;
  p.esub = (p.per_rank + K - 1) / K;
  p.levels = 0;
  while ((1u << p.levels) < K) ++p.levels;
  return p;
}

// Keys (src << S | dst) of the generator ranks vranks, 2 * per_rank each, in
// rank order (same order as host rmat_stream_of).
void rmat_keys_device(const RmatPlan& p, const std::vector<uint64_t>& vranks, uint64_t* d_keys, hipStream_t stream) {
  const uint32_t R = static_cast<uint32_t>(vranks.size());
  if (!R || !p.per_rank) return;
  const uint64_t nwin = uint64_t(R) * p.K;
  std::vector<uint32_t> w0(nwin * kMtN, 0);
  for (uint32_t g = 0; g < R; ++g) mtj::seed_window(static_cast<uint32_t>(rmat_seed(vranks[g])), w0.data() + uint64_t(g) * p.K * kMtN);
  DevBuf bw, bp;
  uint32_t* d_win = bw.alloc<uint32_t>(nwin * kMtN);
  PM_HIP_CHECK(hipMemcpyAsync(d_win, w0.data(), w0.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
  if (p.levels) {
    // q_m = x^(2^m * J) mod phi, J = draws of one substream
    const uint64_t J = 5ull * p.scale * p.esub;
    std::vector<mtj::Poly> q(p.levels);
    q[0] = mtj::jump_poly(J);
    for (uint32_t m = 1; m < p.levels; ++m) q[m] = mtj::square_mod(q[m - 1]);
    uint64_t* d_poly = bp.alloc<uint64_t>(uint64_t(p.levels) * mtj::kWords);
    for (uint32_t m = 0; m < p.levels; ++m)
      PM_HIP_CHECK(hipMemcpyAsync(d_poly + uint64_t(m) * mtj::kWords, q[m].data(), mtj::kWords * sizeof(uint64_t),
                                  hipMemcpyHostToDevice, stream));
    for (uint32_t L = 0; L < p.levels; ++L) {
      const uint32_t nsrc = 1u << L, stride = p.K >> L;
      hipLaunchKernelGGL(k_mt_jump, dim3(R * nsrc), dim3(kJumpThreads), 0, stream, d_win, p.K, nsrc, stride,
                         d_poly + uint64_t(p.levels - 1 - L) * mtj::kWords);
      PM_HIP_CHECK(hipGetLastError());
    }
    PM_HIP_CHECK(hipStreamSynchronize(stream));  // host polynomials go out of scope
  }
  const uint32_t ring = kEdgesPerRound * 5u * static_cast<uint32_t>(p.scale) + kMtN;
  const size_t lds = (2 * kMtN + ring) * sizeof(uint32_t);
  hipLaunchKernelGGL(k_rmat_gen, dim3(static_cast<unsigned>(nwin)), dim3(kGenThreads), lds, stream, d_win, p.K,
                     p.per_rank, p.esub, static_cast<int>(p.scale), ring, d_keys);
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(stream));
}

// Sorted keys (2 * scale bits) -> device CSR of n = 2^scale rows; frees the key buffers.
static DevCsr csr_from_unsorted(uint64_t scale, DevBuf& ka, DevBuf& kb, uint64_t nkeys, hipStream_t stream) {
  DevCsr g;
  g.n = uint64_t(1) << scale;
  g.nnz = nkeys;
  uint64_t* a = static_cast<uint64_t*>(ka.p);
  uint64_t* b = static_cast<uint64_t*>(kb.p);
  DevBuf tmp;
  rocprim::double_buffer<uint64_t> db(a, b);
  size_t tb = 0;
  PM_HIP_CHECK(rocprim::radix_sort_keys(nullptr, tb, db, nkeys, 0u, static_cast<unsigned>(2 * scale), stream));
  void* d_tmp = tmp.alloc<char>(tb);
  PM_HIP_CHECK(rocprim::radix_sort_keys(d_tmp, tb, db, nkeys, 0u, static_cast<unsigned>(2 * scale), stream));
  PM_HIP_CHECK(hipStreamSynchronize(stream));
  tmp.reset();
  const uint64_t* sorted = db.current();
  if (sorted == a) kb.reset(); else ka.reset();
  PM_HIP_CHECK(hipMalloc(&g.d_off, (g.n + 1) * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMalloc(&g.d_col, std::max<uint64_t>(nkeys, 1) * sizeof(uint32_t)));
  if (nkeys) {
    hipLaunchKernelGGL(k_csr_from_keys, dim3(grid_of(nkeys, 256, 1u << 20)), dim3(256), 0, stream, sorted, nkeys,
                       static_cast<int>(scale), g.n, g.d_off, g.d_col);
  } else {
    hipLaunchKernelGGL(k_fill_u64, dim3(grid_of(g.n + 1, 256, 8192)), dim3(256), 0, stream, g.d_off, g.n + 1, 0ull);
  }
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(stream));
  ka.reset();
  kb.reset();
  return g;
}

DevCsr rmat_shard_device(uint64_t scale, uint64_t p_gen, uint64_t hub_threshold, Comm& comm, uint32_t nshards,
                         uint32_t shard, std::vector<uint32_t>& gdeg, hipStream_t stream) {
  if (nshards == 0 || nshards > 64 || shard >= nshards) throw std::runtime_error("rmat shard: 1..64 shards");
  const RmatPlan p = rmat_plan(scale, p_gen);
  std::vector<uint64_t> mine;
  for (uint64_t r = shard; r < p_gen; r += nshards) mine.push_back(r);
  const uint64_t nkeys = 2 * p.per_rank * mine.size();
  const uint64_t n = uint64_t(1) << scale;
  const int S = static_cast<int>(scale);
  DevBuf ka, kb, bdeg, bcnt;
  uint64_t* a = ka.alloc<uint64_t>(nkeys);
  rmat_keys_device(p, mine, a, stream);
  // global degrees (delegates are decided on them): a histogram of the sources, summed over the shards
  uint32_t* deg = bdeg.alloc<uint32_t>(n);
  PM_HIP_CHECK(hipMemsetAsync(deg, 0, n * sizeof(uint32_t), stream));
  if (nkeys)
    hipLaunchKernelGGL(k_key_degrees, dim3(grid_of(nkeys, 256, 1u << 16)), dim3(256), 0, stream, a, nkeys, S, deg);
  comm.allreduce_sum_u32(deg, n, stream);
  gdeg.resize(n);
  PM_HIP_CHECK(hipMemcpyAsync(gdeg.data(), deg, n * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  PM_HIP_CHECK(hipStreamSynchronize(stream));
  uint64_t nrecv = nkeys;
  if (nshards > 1) {
    // owners' blocks: counts, the G x G count matrix, then one all-to-all of the 8-B entries
    const uint32_t G = nshards;
    auto* cnt = bcnt.alloc<unsigned long long>(2 * G + uint64_t(G) * G);
    PM_HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * G * sizeof(unsigned long long), stream));
    if (nkeys)
      hipLaunchKernelGGL(k_owner_count, dim3(grid_of(nkeys, 256, 4096)), dim3(256), 0, stream, a, nkeys, S, deg,
                         hub_threshold, G, cnt);
    comm.allgather(cnt, cnt + 2 * G, G * sizeof(uint64_t), stream);
    std::vector<uint64_t> m(uint64_t(G) * G);
    PM_HIP_CHECK(hipMemcpyAsync(m.data(), cnt + 2 * G, m.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
    PM_HIP_CHECK(hipStreamSynchronize(stream));
    std::vector<uint64_t> sb(G), rb(G), cur(G, 0);
    nrecv = 0;
    for (uint32_t g = 0; g < G; ++g) {
      sb[g] = m[uint64_t(shard) * G + g] * sizeof(uint64_t);
      rb[g] = m[uint64_t(g) * G + shard] * sizeof(uint64_t);
      nrecv += m[uint64_t(g) * G + shard];
      if (g) cur[g] = cur[g - 1] + m[uint64_t(shard) * G + g - 1];
    }
    uint64_t* send = kb.alloc<uint64_t>(nkeys);
    PM_HIP_CHECK(hipMemcpyAsync(cnt + G, cur.data(), G * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
    if (nkeys)
      hipLaunchKernelGGL(k_owner_scatter, dim3(grid_of(nkeys, 256, 1u << 16)), dim3(256), 0, stream, a, nkeys, S,
                         deg, hub_threshold, G, cnt + G, send);
    PM_HIP_CHECK(hipGetLastError());
    PM_HIP_CHECK(hipStreamSynchronize(stream));
    ka.reset();
    uint64_t* recv = ka.alloc<uint64_t>(nrecv);
    comm.alltoallv(send, sb.data(), recv, rb.data(), stream);
    PM_HIP_CHECK(hipStreamSynchronize(stream));
    kb.reset();
  }
  bdeg.reset();
  kb.alloc<uint64_t>(nrecv);  // the sort's second buffer
  return csr_from_unsorted(scale, ka, kb, nrecv, stream);
}

DevCsr rmat_csr_device(uint64_t scale, uint64_t p_gen, hipStream_t stream) {
  const RmatPlan p = rmat_plan(scale, p_gen);
  std::vector<uint64_t> all(p_gen);
  for (uint64_t r = 0; r < p_gen; ++r) all[r] = r;
  const uint64_t nkeys = 2 * p.per_rank * p_gen;
  DevCsr g;
  g.n = uint64_t(1) << scale;
  g.nnz = nkeys;
  DevBuf ka, kb, tmp;
  uint64_t* a = ka.alloc<uint64_t>(nkeys);
  rmat_keys_device(p, all, a, stream);
  uint64_t* b = kb.alloc<uint64_t>(nkeys);
  rocprim::double_buffer<uint64_t> db(a, b);
  size_t tb = 0;
  PM_HIP_CHECK(rocprim::radix_sort_keys(nullptr, tb, db, nkeys, 0u, static_cast<unsigned>(2 * scale), stream));
  void* d_tmp = tmp.alloc<char>(tb);
  PM_HIP_CHECK(rocprim::radix_sort_keys(d_tmp, tb, db, nkeys, 0u, static_cast<unsigned>(2 * scale), stream));
  PM_HIP_CHECK(hipStreamSynchronize(stream));
  tmp.reset();
  const uint64_t* sorted = db.current();
  // free the other buffer before the CSR arrays are allocated
  if (sorted == a) kb.reset(); else ka.reset();
  PM_HIP_CHECK(hipMalloc(&g.d_off, (g.n + 1) * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMalloc(&g.d_col, std::max<uint64_t>(nkeys, 1) * sizeof(uint32_t)));
  if (nkeys) {
    hipLaunchKernelGGL(k_csr_from_keys, dim3(grid_of(nkeys, 256, 1u << 20)), dim3(256), 0, stream, sorted, nkeys,
                       static_cast<int>(scale), g.n, g.d_off, g.d_col);
  } else {
    hipLaunchKernelGGL(k_fill_u64, dim3(grid_of(g.n + 1, 256, 8192)), dim3(256), 0, stream, g.d_off, g.n + 1, 0ull);
  }
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(stream));
  return g;
}

}  // namespace pm
