// Sharded search: the exchanges between the shards of one
// pattern search and the two Comm implementations.
//
// The reference partitions vertices 1D-cyclically (owner = id % P,
// delegate_partitioned_graph.ipp:1679-1696) and moves every LCC/NLCC message
// through the MPI mailbox (new_mailbox.hpp:289-713); state sync of delegates
// uses MPI_Allreduce (impl/vertex_data.hpp:114-126).  Here shard q owns the
// rows of ids v % nshards == q and the per-superstep exchange is BSP:
//   * LCC: every row pulls its neighbours' T_pub, so after each superstep the
//     shards all-gather the T_pub of their slist entries (the only vertices
//     that can be in S) -- 2 B per entry, no per-edge messages;
//   * NLCC: walks are independent per source (the (vertex, source) dedup of
//     nem_1.hpp:131-139 and TDS walks never mix sources), so each shard runs
//     the walks of its own sources over an all-gathered copy of the alive M
//     rows of S (small after the first LCC call) and the replicated T_pub;
//   * counters and flags: one u64 sum all-reduce per LCC call / NLC line.
// Results are identical for every shard count.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "pm_device.hpp"
#include "pm_internal.hpp"
#include "pm_shard.hpp"

namespace pm {

#define PM_NCCL_CHECK(expr)                                                                          \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess)                                                                           \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " #expr); \
  } while (0)

// ---------------------------------------------------------------------------
// RCCL (one process per GPU, xGMI): stream-ordered, no host synchronisation.
class RcclComm : public Comm {
 public:
  RcclComm(const void* unique_id, int nranks, int rank) : nranks_(nranks) {
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    PM_NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
  }
  ~RcclComm() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  // One rank: a copy / nothing (one-rank RCCL collectives of large buffers
  // raise SIGFPE in this RCCL build; the communicator is still initialised).
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (nranks_ == 1) {
      if (bytes && send != recv) PM_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    PM_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }
  void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    if (nranks_ == 1) return;
    PM_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, comm_, s));
  }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_ = 1;
};

Comm* make_rccl_comm(const void* unique_id, int nranks, int rank) { return new RcclComm(unique_id, nranks, rank); }

size_t rccl_unique_id(void* out, size_t len) {
  ncclUniqueId id;
  if (len < sizeof(id)) throw std::runtime_error("unique id buffer shorter than ncclUniqueId");
  PM_NCCL_CHECK(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return sizeof(id);
}

// ---------------------------------------------------------------------------
// Threads of one process, all shards on one device (parity tests on a
// one-GPU box).  Shards compute one at a time (ThreadGroup::device is held
// outside collectives), so their cooperative line kernels never share the
// chip; a collective synchronises the caller's stream, releases the device,
// meets the other shards at a barrier and copies with hipMemcpy.
void ThreadGroup::barrier() {
  std::unique_lock<std::mutex> lk(m);
  if (aborted) throw std::runtime_error("another shard failed");
  const uint64_t g = gen;
  if (++arrived == n) {
    arrived = 0;
    ++gen;
    cv.notify_all();
    return;
  }
  cv.wait(lk, [&] { return gen != g || aborted; });
  if (aborted) throw std::runtime_error("another shard failed");
}

void ThreadGroup::abort() {
  std::lock_guard<std::mutex> lk(m);
  aborted = true;
  cv.notify_all();
}

namespace {
struct DeviceReleased {  // device mutex released for the scope of a collective
  explicit DeviceReleased(ThreadGroup* g) : g_(g) { g_->device.unlock(); }
  ~DeviceReleased() { g_->device.lock(); }
  ThreadGroup* g_;
};
}  // namespace

class ThreadComm : public Comm {
 public:
  ThreadComm(ThreadGroup* g, int rank) : g_(g), rank_(rank) {}
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));
    DeviceReleased rel(g_);
    g_->ptrs[rank_] = send;
    g_->barrier();
    // on the caller's stream, completed before the barrier: a device-to-device
    // hipMemcpy may return before the copy is done, and the caller's
    // non-blocking stream is not ordered after the null stream
    for (int q = 0; q < g_->n; ++q)
      if (bytes)
        PM_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + size_t(q) * bytes, g_->ptrs[q], bytes,
                                    hipMemcpyDeviceToDevice, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));
    g_->barrier();
  }
  void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));
    DeviceReleased rel(g_);
    std::vector<uint64_t> h(count), sum(count, 0);
    if (count) PM_HIP_CHECK(hipMemcpyAsync(h.data(), buf, count * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));
    g_->hvec[rank_] = &h;
    g_->barrier();
    for (int q = 0; q < g_->n; ++q)
      for (size_t i = 0; i < count; ++i) sum[i] += (*g_->hvec[q])[i];
    g_->barrier();
    if (count) PM_HIP_CHECK(hipMemcpyAsync(buf, sum.data(), count * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));
  }

 private:
  ThreadGroup* g_;
  int rank_;
};

Comm* make_thread_comm(ThreadGroup* g, int rank) { return new ThreadComm(g, rank); }

// ---------------------------------------------------------------------------
// exchange kernels
static constexpr int kXBlock = 256;

static unsigned xgrid(uint64_t items) {
  uint64_t g = (items + kXBlock - 1) / kXBlock;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, 65535)));
}

__global__ void k_pack_tpub(const uint32_t* __restrict__ slist, uint32_t nS, const uint16_t* __restrict__ tpub,
                            uint16_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nS; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = tpub[slist[i]];
}

// Entries of the other shards: tpub[xslist[g][i]] = recv[g][i].
__global__ void k_unpack_tpub(const uint32_t* __restrict__ xslist, const uint32_t* __restrict__ xnS, uint32_t maxS,
                              uint32_t G, uint32_t me, const uint16_t* __restrict__ recv, uint16_t* __restrict__ tpub) {
  const uint64_t total = uint64_t(G) * maxS;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxS), i = static_cast<uint32_t>(j % maxS);
    if (g != me && i < xnS[g]) tpub[xslist[j]] = recv[j];
  }
}

// Alive-entry count of each own slist entry in S (0 outside S and past nS).
__global__ void k_m_counts(const uint32_t* __restrict__ slist, uint32_t nS, uint32_t maxS,
                           const uint16_t* __restrict__ tpub, const uint32_t* __restrict__ malive,
                           uint32_t* __restrict__ cnt) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < maxS; i += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t x = 0;
    if (i < nS) {
      const uint32_t s = slist[i];
      if (tpub[s]) x = malive[s];
    }
    cnt[i] = x;
  }
}

// One wave per own slist entry: the alive entries of M[s], in row order, at
// out + moff[i] (ballot compaction).
__global__ __launch_bounds__(kXBlock) void k_m_pack(const uint32_t* __restrict__ slist, uint32_t nS,
                                                    const uint16_t* __restrict__ tpub,
                                                    const uint64_t* __restrict__ offp,
                                                    const uint32_t* __restrict__ mlen,
                                                    const uint32_t* __restrict__ mcol,
                                                    const uint64_t* __restrict__ moff, uint32_t* __restrict__ out) {
  const int lane = lane_id();
  const uint64_t nw = uint64_t(gridDim.x) * (kXBlock / kWave);
  for (uint64_t i = blockIdx.x * uint64_t(kXBlock / kWave) + threadIdx.x / kWave; i < nS; i += nw) {
    const uint32_t s = slist[i];
    if (!tpub[s]) continue;
    const uint64_t b = offp[s];
    const uint32_t L = mlen[s];
    uint64_t o = moff[i];
    for (uint32_t j0 = 0; j0 < L; j0 += kWave) {
      const uint32_t j = j0 + lane;
      const uint32_t x = j < L ? mcol[b + j] : 0u;
      const bool alive = (x & kAlive) != 0;
      const uint64_t bal = __ballot(alive);
      if (alive) out[o + __builtin_popcountll(bal & ((1ull << lane) - 1))] = x;
      o += __builtin_popcountll(bal);
    }
  }
}

// Start of each shard's block in the all-gathered counts' exclusive scan.
__global__ void k_seg_starts(const uint64_t* __restrict__ xoff, uint32_t maxS, uint32_t G, uint64_t* __restrict__ out) {
  const uint32_t g = threadIdx.x;
  if (g <= G) out[g] = xoff[uint64_t(g) * maxS];
}

// Remote rows: offp / mlen / malive of the other shards' slist entries point
// into the gathered region (block g at base + g * maxT).
__global__ void k_m_unpack(const uint32_t* __restrict__ xslist, const uint32_t* __restrict__ xnS,
                           const uint32_t* __restrict__ xcnt, const uint64_t* __restrict__ xoff,
                           const uint64_t* __restrict__ seg, uint32_t maxS, uint32_t G, uint32_t me, uint64_t base,
                           uint64_t maxT, uint64_t* __restrict__ offp, uint32_t* __restrict__ mlen,
                           uint32_t* __restrict__ malive) {
  const uint64_t total = uint64_t(G) * maxS;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxS), i = static_cast<uint32_t>(j % maxS);
    if (g == me || i >= xnS[g]) continue;
    const uint32_t p = xslist[j];
    offp[p] = base + uint64_t(g) * maxT + (xoff[j] - seg[g]);
    mlen[p] = xcnt[j];
    malive[p] = xcnt[j];
  }
}

// This shard's S members (slist entries with T_pub != 0), unordered.
__global__ void k_s_collect(const uint32_t* __restrict__ slist, uint32_t nS, const uint16_t* __restrict__ tpub,
                            uint32_t* __restrict__ out, unsigned int* __restrict__ ctr) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nS; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = slist[i];
    if (tpub[p]) out[atomicAdd(ctr, 1u)] = p;
  }
}

// ---------------------------------------------------------------------------
// host side
template <typename T>
static void regrow(T*& p, size_t& cap, size_t want) {
  if (cap >= want && p) return;
  if (p) (void)hipFree(p);
  p = nullptr;
  PM_HIP_CHECK(hipMalloc(&p, std::max<size_t>(1, want) * sizeof(T)));
  cap = want;
}

std::vector<uint64_t> shard_allreduce(Ctx& c, const std::vector<uint64_t>& v) {
  if (!c.comm || v.empty()) return v;
  regrow(c.d_xred, c.xred_cap, v.size());
  PM_HIP_CHECK(hipMemcpyAsync(c.d_xred, v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  c.comm->allreduce_sum_u64(c.d_xred, v.size(), c.stream);
  std::vector<uint64_t> out(v.size());
  PM_HIP_CHECK(hipMemcpyAsync(out.data(), c.d_xred, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return out;
}

std::vector<std::vector<uint32_t>> shard_allgatherv(Ctx& c, const std::vector<uint32_t>& v) {
  if (!c.comm) return {v};
  const uint32_t G = c.nshards;
  std::vector<uint64_t> sz(G, 0);
  sz[c.shard] = v.size();
  sz = shard_allreduce(c, sz);
  const uint64_t maxL = std::max<uint64_t>(1, *std::max_element(sz.begin(), sz.end()));
  uint32_t *d_send = nullptr, *d_recv = nullptr;
  PM_HIP_CHECK(hipMalloc(&d_send, maxL * sizeof(uint32_t)));
  PM_HIP_CHECK(hipMalloc(&d_recv, G * maxL * sizeof(uint32_t)));
  std::vector<uint32_t> all(G * maxL);
  try {
    if (!v.empty())
      PM_HIP_CHECK(hipMemcpyAsync(d_send, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
    c.comm->allgather(d_send, d_recv, maxL * sizeof(uint32_t), c.stream);
    PM_HIP_CHECK(hipMemcpyAsync(all.data(), d_recv, all.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  } catch (...) {
    (void)hipFree(d_send);
    (void)hipFree(d_recv);
    throw;
  }
  (void)hipFree(d_send);
  (void)hipFree(d_recv);
  std::vector<std::vector<uint32_t>> out(G);
  for (uint32_t g = 0; g < G; ++g) out[g].assign(all.begin() + g * maxL, all.begin() + g * maxL + sz[g]);
  return out;
}

void shard_exchange_tpub(Ctx& c) {
  if (!c.comm) return;
  const uint32_t G = c.nshards, maxS = c.xmaxS, nS = c.xnS[c.shard];
  if (nS) hipLaunchKernelGGL(k_pack_tpub, dim3(xgrid(nS)), dim3(kXBlock), 0, c.stream, c.d_slist, nS, c.d_tpub[c.cur],
                             c.d_xsend);
  c.comm->allgather(c.d_xsend, c.d_xrecv, size_t(maxS) * sizeof(uint16_t), c.stream);
  hipLaunchKernelGGL(k_unpack_tpub, dim3(xgrid(uint64_t(G) * maxS)), dim3(kXBlock), 0, c.stream, c.d_xslist, c.d_xnS,
                     maxS, G, c.shard, c.d_xrecv, c.d_tpub[c.cur]);
  PM_HIP_CHECK(hipGetLastError());
}

void shard_exchange_tpub_s(Ctx& c) {
  if (!c.comm) return;
  const uint32_t G = c.nshards, maxA = std::max<uint32_t>(c.amax, 1), nA = c.anum[c.shard];
  if (nA) hipLaunchKernelGGL(k_pack_tpub, dim3(xgrid(nA)), dim3(kXBlock), 0, c.stream, c.d_aown, nA, c.d_tpub[c.cur],
                             c.d_asend);
  c.comm->allgather(c.d_asend, c.d_arecv, size_t(maxA) * sizeof(uint16_t), c.stream);
  hipLaunchKernelGGL(k_unpack_tpub, dim3(xgrid(uint64_t(G) * maxA)), dim3(kXBlock), 0, c.stream, c.d_axl, c.d_anum,
                     maxA, G, c.shard, c.d_arecv, c.d_tpub[c.cur]);
  PM_HIP_CHECK(hipGetLastError());
}

void shard_after_first(Ctx& c) {
  if (!c.comm) return;
  const uint32_t G = c.nshards;
  uint32_t nS = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&nS, c.d_nS, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.nS_host = nS;
  std::vector<uint64_t> cnt(G, 0);
  cnt[c.shard] = nS;
  cnt = shard_allreduce(c, cnt);
  c.xnS.assign(G, 0);
  uint32_t maxS = 1;
  for (uint32_t g = 0; g < G; ++g) {
    c.xnS[g] = static_cast<uint32_t>(cnt[g]);
    maxS = std::max(maxS, c.xnS[g]);
  }
  if (maxS > c.xmaxS || !c.d_xslist) {
    void* ptrs[] = {c.d_xslist, c.d_xnS, c.d_xsend, c.d_xrecv};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    PM_HIP_CHECK(hipMalloc(&c.d_xslist, size_t(G) * maxS * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_xnS, G * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_xsend, size_t(maxS) * sizeof(uint16_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_xrecv, size_t(G) * maxS * sizeof(uint16_t)));
  }
  c.xmaxS = maxS;
  PM_HIP_CHECK(hipMemcpyAsync(c.d_xnS, c.xnS.data(), G * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  // d_slist holds V entries >= maxS: the block past nS is padding
  c.comm->allgather(c.d_slist, c.d_xslist, size_t(maxS) * sizeof(uint32_t), c.stream);
  shard_exchange_tpub(c);
  c.m_dirty = true;
}

void shard_replicate_m(Ctx& c) {
  if (!c.comm || !c.m_dirty) return;
  const uint32_t G = c.nshards, nS = c.xnS[c.shard];
  const uint16_t* tpub = c.d_tpub[c.cur];
  c.arena.reset();
  // 1. this shard's S list (the only rows token passing reads from it), then every shard's
  if (c.acap < std::max<uint32_t>(nS, 1)) {
    if (c.d_aown) (void)hipFree(c.d_aown);
    c.acap = std::max<uint32_t>(nS, 1);
    PM_HIP_CHECK(hipMalloc(&c.d_aown, c.acap * sizeof(uint32_t)));
  }
  auto* actr = static_cast<unsigned int*>(c.arena.get(sizeof(unsigned int)));
  PM_HIP_CHECK(hipMemsetAsync(actr, 0, sizeof(unsigned int), c.stream));
  if (nS)
    hipLaunchKernelGGL(k_s_collect, dim3(xgrid(nS)), dim3(kXBlock), 0, c.stream, c.d_slist, nS, tpub, c.d_aown, actr);
  uint64_t* pin = pinned(c, 4);
  PM_HIP_CHECK(hipMemcpyAsync(pin, actr, sizeof(unsigned int), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  const uint32_t na = static_cast<uint32_t>(pin[0] & 0xFFFFFFFFull);
  std::vector<uint64_t> an(G, 0);
  an[c.shard] = na;
  an = shard_allreduce(c, an);
  c.anum.assign(G, 0);
  uint32_t amax = 1;
  for (uint32_t g = 0; g < G; ++g) {
    c.anum[g] = static_cast<uint32_t>(an[g]);
    amax = std::max(amax, c.anum[g]);
  }
  if (amax > c.amax || !c.d_axl) {
    void* ptrs[] = {c.d_axl, c.d_anum, c.d_asend, c.d_arecv};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    PM_HIP_CHECK(hipMalloc(&c.d_axl, size_t(G) * amax * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_anum, G * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_asend, size_t(amax) * sizeof(uint16_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_arecv, size_t(G) * amax * sizeof(uint16_t)));
  }
  if (c.acap < amax) {  // the send block is amax entries long
    uint32_t* nb = nullptr;
    PM_HIP_CHECK(hipMalloc(&nb, amax * sizeof(uint32_t)));
    if (na) PM_HIP_CHECK(hipMemcpyAsync(nb, c.d_aown, na * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    (void)hipFree(c.d_aown);
    c.d_aown = nb;
    c.acap = amax;
  }
  c.amax = amax;
  PM_HIP_CHECK(hipMemcpyAsync(c.d_anum, c.anum.data(), G * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  c.comm->allgather(c.d_aown, c.d_axl, size_t(amax) * sizeof(uint32_t), c.stream);
  // 2. alive-entry counts per S entry, every shard's, and their exclusive scans
  auto* cnt = static_cast<uint32_t*>(c.arena.get(size_t(amax) * sizeof(uint32_t)));
  auto* xcnt = static_cast<uint32_t*>(c.arena.get(size_t(G) * amax * sizeof(uint32_t)));
  auto* moff = static_cast<uint64_t*>(c.arena.get((size_t(amax) + 1) * sizeof(uint64_t)));
  auto* xoff = static_cast<uint64_t*>(c.arena.get((size_t(G) * amax + 1) * sizeof(uint64_t)));
  auto* seg = static_cast<uint64_t*>(c.arena.get((G + 1) * sizeof(uint64_t)));
  hipLaunchKernelGGL(k_m_counts, dim3(xgrid(amax)), dim3(kXBlock), 0, c.stream, c.d_aown, na, amax, tpub, c.d_malive,
                     cnt);
  c.comm->allgather(cnt, xcnt, size_t(amax) * sizeof(uint32_t), c.stream);
  PM_HIP_CHECK(hipMemsetAsync(moff, 0, sizeof(uint64_t), c.stream));
  PM_HIP_CHECK(hipMemsetAsync(xoff, 0, sizeof(uint64_t), c.stream));
  size_t t1 = 0, t2 = 0;
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, t1, cnt, moff + 1, static_cast<int>(amax), c.stream));
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, t2, xcnt, xoff + 1, static_cast<int>(uint64_t(G) * amax),
                                                c.stream));
  size_t tb = std::max(t1, t2);
  void* tmp = c.arena.get(tb);
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp, tb, cnt, moff + 1, static_cast<int>(amax), c.stream));
  tb = std::max(t1, t2);
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp, tb, xcnt, xoff + 1, static_cast<int>(uint64_t(G) * amax),
                                                c.stream));
  hipLaunchKernelGGL(k_seg_starts, dim3(1), dim3(64 * ((G + 64) / 64)), 0, c.stream, xoff, amax, G, seg);
  pin = pinned(c, G + 1);
  PM_HIP_CHECK(hipMemcpyAsync(pin, seg, (G + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  uint64_t maxT = 1;
  for (uint32_t g = 0; g < G; ++g) maxT = std::max(maxT, pin[g + 1] - pin[g]);
  // 3. the alive rows of every shard's S into the remote region after this shard's own slots
  const uint64_t need = c.nq + uint64_t(G) * maxT;
  if (need > c.mcap) {
    const uint64_t cap = std::max(need, c.mcap + c.mcap / 4);
    uint32_t* nb = nullptr;
    PM_HIP_CHECK(hipMalloc(&nb, (cap + kTileEntries) * sizeof(uint32_t)));  // + tail padding (k1_load)
    if (c.nq) PM_HIP_CHECK(hipMemcpyAsync(nb, c.d_mcol, c.nq * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    (void)hipFree(c.d_mcol);
    c.d_mcol = nb;
    c.mcap = cap;
  }
  auto* send = static_cast<uint32_t*>(c.arena.get(maxT * sizeof(uint32_t)));
  if (na)
    hipLaunchKernelGGL(k_m_pack, dim3(xgrid(uint64_t(na) * kWave)), dim3(kXBlock), 0, c.stream, c.d_aown, na, tpub,
                       c.d_offp, c.d_mlen, c.d_mcol, moff, send);
  c.comm->allgather(send, c.d_mcol + c.nq, maxT * sizeof(uint32_t), c.stream);
  hipLaunchKernelGGL(k_m_unpack, dim3(xgrid(uint64_t(G) * amax)), dim3(kXBlock), 0, c.stream, c.d_axl, c.d_anum, xcnt,
                     xoff, seg, amax, G, c.shard, c.nq, maxT, c.d_offp, c.d_mlen, c.d_malive);
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.arena.reset();
  c.m_dirty = false;
}

}  // namespace pm
