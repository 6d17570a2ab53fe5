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
//   * NLCC / TDS: after every walk position the tokens (vertex, source,
//     parent) and walks move to the owner of their next vertex in one RCCL
//     all-to-all (shard_route: ncclSend / ncclRecv pairs in a group), so the
//     (vertex, source) dedup of nem_1.hpp:131-139, M[u] and the terminal
//     checks stay local; acknowledgements travel to the source's owner;
//   * counters and flags: one u64 sum all-reduce per LCC call / NLC line.
// Results are identical for every shard count.

#include <hip/hip_runtime.h>

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
  // Every call goes through RCCL, one rank included (tests/test_gpu_shards.py
  // ::test_rccl_shard_single_rank exercises the communicator); zero-sized calls
  // are skipped on the host.
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (!bytes) return;
    PM_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }
  void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    if (!count) return;
    PM_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, comm_, s));
  }
  // grouped point-to-point sends / receives over xGMI (one pair per peer)
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                 hipStream_t s) override {
    uint64_t so = 0, ro = 0;
    PM_NCCL_CHECK(ncclGroupStart());
    for (int g = 0; g < nranks_; ++g) {
      if (sbytes[g]) PM_NCCL_CHECK(ncclSend(static_cast<const char*>(send) + so, sbytes[g], ncclUint8, g, comm_, s));
      if (rbytes[g]) PM_NCCL_CHECK(ncclRecv(static_cast<char*>(recv) + ro, rbytes[g], ncclUint8, g, comm_, s));
      so += sbytes[g];
      ro += rbytes[g];
    }
    PM_NCCL_CHECK(ncclGroupEnd());
  }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_ = 1;
};

Comm* make_rccl_comm(const void* unique_id, int nranks, int rank) { return new RcclComm(unique_id, nranks, rank); }

// Diagnostics: one-rank RCCL collective of `bytes` on `device` (op 0:
// ncclAllGather, 1: ncclAllReduce u64 sum), result checked; the communicator
// is created and destroyed here.  Returns 0 when the result is right.
int rccl_selftest(int device, uint64_t bytes, int op) {
  PM_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  PM_NCCL_CHECK(ncclGetUniqueId(&id));
  ncclComm_t comm = nullptr;
  PM_NCCL_CHECK(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t st;
  PM_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const uint64_t words = bytes / 8;  // 0: a zero-sized collective
  uint64_t *a = nullptr, *b = nullptr;
  PM_HIP_CHECK(hipMalloc(&a, std::max<uint64_t>(words, 1) * 8));
  PM_HIP_CHECK(hipMalloc(&b, std::max<uint64_t>(words, 1) * 8));
  std::vector<uint64_t> h(words);
  for (uint64_t i = 0; i < words; ++i) h[i] = i * 0x9E3779B97F4A7C15ull;
  if (words) PM_HIP_CHECK(hipMemcpy(a, h.data(), words * 8, hipMemcpyHostToDevice));
  if (op == 0) PM_NCCL_CHECK(ncclAllGather(a, b, words * 8, ncclUint8, comm, st));
  else PM_NCCL_CHECK(ncclAllReduce(a, b, words, ncclUint64, ncclSum, comm, st));
  PM_HIP_CHECK(hipStreamSynchronize(st));
  std::vector<uint64_t> r(words);
  if (words) PM_HIP_CHECK(hipMemcpy(r.data(), b, words * 8, hipMemcpyDeviceToHost));
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipStreamDestroy(st);
  (void)ncclCommDestroy(comm);
  return r == h ? 0 : 1;
}

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
// outside collectives), so their kernels never share the chip; a collective
// synchronises the caller's stream, releases the device, meets the other
// shards at a barrier and copies with hipMemcpyAsync on the caller's stream
// (synchronised before the closing barrier).
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
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                 hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));
    DeviceReleased rel(g_);
    const int G = g_->n;
    g_->ptrs[rank_] = send;
    g_->counts[rank_].assign(sbytes, sbytes + G);
    g_->barrier();
    uint64_t ro = 0;
    for (int q = 0; q < G; ++q) {  // block for this rank inside shard q's send buffer
      uint64_t off = 0;
      for (int k = 0; k < rank_; ++k) off += g_->counts[q][k];
      const uint64_t n = g_->counts[q][rank_];
      if (n != rbytes[q]) throw std::runtime_error("alltoallv: receive size mismatch");
      if (n)
        PM_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + ro, static_cast<const char*>(g_->ptrs[q]) + off, n,
                                    hipMemcpyDeviceToDevice, s));
      ro += n;
    }
    PM_HIP_CHECK(hipStreamSynchronize(s));
    g_->barrier();
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

// Owner-bucketed routing of fixed-size records (the mailbox exchange of
// new_mailbox.hpp:289-713 as one RCCL all-to-all per BSP step): record i is
// `words` u32, its destination the owner of the position in word kw.
__global__ void k_route_count(const uint32_t* __restrict__ items, uint64_t n, int words, int kw,
                              const uint32_t* __restrict__ perm, uint32_t G, uint32_t* __restrict__ dest,
                              unsigned long long* __restrict__ cnt) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = perm[items[i * words + kw]] % G;
    dest[i] = g;
    atomicAdd(&cnt[g], 1ull);
  }
}

__global__ void k_route_scatter(const uint32_t* __restrict__ items, uint64_t n, int words,
                                const uint32_t* __restrict__ dest, unsigned long long* __restrict__ cursor,
                                uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t o = atomicAdd(&cursor[dest[i]], 1ull);
    for (int w = 0; w < words; ++w) out[o * words + w] = items[i * words + w];
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

uint32_t* shard_route(Ctx& c, const uint32_t* items, uint64_t n, int words, int kw, uint64_t& nout) {
  const uint32_t G = c.nshards;
  auto* cnt = static_cast<unsigned long long*>(c.arena.get(2 * G * sizeof(unsigned long long)));
  auto* cursor = cnt + G;
  auto* allc = static_cast<uint64_t*>(c.arena.get(uint64_t(G) * G * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMemsetAsync(cnt, 0, G * sizeof(unsigned long long), c.stream));
  auto* dest = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(n, 1) * sizeof(uint32_t)));
  if (n)
    hipLaunchKernelGGL(k_route_count, dim3(xgrid(n)), dim3(kXBlock), 0, c.stream, items, n, words, kw, c.d_perm, G,
                       dest, cnt);
  c.comm->allgather(cnt, allc, G * sizeof(uint64_t), c.stream);  // allc[q * G + g]: shard q -> shard g
  std::vector<uint64_t> m(uint64_t(G) * G);
  PM_HIP_CHECK(hipMemcpyAsync(m.data(), allc, m.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  std::vector<uint64_t> sb(G), rb(G), soff(G, 0);
  uint64_t nrecv = 0;
  for (uint32_t g = 0; g < G; ++g) {
    sb[g] = m[uint64_t(c.shard) * G + g] * words * sizeof(uint32_t);
    rb[g] = m[uint64_t(g) * G + c.shard] * words * sizeof(uint32_t);
    nrecv += m[uint64_t(g) * G + c.shard];
    if (g) soff[g] = soff[g - 1] + m[uint64_t(c.shard) * G + g - 1];
  }
  auto* send = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(n, 1) * words * sizeof(uint32_t)));
  auto* recv = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(nrecv, 1) * words * sizeof(uint32_t)));
  if (n) {
    PM_HIP_CHECK(hipMemcpyAsync(cursor, soff.data(), G * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(k_route_scatter, dim3(xgrid(n)), dim3(kXBlock), 0, c.stream, items, n, words, dest, cursor,
                       send);
  }
  PM_HIP_CHECK(hipGetLastError());
  c.comm->alltoallv(send, sb.data(), recv, rb.data(), c.stream);
  nout = nrecv;
  return recv;
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
}

}  // namespace pm
