// Sharded search: the exchanges between the shards of one
// pattern search and the two Comm implementations.
//
// The reference partitions vertices 1D-cyclically (owner = id % P,
// delegate_partitioned_graph.ipp:1679-1696) and moves every LCC/NLCC message
// through the MPI mailbox (new_mailbox.hpp:289-713); state sync of delegates
// uses MPI_Allreduce (impl/vertex_data.hpp:114-126).  Here shard q owns the
// rows of ids v % nshards == q and the search is BSP with three exchanges:
//   * after superstep 0 (the full-adjacency scan, split over the shards): the
//     survivors' T_pub codes, all-gathered (2 bits per survivor + its position),
//     which is all the first later superstep's row pulls read of other shards;
//   * after that superstep (S has collapsed: S=28 tree 9.8 M -> 0.8 M vertices,
//     31 M -> 0.85 M edges): the state of S -- T_pub, T_state, M rows --
//     all-gathered into a replica that every shard holds; the rest of the
//     search (later supersteps, NLC lines, later LCC calls) runs on the replica
//     with no further exchange, identically on every shard;
//   * counters: one u64 sum all-reduce over the sharded supersteps' slots.
// Results are identical for every shard count.

#include <hip/hip_runtime.h>

#include <rccl/rccl.h>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

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
    Timer timer(this);
    count(bytes);
    if (!bytes) return;
    PM_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }
  void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    Timer timer(this);
    Comm::count(count * 8);
    if (!count) return;
    PM_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, comm_, s));
  }
  void allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t s) override {
    Timer timer(this);
    Comm::count(count * 4);
    if (!count) return;
    PM_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint32, ncclSum, comm_, s));
  }
  // grouped point-to-point sends / receives over xGMI (one pair per peer)
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                 hipStream_t s) override {
    Timer timer(this);
    uint64_t so = 0, ro = 0;
    for (int g = 0; g < nranks_; ++g) so += sbytes[g];
    count(so);
    so = 0;
    PM_NCCL_CHECK(ncclGroupStart());
    for (int g = 0; g < nranks_; ++g) {
      if (sbytes[g]) PM_NCCL_CHECK(ncclSend(static_cast<const char*>(send) + so, sbytes[g], ncclUint8, g, comm_, s));
      if (rbytes[g]) PM_NCCL_CHECK(ncclRecv(static_cast<char*>(recv) + ro, rbytes[g], ncclUint8, g, comm_, s));
      so += sbytes[g];
      ro += rbytes[g];
    }
    PM_NCCL_CHECK(ncclGroupEnd());
  }
  int ranks() const override {
    int c = 0;
    PM_NCCL_CHECK(ncclCommCount(comm_, &c));
    return c;
  }
  int transport() const override { return PM_TRANSPORT_RCCL; }

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
// Host-staged collectives of the caller (include/pm_abi.h pm_host_comm): the exchange the reference makes
// over MPI (new_mailbox.hpp:358-405, impl/vertex_data.hpp:114-126), with the transport left to the host --
// an MPI communicator, torch.distributed gloo (tests/test_gpu_multiprocess.py), any process group.  Every
// call synchronises the stream, copies the device buffer to pinned host staging, calls the caller's
// collective and copies the result back; the processes may share one device or use one each.
class HostComm : public Comm {
 public:
  explicit HostComm(const pm_host_comm& h) : h_(h) {
    if (!h.allgather || !h.allreduce_sum_u64 || !h.allreduce_sum_u32 || !h.alltoallv)
      throw std::runtime_error("pm_host_comm: every collective must be given");
  }
  ~HostComm() override {
    for (auto& b : buf_)
      if (b.p) (void)hipHostFree(b.p);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    count(bytes);
    const int G = size();
    char* hs = stage(0, bytes);
    char* hr = stage(1, bytes * G);
    to_host(hs, send, bytes, s);
    check(h_.allgather(h_.user, hs, hr, bytes), "allgather");
    to_device(recv, hr, bytes * G, s);
  }
  void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    Comm::count(count * 8);
    auto* h = reinterpret_cast<uint64_t*>(stage(0, count * 8));
    to_host(h, buf, count * 8, s);
    check(h_.allreduce_sum_u64(h_.user, h, count), "allreduce_sum_u64");
    to_device(buf, h, count * 8, s);
  }
  void allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    Comm::count(count * 4);
    auto* h = reinterpret_cast<uint32_t*>(stage(0, count * 4));
    to_host(h, buf, count * 4, s);
    check(h_.allreduce_sum_u32(h_.user, h, count), "allreduce_sum_u32");
    to_device(buf, h, count * 4, s);
  }
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                 hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    const int G = size();
    uint64_t so = 0, ro = 0;
    for (int g = 0; g < G; ++g) {
      so += sbytes[g];
      ro += rbytes[g];
    }
    count(so);
    char* hs = stage(0, so);
    char* hr = stage(1, ro);
    to_host(hs, send, so, s);
    check(h_.alltoallv(h_.user, hs, sbytes, hr, rbytes), "alltoallv");
    to_device(recv, hr, ro, s);
  }
  int ranks() const override { return static_cast<int>(h_.nshards); }
  int transport() const override { return PM_TRANSPORT_HOST; }

 private:
  struct Buf {
    char* p = nullptr;
    size_t cap = 0;
  };
  int size() const { return static_cast<int>(h_.nshards); }
  char* stage(int k, size_t bytes) {
    Buf& b = buf_[k];
    if (b.cap < bytes || !b.p) {
      if (b.p) (void)hipHostFree(b.p);
      b.p = nullptr;
      const size_t cap = std::max<size_t>(bytes + bytes / 4, 1 << 16);
      PM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.p), cap, hipHostMallocDefault));
      b.cap = cap;
    }
    return b.p;
  }
  static void to_host(void* h, const void* d, size_t bytes, hipStream_t s) {
    if (bytes) PM_HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (also orders the caller's kernels before the exchange)
  }
  static void to_device(void* d, const void* h, size_t bytes, hipStream_t s) {
    if (bytes) PM_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the staging buffer is reused by the next call)
  }
  static void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string("pm_host_comm ") + what + " failed (" + std::to_string(rc) + ")");
  }
  pm_host_comm h_;
  Buf buf_[2];
};

Comm* make_host_comm(const pm_host_comm& h) { return new HostComm(h); }

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
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    count(bytes);
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
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    Comm::count(count * 8);
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
  void allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    Comm::count(count * 4);
    DeviceReleased rel(g_);
    std::vector<uint32_t> h(count);
    std::vector<uint64_t> hv(count);
    if (count) PM_HIP_CHECK(hipMemcpyAsync(h.data(), buf, count * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));
    for (size_t i = 0; i < count; ++i) hv[i] = h[i];
    g_->hvec[rank_] = &hv;
    g_->barrier();
    std::vector<uint32_t> sum(count, 0);
    for (int q = 0; q < g_->n; ++q)
      for (size_t i = 0; i < count; ++i) sum[i] += static_cast<uint32_t>((*g_->hvec[q])[i]);
    g_->barrier();
    if (count) PM_HIP_CHECK(hipMemcpyAsync(buf, sum.data(), count * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    PM_HIP_CHECK(hipStreamSynchronize(s));
  }
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                 hipStream_t s) override {
    PM_HIP_CHECK(hipStreamSynchronize(s));  // (the shard's own work: not collective time)
    Timer timer(this);
    uint64_t sent = 0;
    for (int q = 0; q < g_->n; ++q) sent += sbytes[q];
    count(sent);
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
  int ranks() const override { return g_->n; }
  int transport() const override { return PM_TRANSPORT_THREADS; }

 private:
  ThreadGroup* g_;
  int rank_;
};

Comm* make_thread_comm(ThreadGroup* g, int rank) { return new ThreadComm(g, rank); }

// ---------------------------------------------------------------------------
// exchange kernels
static constexpr int kXBlock = 256;

// Per-shard counts of one gather, passed by value (G <= 64): rows / entries and
// their first index in the concatenation over the shards.
struct XCounts {
  uint64_t n[64], m[64], base[64], ebase[64];
};

static unsigned xgrid(uint64_t items) {
  uint64_t g = (items + kXBlock - 1) / kXBlock;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, 65535)));
}

template <typename T>
static T* grow(void*& p, size_t& cap, size_t bytes) {
  if (cap < bytes || !p) {
    if (p) (void)hipFree(p);
    p = nullptr;
    const size_t b = std::max<size_t>(bytes + bytes / 8, 4096);
    PM_HIP_CHECK(hipMalloc(&p, b));
    cap = b;
  }
  return static_cast<T*>(p);
}

__global__ void k_count_to_u64(const uint32_t* __restrict__ n, uint64_t* __restrict__ out) { *out = *n; }

// Code records of this shard's superstep-0 survivors: position | code << 30
// (2-bit tpub_code), or, when some label has more than two template vertices
// (its code 3 means "gather T_pub"), position | T_pub << 32 | code << 62.
__global__ void k_pack_codes(const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp,
                             const uint32_t* __restrict__ tcode, const uint16_t* __restrict__ tpub,
                             const uint4* __restrict__ srec, int wide, LabelRuns lr, uint32_t* __restrict__ out32,
                             unsigned long long* __restrict__ out64) {
  const uint64_t n = *nSp;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = slist[i];
    const uint32_t ci = code_index(p, lr);  // (a member of S: in its label's run)
    const uint32_t code = (tcode[ci >> 4] >> ((ci & 15u) << 1)) & 3u;
    const uint16_t T = srec ? static_cast<uint16_t>(srec[i].y) : tpub[p];  // superstep-0 records: T_pub there
    if (wide) out64[i] = p | (static_cast<unsigned long long>(T) << 32) | (static_cast<unsigned long long>(code) << 62);
    else out32[i] = p | (code << 30);
  }
}

// The other shards' code records into this shard's 2-bit codes (and T_pub).
__global__ void k_unpack_codes(const uint32_t* __restrict__ in32, const unsigned long long* __restrict__ in64,
                               uint64_t maxS, uint32_t G, uint32_t me, XCounts x, LabelRuns lr,
                               uint32_t* __restrict__ tcode, uint16_t* __restrict__ tpub) {
  const uint64_t total = uint64_t(G) * maxS;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxS);
    if (g == me || j % maxS >= x.n[g]) continue;
    uint32_t p, code;
    if (in64) {
      const unsigned long long r = in64[j];
      p = static_cast<uint32_t>(r & 0x3FFFFFFFull);
      code = static_cast<uint32_t>(r >> 62);
      tpub[p] = static_cast<uint16_t>(r >> 32);  // (the next superstep's code-3 gathers, k_lcc_step tpub_of)
    } else {
      p = in32[j] & 0x3FFFFFFFu;
      code = in32[j] >> 30;
    }
    const uint32_t ci = code_index(p, lr);
    atomicOr(&tcode[ci >> 4], code << ((ci & 15u) << 1));
  }
}

// u64 mode, after the first later superstep: the T_pub buffer superstep 0
// wrote (read by that superstep) is cleared at the other shards' survivors.
__global__ void k_clear_codes(const unsigned long long* __restrict__ in64, uint64_t maxS, uint32_t G, uint32_t me,
                              XCounts x, uint16_t* __restrict__ tpub) {
  const uint64_t total = uint64_t(G) * maxS;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxS);
    if (g == me || j % maxS >= x.n[g]) continue;
    tpub[static_cast<uint32_t>(in64[j] & 0x3FFFFFFFull)] = 0;
  }
}

// pack_state, pass 1: per slist entry whether it is in S and its alive M count.
__global__ void k_pack_count(const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp, uint64_t cap,
                             const uint16_t* __restrict__ tpub, const uint32_t* __restrict__ malive,
                             uint32_t* __restrict__ keep, uint32_t* __restrict__ cnt) {
  const uint64_t n = min(static_cast<uint64_t>(*nSp), cap);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < cap; i += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t k = 0, m = 0;
    if (i < n) {
      const uint32_t u = slist[i];
      if (tpub[u]) {
        k = 1;
        m = malive[u];
      }
    }
    keep[i] = k;
    cnt[i] = m;
  }
}

// pass 2: rows {position, T_pub | T_state << 16, |M|, first entry} and their alive entries.  A wave per 64
// rows: rows of up to kPackShort entries are walked by their lane, longer ones (delegates: 10^5 entries at C5's
// scale) by the whole wave in turn (a lane walking a hub row took 0.1 s).
static constexpr uint32_t kPackShort = 32;
__global__ void k_pack_write(const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp, uint64_t cap,
                             const uint32_t* __restrict__ keep, const uint32_t* __restrict__ ridx,
                             const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ eoff,
                             const uint16_t* __restrict__ tpub, const uint16_t* __restrict__ tst,
                             const uint32_t* __restrict__ mlen, const uint64_t* __restrict__ moff,
                             const uint32_t* __restrict__ mcol, uint32_t* __restrict__ rec, uint32_t* __restrict__ ent,
                             uint64_t ent_cap, uint64_t nv,
                             unsigned long long* __restrict__ totals, unsigned long long* __restrict__ err) {
  const uint64_t n = min(static_cast<uint64_t>(*nSp), cap);
  const int lane = threadIdx.x & 63;
  const uint64_t nw = uint64_t(gridDim.x) * (blockDim.x / 64);
  for (uint64_t ch = blockIdx.x * uint64_t(blockDim.x / 64) + threadIdx.x / 64; ch * 64 < n; ch += nw) {
    const uint64_t i = ch * 64 + lane;
    bool mine = false;
    uint32_t u = 0, L = 0, c = 0;
    uint64_t b = 0, e0 = 0;
    if (i < n) {
      if (i == n - 1) {
        totals[0] = ridx[i] + keep[i];
        totals[1] = eoff[i] + cnt[i];
      }
      if (keep[i] && rec) {
        u = slist[i];
        b = moff[u];
        L = mlen[u];
        c = cnt[i];
        e0 = eoff[i];
        uint32_t* r = rec + 4 * uint64_t(ridx[i]);
        r[0] = u;
        r[1] = tpub[u] | (static_cast<uint32_t>(tst[u]) << 16);
        r[2] = c;
        r[3] = static_cast<uint32_t>(e0);
        mine = true;
      }
    }
    if (mine && L <= kPackShort) {
      uint64_t k = e0;
      for (uint32_t j = 0; j < L; ++j) {
        const uint32_t m = mcol[b + j];
        if (!(m & kAlive)) continue;
        if ((m & kPosMask) >= nv) {  // (not an M entry: the row's bounds are wrong -- reported, not packed)
          atomicCAS(err, 0ull, (1ull << 63) | u);
          continue;
        }
        if (k < ent_cap) ent[k++] = m;
      }
      if (k - e0 != c && e0 + c <= ent_cap) atomicCAS(err, 0ull, (1ull << 62) | u);  // |M| != alive entries
    }
    uint64_t lb = __ballot(mine && L > kPackShort);
    while (lb) {
      const int q = __ffsll(static_cast<long long>(lb)) - 1;
      lb &= lb - 1;
      const uint32_t uq = __shfl(u, q, 64), Lq = __shfl(L, q, 64), cq = __shfl(c, q, 64);
      const uint64_t bq = __shfl(b, q, 64);
      const uint64_t e0q = __shfl(e0, q, 64);
      uint64_t k = e0q;
      for (uint32_t j0 = 0; j0 < Lq; j0 += 64) {
        const uint32_t j = j0 + lane;
        const uint32_t m = j < Lq ? mcol[bq + j] : 0u;
        const bool bad = (m & kAlive) && (m & kPosMask) >= nv;
        if (bad) atomicCAS(err, 0ull, (1ull << 63) | uq);
        const bool ok = (m & kAlive) && !bad;
        const uint64_t bal = __ballot(ok);
        const uint64_t at = k + __builtin_popcountll(bal & ((1ull << lane) - 1));
        if (ok && at < ent_cap) ent[at] = m;
        k += __builtin_popcountll(bal);
      }
      if (lane == 0 && k - e0q != cq && e0q + cq <= ent_cap) atomicCAS(err, 0ull, (1ull << 62) | uq);
    }
  }
  if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) totals[0] = totals[1] = 0;
}

// The replica: every shard's rows (block g of the gather, x.n[g] rows) in shard order.
__global__ void k_unpack_rows(const uint32_t* __restrict__ rec, uint64_t maxR, uint32_t G, XCounts x,
                              uint32_t* __restrict__ slist, uint16_t* __restrict__ tpub, uint16_t* __restrict__ tst,
                              uint32_t* __restrict__ mlen, uint32_t* __restrict__ malive,
                              uint64_t* __restrict__ rmoff) {
  const uint64_t total = uint64_t(G) * maxR;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxR);
    const uint64_t i = j % maxR;
    if (i >= x.n[g]) continue;
    const uint32_t* r = rec + 4 * j;
    const uint32_t u = r[0];
    slist[x.base[g] + i] = u;
    tpub[u] = static_cast<uint16_t>(r[1]);
    tst[u] = static_cast<uint16_t>(r[1] >> 16);
    mlen[u] = r[2];
    malive[u] = r[2];
    rmoff[u] = x.ebase[g] + r[3];
  }
}

__global__ void k_unpack_entries(const uint32_t* __restrict__ ent, uint64_t maxE, uint32_t G, XCounts x,
                                 uint32_t* __restrict__ rmcol) {
  const uint64_t total = uint64_t(G) * maxE;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxE);
    const uint64_t e = j % maxE;
    if (e < x.m[g]) rmcol[x.ebase[g] + e] = ent[j];
  }
}


// ---------------------------------------------------------------------------
// Delegates (hubs) of a sharded search.  A hub's row is split over the shards
// by target owner (delegate_partitioned_graph.ipp:1402-1648); superstep 0
// scans every share like a heavy row but leaves its TN / distinct count in the
// heavy scratch.  The shares meet at the controller (hub ordinal % nshards,
// ipp:346-355): the partial (count, TN) pairs are all-gathered and OR-ed /
// summed -- the all-gather + OR that stands in for the delegates'
// all_max_reduce (impl/vertex_data.hpp:114-126; RCCL has no bitwise-OR
// reduction) -- and the shares' M entries travel to the controller in one
// all-to-all (grouped ncclSend / ncclRecv), which verifies the hub and holds
// its whole M row (the reference's controller also owns the hub's full
// active-edge map after superstep 0, nonunique_ee.hpp:589-624).
__global__ void k_hub_partials(const HubInfo* __restrict__ info, uint32_t H, const uint32_t* __restrict__ hscr,
                               uint32_t nheavy, unsigned long long* __restrict__ out) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < H; j += gridDim.x * blockDim.x) {
    const uint32_t h = info[j].hidx;
    out[j] = h == kNoHub ? 0ull : (static_cast<unsigned long long>(hscr[nheavy + h]) << 32) | hscr[h];
  }
}

// This shard's share of hub j: its alive M entries in row order to send[soff[j]..].  Only the share's own
// slots are read (its unpadded length, offr): a share of at most kLightMax entries is padded to its class
// length, and the padding slots of the M buffer hold no M entries (after a relayout the former adjacency's
// kNone padding, whose bit pattern includes kAlive).
__global__ void k_hub_pack(const HubInfo* __restrict__ info, uint32_t H, const uint64_t* __restrict__ soff,
                           const uint64_t* __restrict__ offp, const uint64_t* __restrict__ offr,
                           const uint32_t* __restrict__ mcol, uint32_t* __restrict__ send) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t j = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; j < H; j += nw) {
    if (soff[j] == ~0ull) continue;
    const uint32_t p = info[j].pos;
    const uint64_t b = offp[p], len = offr[p + 1] - offr[p];
    uint64_t o = soff[j];
    for (uint64_t i0 = 0; i0 < len; i0 += 64) {
      const uint64_t i = i0 + lane;
      const uint32_t m = i < len ? mcol[b + i] : 0u;
      const bool alive = i < len && (m & kAlive);
      const uint64_t bal = __ballot(alive);
      if (alive) send[o + __builtin_popcountll(bal & ((1ull << lane) - 1))] = m;
      o += __builtin_popcountll(bal);
    }
  }
}

struct HubFinishArgs {
  const uint32_t* ctrl;               // hub ordinals this shard controls
  uint32_t nctrl, G, H, P, nranks;
  const unsigned long long* part;     // G x H (count << 32 | TN)
  const uint64_t* roff;               // nctrl x G: where shard g's share of hub ctrl[k] starts in recv
  const uint32_t* recv;
  const HubInfo* info;
  LabelRuns lr;
  PatArgs pa;
  uint16_t* tpub;
  uint16_t* tst;
  uint32_t* mlen;
  uint32_t* malive;
  uint32_t* tcode;
  uint4* srec;                        // superstep-0 records in use: the hub's record beside its slist entry
  uint32_t* mcol;
  uint32_t* slist;
  uint32_t* nS;
  unsigned long long* slot;           // superstep-0 counters
};

// The controller's verify of each hub it controls (global verify_and_update_vertex_state,
// nonunique_ee.hpp:886-977, on the combined TN) and its whole M row in the hub area.
__global__ void k_hub_finish(HubFinishArgs a) {
  __shared__ uint16_t s_adj[16];
  load_adj(s_adj, a.pa);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t k = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; k < a.nctrl; k += nw) {
    const uint32_t j = a.ctrl[k];
    uint32_t TN = 0;
    uint64_t cnt = 0;
    for (uint32_t g = 0; g < a.G; ++g) {
      const unsigned long long x = a.part[uint64_t(g) * a.H + j];
      TN |= static_cast<uint32_t>(x & 0xFFFFu);
      cnt += x >> 32;
    }
    if (!TN) continue;  // no compatible neighbour: never entered S
    const uint32_t p = a.info[j].pos;
    uint32_t tu = 0;
    for (int l = 0; l < a.lr.n; ++l)
      if (p - a.lr.lo[l] < a.lr.len[l]) tu = a.lr.tu[l];
    const uint16_t T = keep_bits(static_cast<uint16_t>(tu), static_cast<uint16_t>(TN), s_adj);
    if (lane == 0) {
      if (!T) {
        atomicAdd(&a.slot[2 * a.P + 2], 1ull);  // removed from S (not_finished)
      } else {
        a.tst[p] = T;
        // with superstep-0 records T_pub travels in the record (k1_finish_row's rule): the position-indexed
        // T_pub is written only for a label on more than two template vertices (gathered by the next
        // superstep), so a hub that superstep removes leaves both T_pub buffers clean
        if (!a.srec || tpub_wide(tu)) a.tpub[p] = T;
        a.mlen[p] = static_cast<uint32_t>(cnt);
        a.malive[p] = static_cast<uint32_t>(cnt);
        const uint32_t ci = code_index(p, a.lr);
        atomicOr(&a.tcode[ci >> 4], tpub_code(T, tu) << ((ci & 15u) << 1));
        const uint32_t at = atomicAdd(a.nS, 1u);
        a.slist[at] = p;
        if (a.srec) a.srec[at] = make_uint4(p, T, kNone, 0u);  // its M in the hub area (m_off), not dense
        const uint32_t r = a.nranks <= 1 ? 0u : j % a.nranks;  // owner rule of a delegate
        atomicAdd(&a.slot[r], 1ull);
        atomicAdd(&a.slot[a.P + r], static_cast<unsigned long long>(cnt));
      }
    }
    if (!T) continue;
    uint32_t* dst = a.mcol + a.info[j].moff;
    for (uint32_t g = 0; g < a.G; ++g) {
      const uint64_t n = a.part[uint64_t(g) * a.H + j] >> 32;
      const uint32_t* src = a.recv + a.roff[uint64_t(k) * a.G + g];
      for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
      dst += n;
    }
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

// words u64 of every shard: d_xcnt[0 .. words) of this shard -> host [g * words + k] (one host sync)
static std::vector<uint64_t> gather_counts(Ctx& c, int words) {
  const uint32_t G = c.nshards;
  c.comm->allgather(c.d_xcnt, c.d_xcnt + 64, words * sizeof(uint64_t), c.stream);
  uint64_t* pin = pinned(c, uint64_t(G) * words);
  PM_HIP_CHECK(hipMemcpyAsync(pin, c.d_xcnt + 64, uint64_t(G) * words * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return std::vector<uint64_t>(pin, pin + uint64_t(G) * words);
}

static void ensure_xcnt(Ctx& c) {
  if (c.nshards > 64) throw std::runtime_error("more than 64 shards");
  if (!c.d_xcnt) PM_HIP_CHECK(hipMalloc(&c.d_xcnt, (64 + 4 * 64) * sizeof(uint64_t)));
}

std::vector<uint64_t> shard_gather_u64(Ctx& c, uint64_t v) {
  if (!c.comm || c.nshards <= 1) return std::vector<uint64_t>(1, v);
  ensure_xcnt(c);
  PM_HIP_CHECK(hipMemcpyAsync(c.d_xcnt, &v, sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  return gather_counts(c, 1);  // (synchronises the stream: v may leave scope)
}

uint64_t shard_agree_min(Ctx& c, uint64_t v) {
  const std::vector<uint64_t> all = shard_gather_u64(c, v);
  return *std::min_element(all.begin(), all.end());
}


void shard_hub_combine(Ctx& c, uint64_t* d_slot) {
  if (!c.comm || !c.split_hubs) return;
  const uint32_t G = c.nshards, me = c.shard;
  const uint32_t H = static_cast<uint32_t>(c.hubinfo.size());
  auto* part = reinterpret_cast<unsigned long long*>(c.d_hubpart);
  hipLaunchKernelGGL(k_hub_partials, dim3(xgrid(H)), dim3(kXBlock), 0, c.stream, c.d_hubinfo, H, c.d_hscr, c.nheavy,
                     part);
  c.comm->allgather(part, part + H, uint64_t(H) * sizeof(uint64_t), c.stream);
  uint64_t* pin = pinned(c, uint64_t(G) * H);
  PM_HIP_CHECK(hipMemcpyAsync(pin, part + H, uint64_t(G) * H * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  const std::vector<uint64_t> all(pin, pin + uint64_t(G) * H);
  auto cnt = [&](uint32_t g, uint32_t j) { return all[uint64_t(g) * H + j] >> 32; };
  // send: this shard's shares grouped by controller, hubs in order; receive: the shares of the hubs this
  // shard controls, shard by shard
  std::vector<uint64_t> soff(H, ~0ull), sb(G, 0), rb(G, 0), roff;
  std::vector<uint32_t> ctrl;
  uint64_t so = 0;
  for (uint32_t g = 0; g < G; ++g)
    for (uint32_t j = g; j < H; j += G)
      if (cnt(me, j)) {
        soff[j] = so;
        so += cnt(me, j);
        sb[g] += cnt(me, j) * sizeof(uint32_t);
      }
  for (uint32_t j = me; j < H; j += G) ctrl.push_back(j);
  roff.assign(ctrl.size() * G, 0);
  uint64_t ro = 0;
  for (uint32_t g = 0; g < G; ++g)
    for (size_t k = 0; k < ctrl.size(); ++k) {
      roff[k * G + g] = ro;
      ro += cnt(g, ctrl[k]);
      rb[g] += cnt(g, ctrl[k]) * sizeof(uint32_t);
    }
  c.arena.reset();
  auto* d_soff = static_cast<uint64_t*>(c.arena.get(std::max<size_t>(H, 1) * sizeof(uint64_t)));
  auto* d_roff = static_cast<uint64_t*>(c.arena.get(std::max<size_t>(roff.size(), 1) * sizeof(uint64_t)));
  auto* d_ctrl = static_cast<uint32_t*>(c.arena.get(std::max<size_t>(ctrl.size(), 1) * sizeof(uint32_t)));
  PM_HIP_CHECK(hipMemcpyAsync(d_soff, soff.data(), H * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  if (!roff.empty())
    PM_HIP_CHECK(hipMemcpyAsync(d_roff, roff.data(), roff.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  if (!ctrl.empty())
    PM_HIP_CHECK(hipMemcpyAsync(d_ctrl, ctrl.data(), ctrl.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  auto* send = grow<uint32_t>(c.d_xsend, c.xsend_cap, std::max<uint64_t>(so, 1) * sizeof(uint32_t));
  auto* recv = grow<uint32_t>(c.d_xrecv, c.xrecv_cap, std::max<uint64_t>(ro, 1) * sizeof(uint32_t));
  if (so)
    hipLaunchKernelGGL(k_hub_pack, dim3(xgrid(uint64_t(H) * 64)), dim3(kXBlock), 0, c.stream, c.d_hubinfo, H, d_soff,
                       c.d_offp, c.d_offr, c.d_mcol, send);
  debug_point(c, "delegate pack");
  c.comm->alltoallv(send, sb.data(), recv, rb.data(), c.stream);
  HubFinishArgs a{};
  a.ctrl = d_ctrl;
  a.nctrl = static_cast<uint32_t>(ctrl.size());
  a.G = G;
  a.H = H;
  a.nranks = c.nranks;
  a.P = c.nranks <= 1 ? 1 : c.nranks;
  a.part = part + H;
  a.roff = d_roff;
  a.recv = recv;
  a.info = c.d_hubinfo;
  a.lr = c.lr;
  a.pa = c.pa;
  a.tpub = c.d_tpub[c.cur];
  a.tst = c.d_tst;
  a.mlen = c.d_mlen;
  a.malive = c.d_malive;
  a.tcode = c.d_tcode;
  a.srec = c.k1_records ? c.d_srec : nullptr;
  a.mcol = c.d_mcol;
  a.slist = c.d_slist;
  a.nS = c.d_nS;
  a.slot = reinterpret_cast<unsigned long long*>(d_slot);
  if (a.nctrl)
    hipLaunchKernelGGL(k_hub_finish, dim3(xgrid(uint64_t(a.nctrl) * 64)), dim3(kXBlock), 0, c.stream, a);
  PM_HIP_CHECK(hipGetLastError());
  c.nS_host += a.nctrl;  // (an upper bound until the code exchange reads the count)
}

void shard_codes_after_first(Ctx& c) {
  if (!c.comm || c.replicated) return;
  if (!c.xcode_wide) {
    // a position's 2-bit code is set only by the shard that holds its row (a delegate's by its controller):
    // the shards' code arrays have disjoint fields, and their word-wise sum is their union -- one all-reduce
    // of the code words (22 MB at S=28) instead of packing, gathering and unpacking every survivor's record.
    // Writers of tcode: superstep 0's finish paths for the rows a shard holds (a split delegate's share skips
    // them) and k_hub_finish on the controller only.  PM_DEBUG_SYNC=1 checks the invariant: the nonzero
    // 2-bit fields of the sum must number the shards' own (a field set by two shards carries into its
    // neighbour or merges two codes, and both show as fewer fields).
    static const bool check = std::getenv("PM_DEBUG_SYNC") != nullptr;
    const size_t words = tcode_words(c.lr);
    auto fields = [&]() {
      std::vector<uint32_t> h(words);
      if (words) PM_HIP_CHECK(hipMemcpyAsync(h.data(), c.d_tcode, words * 4, hipMemcpyDeviceToHost, c.stream));
      PM_HIP_CHECK(hipStreamSynchronize(c.stream));
      uint64_t k = 0;
      for (uint32_t x : h) k += __builtin_popcount((x | (x >> 1)) & 0x55555555u);
      return k;
    };
    const uint64_t own = check ? fields() : 0;
    c.comm->allreduce_sum_u32(c.d_tcode, words, c.stream);
    if (check) {
      const std::vector<uint64_t> all = shard_gather_u64(c, own);
      uint64_t sum = 0;
      for (uint64_t x : all) sum += x;
      const uint64_t got = fields();
      if (got != sum)
        throw std::runtime_error("superstep-0 code exchange: " + std::to_string(sum) + " code fields set over the "
                                 "shards but " + std::to_string(got) + " in their sum (two shards wrote one field)");
    }
    c.xcode_n.clear();
    c.xcode_in_tpub = false;
    return;
  }
  ensure_xcnt(c);
  const uint32_t G = c.nshards;
  hipLaunchKernelGGL(k_count_to_u64, dim3(1), dim3(1), 0, c.stream, c.d_nS, c.d_xcnt);
  const std::vector<uint64_t> n = gather_counts(c, 1);
  uint64_t maxS = 1;
  for (uint32_t g = 0; g < G; ++g) maxS = std::max(maxS, n[g]);
  c.nS_host = static_cast<uint32_t>(n[c.shard]);
  c.xcode_n = n;
  c.xcode_max = maxS;
  const size_t rb = c.xcode_wide ? 8 : 4;
  auto* send = grow<char>(c.d_xsend, c.xsend_cap, maxS * rb);
  auto* recv = grow<char>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * maxS * rb);
  hipLaunchKernelGGL(k_pack_codes, dim3(xgrid(c.nS_host)), dim3(kXBlock), 0, c.stream, c.d_slist, c.d_nS, c.d_tcode,
                     c.d_tpub[c.cur], c.k1_records ? c.d_srec : nullptr, c.xcode_wide ? 1 : 0, c.lr,
                     reinterpret_cast<uint32_t*>(send), reinterpret_cast<unsigned long long*>(send));
  debug_point(c, "code pack");
  c.comm->allgather(send, recv, maxS * rb, c.stream);
  XCounts x{};
  for (uint32_t g = 0; g < G; ++g) x.n[g] = n[g];
  hipLaunchKernelGGL(k_unpack_codes, dim3(xgrid(uint64_t(G) * maxS)), dim3(kXBlock), 0, c.stream,
                     c.xcode_wide ? nullptr : reinterpret_cast<const uint32_t*>(recv),
                     c.xcode_wide ? reinterpret_cast<const unsigned long long*>(recv) : nullptr, maxS, G, c.shard, x,
                     c.lr, c.d_tcode, c.d_tpub[c.cur]);
  c.xcode_in_tpub = c.xcode_wide;
  PM_HIP_CHECK(hipGetLastError());
}

// After the first later superstep, when the state is replicated only after the second (Ctx::handoff_ss): the
// second superstep pulls T_pub of its rows' M entries, which live on every shard.  Each shard's rows of S
// (its compacted slist) go out as {position, T_pub} records; the other shards' records land in the T_pub
// buffer that superstep reads, and are cleared from it after the superstep (shard_replicate, the code-clear
// path) so that T_pub stays zero outside the replica's rows.  At S=28: 0.80 M records, 6.4 MB over the shards.
__global__ void k_pack_tpub(const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp,
                            const uint16_t* __restrict__ tpub, unsigned long long* __restrict__ out) {
  const uint64_t n = *nSp;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = slist[i];
    out[i] = p | (static_cast<unsigned long long>(tpub[p]) << 32);
  }
}

__global__ void k_unpack_tpub(const unsigned long long* __restrict__ in, uint64_t maxS, uint32_t G, uint32_t me,
                              XCounts x, uint16_t* __restrict__ tpub) {
  const uint64_t total = uint64_t(G) * maxS;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / maxS);
    if (g == me || j % maxS >= x.n[g]) continue;
    const unsigned long long r = in[j];
    tpub[static_cast<uint32_t>(r & 0x3FFFFFFFull)] = static_cast<uint16_t>(r >> 32);
  }
}

void shard_tpub_exchange(Ctx& c) {
  if (!c.comm || c.replicated) return;
  ensure_xcnt(c);
  const uint32_t G = c.nshards;
  XCounts x{};
  // u64 code mode: the other shards' superstep-0 T_pub in the buffer the first later superstep read (the
  // second superstep writes into it)
  if (c.xcode_in_tpub && !c.xcode_n.empty()) {
    for (uint32_t g = 0; g < G; ++g) x.n[g] = c.xcode_n[g];
    hipLaunchKernelGGL(k_clear_codes, dim3(xgrid(uint64_t(G) * c.xcode_max)), dim3(kXBlock), 0, c.stream,
                       reinterpret_cast<const unsigned long long*>(c.d_xrecv), c.xcode_max, G, c.shard, x,
                       c.d_tpub[c.cur ^ 1]);
  }
  c.xcode_n.clear();
  c.xcode_in_tpub = false;
  hipLaunchKernelGGL(k_count_to_u64, dim3(1), dim3(1), 0, c.stream, c.d_nS, c.d_xcnt);
  const std::vector<uint64_t> n = gather_counts(c, 1);
  uint64_t maxS = 1;
  for (uint32_t g = 0; g < G; ++g) maxS = std::max(maxS, n[g]);
  c.nS_host = static_cast<uint32_t>(n[c.shard]);
  auto* send = grow<unsigned long long>(c.d_xsend, c.xsend_cap, maxS * 8);
  auto* recv = grow<unsigned long long>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * maxS * 8);
  hipLaunchKernelGGL(k_pack_tpub, dim3(xgrid(c.nS_host)), dim3(kXBlock), 0, c.stream, c.d_slist, c.d_nS,
                     c.d_tpub[c.cur], send);
  c.comm->allgather(send, recv, maxS * 8, c.stream);
  for (uint32_t g = 0; g < G; ++g) x.n[g] = n[g];
  hipLaunchKernelGGL(k_unpack_tpub, dim3(xgrid(uint64_t(G) * maxS)), dim3(kXBlock), 0, c.stream, recv, maxS, G,
                     c.shard, x, c.d_tpub[c.cur]);
  PM_HIP_CHECK(hipGetLastError());
  // the records stay in d_xrecv: shard_replicate clears their positions from the second superstep's input
  c.xcode_n = n;
  c.xcode_max = maxS;
  c.xcode_in_tpub = true;
}

void pack_state(Ctx& c, uint32_t* rec, uint32_t* ent, uint64_t ent_cap, uint64_t* counts);

// The replica's hub rows in neighbour-id order.  A delegate's M row was assembled at its controller share by
// share (the entries of targets owned by shard 0, then shard 1, ...: each share in id order), but every M row
// is searched by neighbour id -- the push-form receivers flag M[u][v] (k_lcc_push_verify), a cycle terminal
// flags M[s][p] (nem_1.hpp:764-770) -- so the rows of the hubs in the replica are sorted once (segmented radix
// sort by neighbour id) when the replica is built.
__global__ void k_hub_rows(const HubInfo* __restrict__ info, uint32_t H, const uint16_t* __restrict__ tpub,
                           const uint64_t* __restrict__ rmoff, const uint32_t* __restrict__ mlen,
                           unsigned long long* __restrict__ out) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < H; j += gridDim.x * blockDim.x) {
    const uint32_t p = info[j].pos;
    out[2 * j] = tpub[p] ? rmoff[p] : 0ull;
    out[2 * j + 1] = tpub[p] ? mlen[p] : 0ull;
  }
}

__global__ void k_hub_gather(const uint64_t* __restrict__ seg, const uint64_t* __restrict__ src, uint32_t nseg,
                             const uint32_t* __restrict__ rmcol, const uint32_t* __restrict__ perm, uint64_t nv,
                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, bool back,
                             uint32_t* __restrict__ rmcol_out, unsigned long long* __restrict__ bad) {
  // segment k: entries [seg[k], seg[k + 1]) of the temporary arrays <-> rmcol[src[k] ..]
  const int lane = threadIdx.x & 63;
  for (uint32_t k = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; k < nseg; k += gridDim.x * (blockDim.x / 64)) {
    const uint64_t b = seg[k], n = seg[k + 1] - b, r = src[k];
    for (uint64_t i = lane; i < n; i += 64) {
      if (back) {
        rmcol_out[r + i] = vals[b + i];
      } else {
        const uint32_t m = rmcol[r + i];
        const uint32_t p = m & kPosMask;
        if (p >= nv) {  // (not an M entry: reported, the key kept in range)
          atomicCAS(bad, 0ull, (static_cast<unsigned long long>(k) << 32) | static_cast<uint32_t>(i));
          keys[b + i] = 0;
        } else {
          keys[b + i] = perm[p];
        }
        vals[b + i] = m;
      }
    }
  }
}

static void sort_hub_rows(Ctx& c) {
  const uint32_t H = static_cast<uint32_t>(c.hubinfo.size());
  if (!H || !c.d_hubinfo) return;
  auto* d_rows = static_cast<unsigned long long*>(c.arena.get(2 * size_t(H) * sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_hub_rows, dim3(xgrid(H)), dim3(kXBlock), 0, c.stream, c.d_hubinfo, H, c.d_tpub[c.cur],
                     c.d_rmoff, c.d_mlen, d_rows);
  std::vector<unsigned long long> rows(2 * size_t(H));
  PM_HIP_CHECK(hipMemcpyAsync(rows.data(), d_rows, rows.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                              c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  if (std::getenv("PM_DEBUG_HUB_ROWS")) {  // diagnostics: the hubs with T_pub are the replica's rows, once each
    std::vector<uint32_t> sl(c.nS_host);
    if (c.nS_host) PM_HIP_CHECK(hipMemcpy(sl.data(), c.d_slist, sl.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> cntp(c.n, 0);
    for (uint32_t p : sl) ++cntp[p];
    for (uint32_t j = 0; j < H; ++j) {
      const uint32_t p = c.hubinfo[j].pos;
      if ((rows[2 * j + 1] || rows[2 * j]) && cntp[p] != 1)
        std::fprintf(stderr, "[pm dbg] shard %u: hub %u (position %u, id %u) with T_pub in the replica %u times, "
                     "row [%llu, +%llu)\n", c.shard, j, p, c.perm_host[p], cntp[p], rows[2 * j], rows[2 * j + 1]);
    }
    for (size_t i = 0; i < sl.size(); ++i)
      if (cntp[sl[i]] > 1) std::fprintf(stderr, "[pm dbg] shard %u: replica row %zu: position %u (id %u) twice\n",
                                        c.shard, i, sl[i], c.perm_host[sl[i]]);
  }
  std::vector<uint64_t> seg(1, 0), src;
  for (uint32_t j = 0; j < H; ++j)
    if (rows[2 * j + 1] > 1) {
      src.push_back(rows[2 * j]);
      seg.push_back(seg.back() + rows[2 * j + 1]);
    }
  const uint32_t ns = static_cast<uint32_t>(src.size());
  const uint64_t total = seg.back();
  if (!ns) return;
  for (uint32_t k = 0; k < ns; ++k)  // every hub row of the replica lies inside its entries
    if (src[k] + (seg[k + 1] - seg[k]) > c.replica_entries)
      throw std::runtime_error("internal: replica row of a delegate [" + std::to_string(src[k]) + ", +" +
                               std::to_string(seg[k + 1] - seg[k]) + ") outside the replica's " +
                               std::to_string(c.replica_entries) + " entries (shard " + std::to_string(c.shard) + ")");
  auto* d_seg = static_cast<uint64_t*>(c.arena.get(seg.size() * sizeof(uint64_t)));
  auto* d_src = static_cast<uint64_t*>(c.arena.get(src.size() * sizeof(uint64_t)));
  auto* k0 = static_cast<uint32_t*>(c.arena.get(total * 4));
  auto* k1 = static_cast<uint32_t*>(c.arena.get(total * 4));
  auto* v0 = static_cast<uint32_t*>(c.arena.get(total * 4));
  auto* v1 = static_cast<uint32_t*>(c.arena.get(total * 4));
  PM_HIP_CHECK(hipMemcpyAsync(d_seg, seg.data(), seg.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  PM_HIP_CHECK(hipMemcpyAsync(d_src, src.data(), src.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  const unsigned g = static_cast<unsigned>(std::min<uint64_t>(ns, 4096) + 3) / 4;
  auto* d_bad = static_cast<unsigned long long*>(c.arena.get(sizeof(unsigned long long)));
  PM_HIP_CHECK(hipMemsetAsync(d_bad, 0, sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_hub_gather, dim3(g), dim3(kXBlock), 0, c.stream, d_seg, d_src, ns, c.d_rmcol, c.d_perm, c.n,
                     k0, v0, false, c.d_rmcol, d_bad);
  unsigned long long bad = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  if (bad)
    throw std::runtime_error("internal: replica row of a delegate (segment " + std::to_string(bad >> 32) +
                             ", entry " + std::to_string(bad & 0xFFFFFFFFull) + ") holds a non-position (shard " +
                             std::to_string(c.shard) + ")");
  size_t tmp = 0;
  PM_HIP_CHECK(rocprim::segmented_radix_sort_pairs(nullptr, tmp, k0, k1, v0, v1, size_t(total), ns, d_seg, d_seg + 1,
                                                   0, 32, c.stream));
  void* d_tmp = c.arena.get(std::max<size_t>(tmp, 1));
  PM_HIP_CHECK(rocprim::segmented_radix_sort_pairs(d_tmp, tmp, k0, k1, v0, v1, size_t(total), ns, d_seg, d_seg + 1,
                                                   0, 32, c.stream));
  hipLaunchKernelGGL(k_hub_gather, dim3(g), dim3(kXBlock), 0, c.stream, d_seg, d_src, ns,
                     static_cast<const uint32_t*>(nullptr), c.d_perm, c.n, k1, v1, true, c.d_rmcol, d_bad);
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));  // (seg / src live on the host stack)
}

uint64_t pack_state_entry_bound(Ctx& c) {
  // the exact count: pass 1 + scans, then one read-back (the caller sizes its buffer)
  ensure_xcnt(c);
  pack_state(c, nullptr, nullptr, 0, c.d_xcnt);
  uint64_t* pin = pinned(c, 2);
  PM_HIP_CHECK(hipMemcpyAsync(pin, c.d_xcnt, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return pin[1];
}

void pack_state(Ctx& c, uint32_t* rec, uint32_t* ent, uint64_t ent_cap, uint64_t* counts) {
  const uint64_t cap = c.nS_host;
  // (the state right after superstep 0 is never packed: with dense M the first later superstep follows)
  if (c.k1_dense) throw std::runtime_error("internal: pack_state of a dense superstep-0 state");
  ensure_xcnt(c);
  c.arena.reset();
  auto* keep = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(cap, 1) * sizeof(uint32_t)));
  auto* cnt = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(cap, 1) * sizeof(uint32_t)));
  auto* ridx = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(cap, 1) * sizeof(uint32_t)));
  auto* eoff = static_cast<uint64_t*>(c.arena.get(std::max<uint64_t>(cap, 1) * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(uint64_t), c.stream));  // rows, entries, error word
  if (!cap) return;
  hipLaunchKernelGGL(k_pack_count, dim3(xgrid(cap)), dim3(kXBlock), 0, c.stream, c.d_slist, c.d_nS, cap,
                     c.d_tpub[c.cur], c.d_malive, keep, cnt);
  size_t t1 = 0, t2 = 0;
  PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, t1, keep, ridx, 0u, size_t(cap), rocprim::plus<uint32_t>(), c.stream));
  rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> wc(cnt, Widen());
  PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, t2, wc, eoff, uint64_t(0), size_t(cap), rocprim::plus<uint64_t>(),
                                       c.stream));
  void* tmp = c.arena.get(std::max(t1, t2));
  PM_HIP_CHECK(rocprim::exclusive_scan(tmp, t1, keep, ridx, 0u, size_t(cap), rocprim::plus<uint32_t>(), c.stream));
  PM_HIP_CHECK(rocprim::exclusive_scan(tmp, t2, wc, eoff, uint64_t(0), size_t(cap), rocprim::plus<uint64_t>(),
                                       c.stream));
  // rec == nullptr: totals only (the rows are not written); counts[2]: a row the pack found inconsistent
  // (shard_replicate gathers it with the counts: a wrong row would corrupt every replica)
  hipLaunchKernelGGL(k_pack_write, dim3(xgrid(cap)), dim3(kXBlock), 0, c.stream, c.d_slist, c.d_nS, cap, keep,
                     ridx, cnt, eoff, c.d_tpub[c.cur], c.d_tst, c.d_mlen, m_off(c), m_col(c), rec, ent,
                     rec ? ent_cap : 0, c.n, reinterpret_cast<unsigned long long*>(counts),
                     reinterpret_cast<unsigned long long*>(counts + 2));
  PM_HIP_CHECK(hipGetLastError());
}

void shard_replicate(Ctx& c) {
  if (!c.comm || c.replicated) return;
  ensure_xcnt(c);
  const uint32_t G = c.nshards;
  XCounts x{};
  // u64 code mode: the other shards' T_pub that superstep 0's buffer received (the superstep that
  // read it is done; the buffer becomes the next superstep's output)
  if (c.xcode_in_tpub && !c.xcode_n.empty()) {
    for (uint32_t g = 0; g < G; ++g) x.n[g] = c.xcode_n[g];
    hipLaunchKernelGGL(k_clear_codes, dim3(xgrid(uint64_t(G) * c.xcode_max)), dim3(kXBlock), 0, c.stream,
                       reinterpret_cast<const unsigned long long*>(c.d_xrecv), c.xcode_max, G, c.shard, x,
                       c.d_tpub[c.cur ^ 1]);
  }
  c.xcode_n.clear();
  debug_point(c, "replica: code clear");
  // this shard's rows of S, packed once into the send buffers as they stand (grown to the largest shard's
  // block by the previous search), and one gather of every shard's counts and pack error word (one host
  // sync); a shard whose buffers are smaller than the largest block -- the all-gathers read that much from
  // every shard -- grows them and packs again
  auto* rsend = grow<uint32_t>(c.d_xsend, c.xsend_cap, std::max<uint64_t>(c.nS_host, 1) * 16);
  auto* esend = grow<uint32_t>(c.d_xent_send, c.xent_send_cap, std::max<size_t>(c.xent_send_cap, size_t(1) << 18));
  pack_state(c, rsend, esend, c.xent_send_cap / 4, c.d_xcnt);
  const std::vector<uint64_t> cn = gather_counts(c, 3);
  for (uint32_t g = 0; g < G; ++g)
    if (const uint64_t e = cn[3 * g + 2])
      throw std::runtime_error("internal: state row of position " + std::to_string(e & 0x3FFFFFFFull) + " on shard " +
                               std::to_string(g) + ((e >> 63) ? " holds a non-position entry" :
                                                                " has |M| != its alive entries"));
  uint64_t maxR = 1, maxE = 1, rows = 0, ents = 0;
  for (uint32_t g = 0; g < G; ++g) {
    x.n[g] = cn[3 * g];
    x.m[g] = cn[3 * g + 1];
    x.base[g] = rows;
    x.ebase[g] = ents;
    rows += x.n[g];
    ents += x.m[g];
    maxR = std::max(maxR, x.n[g]);
    maxE = std::max(maxE, x.m[g]);
  }
  if (x.m[c.shard] >= (1ull << 32)) throw std::runtime_error("replica: more than 2^32 M entries on one shard");
  if (rows > c.n) throw std::runtime_error("internal: replica larger than the vertex set");
  // every shard's send block is read up to the largest count
  if (c.xsend_cap < maxR * 16 || c.xent_send_cap < maxE * 4) {
    rsend = grow<uint32_t>(c.d_xsend, c.xsend_cap, maxR * 16);
    esend = grow<uint32_t>(c.d_xent_send, c.xent_send_cap, maxE * 4);
    pack_state(c, rsend, esend, c.xent_send_cap / 4, c.d_xcnt);
  }
  auto* rrecv = grow<uint32_t>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * maxR * 16);
  auto* erecv = grow<uint32_t>(c.d_xent_recv, c.xent_recv_cap, uint64_t(G) * maxE * 4);
  c.comm->allgather(rsend, rrecv, maxR * 16, c.stream);
  c.comm->allgather(esend, erecv, maxE * 4, c.stream);
  // the replica's slist replaces this shard's: both T_pub buffers are cleared at this shard's entries first
  // (rows the last superstep removed may hold an old T_pub -- a code-3 row of superstep 0 when no compaction
  // ran, diameter 2 -- and would be outside every later clear); the rows of S get theirs back from the gather
  debug_point(c, "replica: pack + gather");
  launch_clear_tpub(c);
  debug_point(c, "replica: own T_pub clear");
  if (!c.d_rmoff) PM_HIP_CHECK(hipMalloc(&c.d_rmoff, std::max<uint64_t>(c.n, 1) * sizeof(uint64_t)));
  if (c.rmcap < ents + 1 || !c.d_rmcol) {
    if (c.d_rmcol) (void)hipFree(c.d_rmcol);
    c.rmcap = std::max<uint64_t>(ents + ents / 4, 1 << 16);
    PM_HIP_CHECK(hipMalloc(&c.d_rmcol, c.rmcap * sizeof(uint32_t)));
  }
  hipLaunchKernelGGL(k_unpack_rows, dim3(xgrid(uint64_t(G) * maxR)), dim3(kXBlock), 0, c.stream, rrecv, maxR, G, x,
                     c.d_slist, c.d_tpub[c.cur], c.d_tst, c.d_mlen, c.d_malive, c.d_rmoff);
  hipLaunchKernelGGL(k_unpack_entries, dim3(xgrid(uint64_t(G) * maxE)), dim3(kXBlock), 0, c.stream, erecv, maxE, G, x,
                     c.d_rmcol);
  const uint32_t nrows = static_cast<uint32_t>(rows);
  PM_HIP_CHECK(hipMemcpyAsync(c.d_nS, &nrows, sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  PM_HIP_CHECK(hipGetLastError());
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));  // (nrows lives on the host stack)
  c.nS_host = nrows;
  c.replica_rows = rows;
  c.replica_entries = ents;
  c.slist_compacted = true;
  c.smask_valid = false;
  c.k1_dense = false;
  c.replicated = true;
  if (c.split_hubs && !std::getenv("PM_DEBUG_NO_HUB_SORT")) {
    c.arena.reset();
    sort_hub_rows(c);
  }
}

// ---------------------------------------------------------------------------
// Split NLC lines (sharded replica).  A line with many sources runs split by owner: each shard passes the
// tokens of the sources it owns (the reference's visitors of a source live on its owner rank and its tokens
// travel to the owners of the walk's vertices, nem_1.hpp:832-851 / tds_batch_1.hpp:1181; here every shard
// reads the whole replica, so tokens need no exchange).  The line's effects are then combined: the sources
// whose T_pub bit I[0] this shard's post-processing cleared (beta.cpp:956-1000) and the M entries its cycle
// terminals flagged (nem_1.hpp:764-770) are all-gathered and applied to every replica.

// Post-processing of a split line over this shard's own sources (line_post's rule); out: [0] acked,
// [1] deleted, [2] cleared sources (their positions in dels), [3, 3 + 2P) vertices | edges per rank leaving S.
__global__ void k_split_post(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint8_t* __restrict__ tsm,
                             uint16_t* __restrict__ tpub, int i0, const uint32_t* __restrict__ malive, OwnerArgs oa,
                             unsigned long long* __restrict__ dels, unsigned long long* __restrict__ out) {
  const uint32_t P = oa.nranks <= 1 ? 1 : oa.nranks;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    if (tsm[s] == 2) {
      atomicAdd(&out[0], 1ull);
      continue;
    }
    uint16_t T = tpub[s];
    if (!T) continue;
    atomicAdd(&out[1], 1ull);
    if (!((T >> i0) & 1u)) continue;
    T &= static_cast<uint16_t>(~(1u << i0));
    tpub[s] = T;
    dels[atomicAdd(&out[2], 1ull)] = s;
    if (!T) {  // vertex_active = false, erased from the state map
      const uint32_t r = owner_of(s, oa);
      atomicAdd(&out[3 + r], 1ull);
      atomicAdd(&out[3 + P + r], static_cast<unsigned long long>(malive[s]));
    }
  }
}

// The other shards' effects on this replica: lists of block g at g * stride (nf[g] flagged entries, then nd[g]
// cleared sources from offset fmax).
__global__ void k_split_apply(const unsigned long long* __restrict__ all, uint64_t stride, uint64_t fmax, uint32_t G,
                              uint32_t me, XCounts x, uint16_t* __restrict__ tpub, int i0, uint32_t* __restrict__ mcol) {
  const uint64_t total = uint64_t(G) * stride;
  for (uint64_t j = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; j < total; j += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t g = static_cast<uint32_t>(j / stride);
    const uint64_t k = j % stride;
    if (g == me) continue;
    if (k < fmax) {
      if (k < x.n[g]) atomicOr(&mcol[all[j]], kFlag);
    } else if (k - fmax < x.m[g]) {
      const uint32_t p = static_cast<uint32_t>(all[j]);
      tpub[p] &= static_cast<uint16_t>(~(1u << i0));
    }
  }
}

// Host vector of every shard (G x v.size(), shard order): one all-gather, one host sync.
static std::vector<uint64_t> shard_allgather_host(Ctx& c, const std::vector<uint64_t>& v) {
  const uint32_t G = c.nshards;
  auto* d = grow<uint64_t>(c.d_xsend, c.xsend_cap, v.size() * sizeof(uint64_t));
  auto* r = grow<uint64_t>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * v.size() * sizeof(uint64_t));
  PM_HIP_CHECK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  c.comm->allgather(d, r, v.size() * sizeof(uint64_t), c.stream);
  std::vector<uint64_t> out(uint64_t(G) * v.size());
  PM_HIP_CHECK(hipMemcpyAsync(out.data(), r, out.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return out;
}

bool split_line_finish(Ctx& c, size_t pl, const LineStats& st, const uint32_t* kept_dev, bool want_walks,
                       FusedLineOut& out) {
  if (!c.comm) throw std::runtime_error("internal: split NLC line without a communicator");
  const uint32_t G = c.nshards, P = c.nranks <= 1 ? 1 : c.nranks;
  const NlcLine& line = c.pattern.lines[pl];
  const uint32_t stride = out.stride;
  // 1. overflow anywhere: every shard reruns the line on the exact path (no post-processing ran yet; the
  //    flags a finished shard set are among those the rerun sets everywhere)
  const unsigned long long nflag = c.h_pin_lines[3];  // the flag-list counter (control words 6-7 of the launch)
  const std::vector<uint64_t> a =
      shard_allgather_host(c, {st.overflow ? 1ull : 0ull, nflag, st.nsrc, st.trav, st.tokens, st.walks});
  for (uint32_t g = 0; g < G; ++g)
    if (a[6 * g]) return false;
  // 2. this shard's post-processing
  unsigned long long* dels = c.d_xsplit + m_cap(c);
  ensure_xcnt(c);
  auto* d_out = reinterpret_cast<unsigned long long*>(c.d_xcnt);  // 3 + 2P <= 64 + 4 * 64 words
  PM_HIP_CHECK(hipMemsetAsync(d_out, 0, (3 + 2 * P) * sizeof(uint64_t), c.stream));
  OwnerArgs oa{c.d_hubs, c.d_perm, static_cast<uint32_t>(c.hubs_host.size()), c.nranks};
  const int i0 = static_cast<int>(line.indices[0]);
  if (st.nsrc)
    hipLaunchKernelGGL(k_split_post, dim3(xgrid(st.nsrc)), dim3(kXBlock), 0, c.stream, c.d_sources, uint64_t(st.nsrc),
                       c.d_tsm, c.d_tpub[c.cur], i0, c.d_malive, oa, dels, d_out);
  PM_HIP_CHECK(hipGetLastError());
  std::vector<uint64_t> loc(3 + 2 * P);
  PM_HIP_CHECK(hipMemcpyAsync(loc.data(), d_out, loc.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  // 3. every shard's post counts; then the lists, padded to the largest (flags | cleared sources)
  const std::vector<uint64_t> b = shard_allgather_host(c, loc);
  const size_t W = loc.size();
  uint64_t fmax = 0, dmax = 0;
  XCounts x{};
  out.rm_v.assign(c.nranks, 0);
  out.rm_e.assign(c.nranks, 0);
  uint64_t acked = 0, deleted = 0;
  for (uint32_t g = 0; g < G; ++g) {
    x.n[g] = a[6 * g + 1];
    x.m[g] = b[W * g + 2];
    fmax = std::max(fmax, x.n[g]);
    dmax = std::max(dmax, x.m[g]);
    acked += b[W * g];
    deleted += b[W * g + 1];
    for (uint32_t r = 0; r < c.nranks; ++r) {
      out.rm_v[r] += b[W * g + 3 + r];
      out.rm_e[r] += b[W * g + 3 + P + r];
    }
    out.tr.sources += a[6 * g + 2];
    out.tr.edges += a[6 * g + 3];
    out.tr.tokens += a[6 * g + 4];
    out.tr.walks += a[6 * g + 5];
  }
  out.tr.acked = acked;
  out.deleted = deleted ? 1u : 0u;
  out.split = true;
  const uint64_t xs = fmax + dmax;
  if (xs) {
    auto* send = grow<unsigned long long>(c.d_xsend, c.xsend_cap, xs * 8);
    auto* recv = grow<unsigned long long>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * xs * 8);
    if (nflag) PM_HIP_CHECK(hipMemcpyAsync(send, c.d_xsplit, nflag * 8, hipMemcpyDeviceToDevice, c.stream));
    if (loc[2]) PM_HIP_CHECK(hipMemcpyAsync(send + fmax, dels, loc[2] * 8, hipMemcpyDeviceToDevice, c.stream));
    c.comm->allgather(send, recv, xs * 8, c.stream);
    hipLaunchKernelGGL(k_split_apply, dim3(xgrid(uint64_t(G) * xs)), dim3(kXBlock), 0, c.stream, recv, xs, fmax, G,
                       c.shard, x, c.d_tpub[c.cur], i0, m_col(c));
    PM_HIP_CHECK(hipGetLastError());
  }
  // 4. the kept walks of every shard (shard order), for the result files
  if (want_walks && pl >= 4) {
    uint64_t wmax = 0;
    for (uint32_t g = 0; g < G; ++g) wmax = std::max<uint64_t>(wmax, a[6 * g + 5] * stride);
    if (wmax) {
      auto* send = grow<uint32_t>(c.d_xsend, c.xsend_cap, wmax * 4);
      auto* recv = grow<uint32_t>(c.d_xrecv, c.xrecv_cap, uint64_t(G) * wmax * 4);
      if (st.walks)
        PM_HIP_CHECK(hipMemcpyAsync(send, kept_dev + st.wbase[0], st.walks * stride * 4, hipMemcpyDeviceToDevice,
                                    c.stream));
      c.comm->allgather(send, recv, wmax * 4, c.stream);
      std::vector<uint32_t> all(uint64_t(G) * wmax);
      PM_HIP_CHECK(hipMemcpyAsync(all.data(), recv, all.size() * 4, hipMemcpyDeviceToHost, c.stream));
      PM_HIP_CHECK(hipStreamSynchronize(c.stream));
      for (uint32_t g = 0; g < G; ++g)
        out.walks.insert(out.walks.end(), all.begin() + g * wmax, all.begin() + g * wmax + a[6 * g + 5] * stride);
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// Local split lines (one context).  A path / cycle line whose (source, vertex) pairs outgrow the largest table
// (2^31 slots, or no device room) ran on the exact per-position path at ~18 G edges/s (C5 with 64 letters at S=27,
// DESIGN.md §4.6).  Here the fused kernel runs the line over its sources in parts instead -- the split lines'
// owner rule with `parts` parts on one context, each part's post-processing deferred -- and the post-processing
// runs once after every part (line_post's rule over all the line's sources, k_split_post): no part's tokens see
// another part's cleared bits, as in the unsplit line.  Terminal effects (acknowledgements in the token-source
// map, cycle flags on M) are set in place; a part that overflows leaves none, so the line restarts with four times
// the parts (what the earlier parts set, the restart sets again).
bool local_split_line(Ctx& c, size_t pl, bool want_walks, FusedLineOut& out) {
  if (c.comm) return false;
  // (PM_TDS_CAP, tests: a TDS line that overflows the bounded walk storage takes the exact path's chunked
  // enumeration, which those tests exercise)
  if (pl >= 4 && std::getenv("PM_TDS_CAP")) return false;
  const NlcLine& line = c.pattern.lines[pl];
  const uint32_t stride = static_cast<uint32_t>(line.cycle_length + 2);
  const uint32_t P = c.nranks <= 1 ? 1 : c.nranks;
  regrow(c.d_lsrc, c.lsrc_cap, std::max<size_t>(c.n, 1));
  static const uint32_t max_parts =  // PM_LOCAL_SPLIT_MAX (tests): the finest split tried
      std::getenv("PM_LOCAL_SPLIT_MAX") ? static_cast<uint32_t>(std::strtoul(std::getenv("PM_LOCAL_SPLIT_MAX"), nullptr, 10))
                                        : (1u << 14);
  for (uint32_t k = 4; k <= max_parts; k *= 4) {
    FusedLineOut o;
    o.stride = stride;
    uint64_t ns = 0;
    bool ovf = false;
    for (uint32_t i = 0; i < k; ++i) {
      uint32_t* kept = nullptr;
      const LineStats st = run_line_part(c, pl, k, i, kept);
      if (st.overflow) {
        ovf = true;
        break;
      }
      if (ns + st.nsrc > c.lsrc_cap) throw std::runtime_error("internal: local split line sources out of range");
      if (st.nsrc)
        PM_HIP_CHECK(hipMemcpyAsync(c.d_lsrc + ns, c.d_sources, st.nsrc * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                    c.stream));
      ns += st.nsrc;
      o.tr.sources += st.nsrc;
      o.tr.edges += st.trav;
      o.tr.tokens += st.tokens;
      o.tr.walks += st.walks;
      if (want_walks && pl >= 4 && st.walks) {
        const size_t at = o.walks.size();
        o.walks.resize(at + st.walks * stride);
        PM_HIP_CHECK(hipMemcpy(o.walks.data() + at, kept + st.wbase[0], st.walks * stride * sizeof(uint32_t),
                               hipMemcpyDeviceToHost));
      }
    }
    if (ovf) continue;
    // the post-processing over every part's sources (line_post's rule)
    regrow(c.d_ldels, c.ldels_cap, std::max<size_t>(ns, 1));
    ensure_xcnt(c);
    auto* d_out = reinterpret_cast<unsigned long long*>(c.d_xcnt);  // 3 + 2P <= 64 + 4 * 64 words
    PM_HIP_CHECK(hipMemsetAsync(d_out, 0, (3 + 2 * P) * sizeof(uint64_t), c.stream));
    OwnerArgs oa{c.d_hubs, c.d_perm, static_cast<uint32_t>(c.hubs_host.size()), c.nranks};
    if (ns)
      hipLaunchKernelGGL(k_split_post, dim3(xgrid(ns)), dim3(kXBlock), 0, c.stream, c.d_lsrc, uint64_t(ns), c.d_tsm,
                         c.d_tpub[c.cur], static_cast<int>(line.indices[0]), c.d_malive, oa, c.d_ldels, d_out);
    PM_HIP_CHECK(hipGetLastError());
    std::vector<uint64_t> loc(3 + 2 * P);
    PM_HIP_CHECK(hipMemcpyAsync(loc.data(), d_out, loc.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    o.tr.acked = loc[0];
    o.deleted = loc[1] ? 1u : 0u;
    o.rm_v.assign(c.nranks, 0);
    o.rm_e.assign(c.nranks, 0);
    for (uint32_t r = 0; r < c.nranks; ++r) {
      o.rm_v[r] = loc[3 + r];
      o.rm_e[r] = loc[3 + P + r];
    }
    o.split = true;
    // (the line's sources stay the last part's in d_sources; the exact path and launch_post_tp are not used)
    c.nsources = 0;
    c.last_acked = o.tr.acked;
    c.local_split_parts = k;
    out = std::move(o);
    return true;
  }
  return false;
}

}  // namespace pm
