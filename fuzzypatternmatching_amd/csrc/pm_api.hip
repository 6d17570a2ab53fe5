// C-ABI (include/pm_abi.h) and host driver of the MI355X pattern-matching path.
//
// pm_run_beta restates the driver loop of src/run_pattern_matching_beta.cpp
// (:539-1425) on top of the device kernels in pm_kernels.hip and writes the
// same result directory layout.

#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <bitset>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pm_abi.h"
#include "host/graph_store.hpp"
#include "host/mt_jump.hpp"
#include "pm_device.hpp"
#include "pm_internal.hpp"
#include "pm_ingest.hpp"
#include "pm_rmat.hpp"
#include "pm_shard.hpp"
#include <thread>

struct pm_ctx : public pm::Ctx {};
namespace pm {
void gather_floor_forget(const void* owner);  // (diagnostics: the gather-floor cache of a destroyed context)
}

namespace pm {

// per thread: the shards of one process (pm_run_beta_local_shards, the CLI's one-thread-per-GPU mode) fail
// independently
static thread_local std::string g_last_error;

static void mkdir_p(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur += path[i];
    if (path[i] == '/' && cur.size() > 1) ::mkdir(cur.c_str(), 0755);
  }
  ::mkdir(path.c_str(), 0755);
}

static std::string fmt_double(double x) {
  std::ostringstream o;
  o << x;
  return o.str();
}

template <typename T>
static T* dalloc(uint64_t n) {
  T* p = nullptr;
  PM_HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(1, n) * sizeof(T)));
  return p;
}

static void require_gfx950(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= device)
    throw std::runtime_error("no HIP device " + std::to_string(device) + " available (the HIP path has no CPU fallback)");
  hipDeviceProp_t prop;
  PM_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    throw std::runtime_error(std::string("device arch ") + prop.gcnArchName + " is not gfx950 (MI355X)");
  // the driver loop waits on a few small read-backs per search: spin instead of
  // yielding, so the next launch follows the device at once (PM_SPIN=0: runtime
  // default; refused once the device's context is active, which then keeps its flags)
  static const bool spin = !std::getenv("PM_SPIN") || std::string(std::getenv("PM_SPIN")) != "0";
  if (spin && hipSetDevice(device) == hipSuccess && hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess)
    (void)hipGetLastError();
}

// Graph of one context: the whole graph (nshards == 1) or one shard's rows.
struct CtxInput {
  uint64_t n = 0;
  const uint64_t* off = nullptr;   // n + 1 offsets of the rows this context scans
  const uint32_t* col = nullptr;
  const uint32_t* gdeg = nullptr;  // global degrees (null: from off)
  bool symmetric = true;
  uint32_t nranks = 1;
  uint64_t hub_threshold = 1048576;
  uint32_t nshards = 1, shard = 0;
  Comm* comm = nullptr;            // ownership passes to the context
  bool col_on_device = false;      // col is device memory (GPU-built graph); off stays host
  bool col_release = false;        // ... and the context frees it once copied (the caller must not)
  uint32_t inprocess_shards = 1;   // shards of this process on the same device (ThreadComm groups)
  const uint64_t* in_off = nullptr;  // directed graphs: in-rows built by the caller (host offsets,
  const uint32_t* in_col = nullptr;  // columns where col lives), e.g. by the GPU ingest
};

// In-rows of a directed CSR (rows sorted by source id, duplicates adjacent):
// superstep 0 pulls along in-edges, i.e. exactly the messages the reference
// pushes along out-edges (nonunique_ee.hpp:555-560, SURVEY A.6 hazard 10).
static void transpose_csr(uint64_t n, const uint64_t* off, const uint32_t* col, std::vector<uint64_t>& toff,
                          std::vector<uint32_t>& tcol) {
  toff.assign(n + 1, 0);
  for (uint64_t e = 0; e < off[n]; ++e) {
    if (col[e] >= n) throw std::runtime_error("edge target out of range");
    ++toff[col[e] + 1];
  }
  for (uint64_t v = 0; v < n; ++v) toff[v + 1] += toff[v];
  tcol.resize(off[n]);
  std::vector<uint64_t> at(toff.begin(), toff.end() - 1);
  for (uint64_t v = 0; v < n; ++v)
    for (uint64_t e = off[v]; e < off[v + 1]; ++e) tcol[at[col[e]]++] = static_cast<uint32_t>(v);
}

// Degree labels (vertex_data_db_degree.hpp:109) from the global out-degrees (host: the layout uploads them).
static void set_degree_labels(Ctx& c) {
  c.labels_host.assign(c.n, 0);
  for (uint64_t v = 0; v < c.n; ++v) c.labels_host[v] = degree_label(c.deg_host[v]);
}

// Host pages registered with the runtime for the lifetime of the object (large
// uploads only; a range the runtime refuses, e.g. memory that is already
// pinned, is copied as pageable memory).
struct PinnedRange {
  void* base = nullptr;
  PinnedRange(const void* p, size_t bytes) {
    if (!p || bytes < (size_t(16) << 20)) return;
    const size_t page = 4096;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~(page - 1);
    const size_t len = ((reinterpret_cast<uintptr_t>(p) + bytes + page - 1) & ~(page - 1)) - a;
    if (hipHostRegister(reinterpret_cast<void*>(a), len, hipHostRegisterDefault) == hipSuccess)
      base = reinterpret_cast<void*>(a);
    else
      (void)hipGetLastError();
  }
  ~PinnedRange() {
    if (base) (void)hipHostUnregister(base);
  }
  PinnedRange(const PinnedRange&) = delete;
  PinnedRange& operator=(const PinnedRange&) = delete;
};

static void destroy_ctx(pm_ctx* c);

static pm_ctx* create_ctx(const CtxInput& in, const char* pattern_dir, int device) {
  std::unique_ptr<Comm> comm(in.comm);
  // a device-resident input the caller handed over (col_release) is freed as soon as it is copied
  struct ColRelease {
    const uint32_t* p;
    void now() {
      if (p) (void)hipFree(const_cast<uint32_t*>(p));
      p = nullptr;
    }
    ~ColRelease() { now(); }
  } col_release{in.col_on_device && in.col_release ? in.col : nullptr};
  if (!in.off || !in.col) throw std::runtime_error("pm_create: null graph");
  if (in.nshards == 0 || in.shard >= in.nshards) throw std::runtime_error("pm_create: bad shard index");
  if (in.nshards > 1 && !comm) throw std::runtime_error("pm_create: sharded context without a communicator");
  require_gfx950(device);
  // a construction that throws releases what it allocated (device buffers, stream, communicator)
  std::unique_ptr<pm_ctx, void (*)(pm_ctx*)> c(new pm_ctx(), destroy_ctx);
  c->device = device;
  PM_HIP_CHECK(hipSetDevice(device));
  PM_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  c->n = in.n;
  c->nnz = in.off[in.n];
  c->symmetric = in.symmetric;
  c->nranks = in.nranks ? in.nranks : 1;
  c->hub_threshold = in.hub_threshold;
  c->nshards = in.nshards;
  c->shard = in.shard;
  c->comm = comm.get();
  c->comm_owned = comm.release();
  if (c->n >= (1ull << 30)) throw std::runtime_error("more than 2^30 vertices (30-bit positions in M entries)");
  // the rows superstep 0 scans: the CSR itself, or its in-rows for a directed graph
  std::vector<uint64_t> tin_off;
  std::vector<uint32_t> tin_col;
  const uint64_t* soff = in.off;
  const uint32_t* scol = in.col;
  size_t arena = 0;
  bool any_sv = false;
  std::string build_err;
  try {
    if (!c->symmetric) {
      if (in.nshards > 1) throw std::runtime_error("directed input graphs are supported on one shard only");
      if (in.in_off && in.in_col) {
        soff = in.in_off;
        scol = in.in_col;
      } else {
        if (in.col_on_device) throw std::runtime_error("directed device-resident graphs need their in-rows");
        transpose_csr(c->n, in.off, in.col, tin_off, tin_col);
        soff = tin_off.data();
        scol = tin_col.data();
      }
      c->rdeg_host.resize(c->n);
      for (uint64_t v = 0; v < c->n; ++v) c->rdeg_host[v] = static_cast<uint32_t>(soff[v + 1] - soff[v]);
    }
    c->pattern = load_pattern_dir(pattern_dir);
    const PatternGraph& pg = c->pattern.graph;
    if (pg.diameter == 0) throw std::runtime_error("pattern_stat: diameter is 0 or missing");
    for (int t = 0; t < kMaxTemplateVertices; ++t) c->pa.adj[t] = pg.adj[t];
    c->pa.K = static_cast<int32_t>(pg.vertex_data.size());
    for (int t = 0; t < c->pa.K; ++t) c->pa.plabel[t] = pg.vertex_data[t];
    // a label of more than two template vertices: its 2-bit code cannot carry T_pub (tpub_code)
    for (int t = 0; t < c->pa.K; ++t) {
      int k = 0;
      for (int u = 0; u < c->pa.K; ++u) k += c->pa.plabel[u] == c->pa.plabel[t];
      if (k > 2) c->xcode_wide = true;
    }
    any_sv = false;
    for (size_t pl = 0; pl < c->pattern.lines.size(); ++pl) {
      const auto& l = c->pattern.lines[pl];
      if (!l.selected_vertices) continue;
      any_sv = true;
      if (pl >= 4 || l.valid_cycle)  // the reference applies it in nem_1 path checks only
        throw std::runtime_error("pattern_nlc selected_vertices=1 is supported on path lines (index < 4, valid_cycle 0)");
    }
    // global degrees (labels, hubs, layout order) and the lengths of the rows held here
    c->deg_host.resize(c->n);
    if (in.gdeg) c->ldeg_host.reserve(c->n);
    for (uint64_t v = 0; v < c->n; ++v) {
      const uint64_t d = in.gdeg ? in.gdeg[v] : in.off[v + 1] - in.off[v];
      if (d > 0xFFFFFFFFull) throw std::runtime_error("degree above 2^32");
      const uint64_t ld = in.off[v + 1] - in.off[v];
      // a shard holds the whole rows it owns, and of a delegate (degree >= -d) the entries whose target it owns
      if (in.gdeg && ld && (d >= c->hub_threshold && c->nshards > 1 ? ld > d
                                                                     : (ld != d || v % c->nshards != c->shard)))
        throw std::runtime_error("shard rows must be the owned rows (v % nshards == shard) with their full degree, "
                                 "and delegate rows (degree >= hub threshold) split by target owner");
      c->deg_host[v] = static_cast<uint32_t>(d);
      if (d >= c->hub_threshold) c->hubs_host.push_back(v);
      if (in.gdeg) c->ldeg_host.push_back(static_cast<uint32_t>(ld));
      c->held_rows += ld != 0;
      if (ld && d >= c->hub_threshold && c->nshards > 1) c->held_hub_entries += ld;
    }
    c->split_hubs = c->nshards > 1 && !c->hubs_host.empty();
    for (uint64_t j = c->shard; c->split_hubs && j < c->hubs_host.size(); j += c->nshards)
      c->hub_area += c->deg_host[c->hubs_host[j]];
    // device graph + state; padded slot count of the rows scanned here (label independent)
    c->nq = 0;
    for (uint64_t v = 0; v < c->n; ++v) c->nq += padded_degree(soff[v + 1] - soff[v]);
    c->mcap = c->nq;
    c->d_offp = dalloc<uint64_t>(c->n + 1);
    c->d_offr = dalloc<uint64_t>(c->n + 1);
    // slot buffers carry kTileEntries entries of tail padding (superstep-0 tile loads read whole tiles)
    // dense superstep-0 M region behind the tail padding (both buffers: relayout swaps them)
    if (c->symmetric && c->nq)
      c->dcap = std::min<uint64_t>(0xFFFFFFF0ull, std::max<uint64_t>(uint64_t(1) << 16, c->nq / 8));
    c->dbase = c->nq + kTileEntries;
    c->d_colp = dalloc<uint32_t>(c->nq + kTileEntries + c->dcap + c->hub_area);
    c->d_perm = dalloc<uint32_t>(c->n);
    c->d_pos = dalloc<uint32_t>(c->n);
    if (!c->hubs_host.empty()) {
      c->d_hubs = dalloc<uint64_t>(c->hubs_host.size());
      PM_HIP_CHECK(hipMemcpy(c->d_hubs, c->hubs_host.data(), c->hubs_host.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    c->d_tpub[0] = dalloc<uint16_t>(c->n);
    c->d_tpub[1] = dalloc<uint16_t>(c->n);
    c->d_tst = dalloc<uint16_t>(c->n);
    c->d_mcol = dalloc<uint32_t>(c->nq + kTileEntries + c->dcap + c->hub_area);
    c->d_mlen = dalloc<uint32_t>(c->n);
    c->d_malive = dalloc<uint32_t>(c->n);
    c->d_slist = dalloc<uint32_t>(c->n);
    c->d_smask[0] = dalloc<uint64_t>((c->n + 63) / 64 + 1);
    c->d_smask[1] = dalloc<uint64_t>((c->n + 63) / 64 + 1);
    c->d_sources = dalloc<uint32_t>(c->n);
    c->d_nS = dalloc<uint32_t>(2);  // [1]: long-row stamp (launch_compact_rows)
    PM_HIP_CHECK(hipMemset(c->d_nS, 0, 2 * sizeof(uint32_t)));
    c->d_flags = dalloc<uint32_t>(4);
    c->d_tsm = dalloc<uint8_t>(c->n);
    c->d_tcode = dalloc<uint32_t>((c->n + 15) / 16 + 1);
    if (c->nranks > 64) throw std::runtime_error("more than 64 ranks for result-file attribution");
    c->d_part = dalloc<uint64_t>(uint64_t(kPartGridMax) * slot_words(*c));
    size_t free_b = 0, total_b = 0;
    PM_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    arena = std::min<size_t>(free_b / 2, size_t(32) << 30);
    if (in.inprocess_shards > 1)  // in-process shard groups share one device
      arena = std::min<size_t>(arena, std::max<size_t>(size_t(1) << 30, free_b / (2 * in.inprocess_shards)));
    arena = std::max<size_t>(arena, size_t(64) << 20);
    // PM_ARENA_MB=<MiB> (tests): a smaller arena (the exact path lines' source batches)
    if (const char* e = std::getenv("PM_ARENA_MB"))
      arena = std::min<size_t>(arena, std::max<size_t>(1, std::strtoull(e, nullptr, 10)) << 20);
  } catch (const std::exception& e) {
    build_err = e.what();
    arena = 0;
  }
  // one size on every shard: the replicated lines' walk storage and TDS chunk caps come from it, and a line
  // that overflowed on some shards only would send those into collectives the others never make
  // -- and construction is collective: a shard that failed above still takes part (arena 0), so the others
  // are not left in a collective it never makes, and every shard then fails
  arena = static_cast<size_t>(shard_agree_min(*c, arena));
  if (!build_err.empty()) throw std::runtime_error(build_err);
  if (arena == 0) throw std::runtime_error("another shard failed while building its context");
  c->arena.base = dalloc<char>(arena);
  c->arena.cap = arena;
  if (const char* e = std::getenv("PM_FUSED_LINES")) c->fused_lines = std::string(e) != "0";
  if (const char* e = std::getenv("PM_ROW_COMPACTION")) c->no_row_compaction = std::string(e) == "0";
  if (const char* e = std::getenv("PM_PULL_PIECES")) c->long_seen_off = std::string(e) == "0";
  if (const char* e = std::getenv("PM_PULL_LONG")) c->pull_long = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("PM_DIAG_STEP")) c->diag_step = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  if (any_sv) c->fused_lines = false;  // token-source sets across lines: the per-position path keeps them
  c->any_sv = any_sv;
  // Grid-barrier kernels (k_lines, the list compaction's scan) need every block resident.  A cooperative launch
  // guarantees it but costs ~28 us per launch (85 us per S=28 step for three launches, tools/gpu_coop_ab.sh); with one
  // context on the device the grids are sized to fit and nothing else that waits on them runs beside them, so an
  // ordinary launch is used.  Shards sharing a device (in-process shards, host-collective ranks) could hold each
  // other's blocks out with their spinning grids: cooperative.  PM_COOP=1 / PM_LINES_NOCOOP=1 force either.
  c->coop = in.inprocess_shards > 1 || (c->comm && c->comm->transport() != PM_TRANSPORT_RCCL);
  // (host collectives: the ranks may share the device -- several processes on one GPU; RCCL never puts two ranks
  // on one device.  A caller running two unrelated contexts concurrently on one GPU sets PM_COOP=1.)
  if (const char* e = std::getenv("PM_COOP")) c->coop = std::string(e) == "1";
  if (const char* e = std::getenv("PM_LINES_NOCOOP")) if (std::string(e) == "1") c->coop = false;
  if (const char* e = std::getenv("PM_SPLIT_LINES")) c->split_min = std::strtoull(e, nullptr, 10);
  if (const char* e = std::getenv("PM_HASH_SLOTS")) c->hash_slots = std::strtoull(e, nullptr, 10);
  if (const char* e = std::getenv("PM_HANDOFF")) c->handoff_ss = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  if (const char* e = std::getenv("PM_DEBUG_NOGROW_SHARD")) c->nogrow_shard = std::strtoll(e, nullptr, 10);
  if (const char* e = std::getenv("PM_DEBUG_OVERFLOW_SHARD")) c->overflow_shard = std::strtoll(e, nullptr, 10);
  // diagnostics: PM_FORCE_PULL=1 keeps the pull form in every LCC call (an
  // asymmetric M then aborts the search: tests use it to find such inputs)
  if (const char* e = std::getenv("PM_FORCE_PULL")) c->force_pull = std::string(e) == "1" && c->symmetric;
  // default labels = degree labels; the id-major adjacency is staged in the
  // M column buffer and permuted into the label-major d_colp
  if (c->nnz) {
    if (in.col_on_device) {
      PM_HIP_CHECK(hipMemcpy(c->d_mcol, scol, c->nnz * sizeof(uint32_t), hipMemcpyDeviceToDevice));
      col_release.now();
    } else {
      // pinned staging: the caller's pages are registered for the copy, so the
      // adjacency moves by DMA without a bounce through driver staging buffers
      PinnedRange pin(scol, c->nnz * sizeof(uint32_t));
      PM_HIP_CHECK(hipMemcpy(c->d_mcol, scol, c->nnz * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
  }
  set_degree_labels(*c);
  const auto t_lay = std::chrono::steady_clock::now();
  build_label_layout(*c, c->d_mcol, false, c->d_colp);
  build_tiling(*c);
  PM_HIP_CHECK(hipStreamSynchronize(c->stream));
  c->layout_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_lay).count();
  return c.release();
}

static pm_ctx* create_ctx(const pm_graph_desc* g, const char* pattern_dir, int device) {
  if (!g || !g->off || !g->col) throw std::runtime_error("pm_create: null graph");
  CtxInput in;
  in.n = g->n;
  in.off = g->off;
  in.col = g->col;
  in.symmetric = g->symmetric != 0;
  in.nranks = g->nranks;
  in.hub_threshold = g->hub_threshold;
  return create_ctx(in, pattern_dir, device);
}

static void destroy_ctx(pm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  void* ptrs[] = {c->d_offp, c->d_offr, c->d_colp, c->d_perm, c->d_pos, c->d_labs, c->d_hubs,
                  c->d_ktab, c->d_ttab, c->d_hseg, c->d_hscr, c->d_tpub[0], c->d_tpub[1], c->d_tst, c->d_mcol,
                  c->d_mlen, c->d_malive, c->d_slist, c->d_slist2, c->d_nS2, c->d_ccnt, c->d_cbase, c->d_ctmp, c->d_smask[0], c->d_smask[1], c->d_kmask, c->d_sources, c->d_nS, c->d_flags, c->d_tsm,
                  c->d_counts, c->d_part, c->d_tmask, c->d_tbase, c->d_scan_tmp, c->arena.base, c->d_tn, c->d_pseen,
                  c->d_tcode, c->d_rarea, c->d_rbase, c->d_rcnt, c->d_rofs, c->d_hrec, c->d_srec, c->d_rscan_tmp, c->d_cdesc,
                  c->d_xsend, c->d_xrecv, c->d_xent_send,
                  c->d_xent_recv, c->d_xcnt, c->d_rmoff, c->d_rmcol, c->d_xred, c->d_hubinfo, c->d_moff, c->d_hubpart, c->d_xsplit, c->d_push,
                  c->d_lrows, c->d_lscr, c->d_clstat, c->d_lsrc, c->d_ldels,
                  };
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete c->comm_owned;
  if (c->h_pin) (void)hipHostFree(c->h_pin);
  if (c->h_pin_lines) (void)hipHostFree(c->h_pin_lines);
  free_line_buffers(*c);
  for (auto e : c->events) (void)hipEventDestroy(e);
  if (c->ev_handoff) (void)hipEventDestroy(c->ev_handoff);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->rstream) (void)hipStreamDestroy(c->rstream);
  if (c->ev_rb) (void)hipEventDestroy(c->ev_rb);
  if (c->ev_tz0) (void)hipEventDestroy(c->ev_tz0);
  if (c->ev_tz) (void)hipEventDestroy(c->ev_tz);
  delete c;
}

// New labels: rebuild the label-major layout from the current one (the M
// column buffer is free between searches and receives the new adjacency).
static void relayout(Ctx& c) {
  const auto t_lay = std::chrono::steady_clock::now();
  build_label_layout(c, c.d_colp, true, c.d_mcol);
  std::swap(c.d_colp, c.d_mcol);
  c.mcap = c.nq;  // d_mcol is the former d_colp (nq entries, no remote region)
  build_tiling(c);
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.layout_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_lay).count();
  c.lcc_started = false;
  c.tpub_clean = false;  // positions changed: the next reset clears T_pub entirely
  c.long_seen.clear();   // (new labels: where long rows survive is not known)
  c.tcode_zeroed = false;  // (new labels: more code words than the last clear covered)
  // the line grid of a search's prelaunched lines is sized by the previous search's |S| (identical for repeated
  // searches of one layout); new labels: the full grid until a search has run
  c.live_hint = ~0ull;
}

// defer: the fills stay queued for the search's first launch (flush_zero batches them into one)
static void reset_state(Ctx& c, bool defer = false) {
  if (c.tpub_clean && c.lcc_started) {
    c.clear_pending = true;  // nonzero T_pub only at (every shard's) slist entries; d_nS zeroed after the clear
    c.clear_cap = c.nS_host;
  } else {
    if (!c.tpub_clean) {
      PM_HIP_CHECK(hipMemsetAsync(c.d_tpub[0], 0, c.n * sizeof(uint16_t), c.stream));
      PM_HIP_CHECK(hipMemsetAsync(c.d_tpub[1], 0, c.n * sizeof(uint16_t), c.stream));
    }
    zero_later(c, c.d_nS, sizeof(uint32_t));
  }
  c.tpub_clean = true;
  c.lines_prelaunched = false;  // (a failed search may leave one behind; the stream has run it)
  // d_tsm needs no reset: only sources are read, and selecting a source resets its entry
  c.smask_valid = false;
  zero_later(c, c.d_flags, 4 * sizeof(uint32_t));
  queue_lines_ctl_clear(c);
  if (!defer) flush_zero(c);
  c.cur = 0;
  c.nS_host = 0;
  c.push_long = true;  // full-length rows until the first row compaction
  c.lcc_started = false;
  c.replicated = false;
  c.k1_dense = false;
  c.nsources = 0;
  c.npseen = 0;
}

// Per-superstep outputs of one LCC call.
struct LccOut {
  std::vector<std::vector<uint64_t>> vcount, ecount;  // [superstep][rank]
  std::vector<uint64_t> trav;
  std::vector<double> seconds;
  bool not_finished = false;
  uint64_t matching_rows = 0;  // vertices with a label match (superstep 0 of the first call)
  // this shard's counts: per rank after the last superstep; superstep-0 survivors and M entries
  std::vector<uint64_t> loc_vc, loc_ec;
  uint64_t loc_surv = 0, loc_edges = 0;
};

void debug_point(Ctx& c, const char* where) {
  static const int level = std::getenv("PM_DEBUG_SYNC") ? std::atoi(std::getenv("PM_DEBUG_SYNC")) : 0;
  if (!level) return;
  hipError_t e = hipStreamSynchronize(c.stream);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("device fault before debug point '") + where + "' (shard " +
                             std::to_string(c.shard) + "): " + hipGetErrorString(e));
  if (level >= 2) std::fprintf(stderr, "[pm dbg] shard %u: %s ok\n", c.shard, where);
}

// PM_DEBUG_WATCH_ID=<vertex id> (diagnostics): the vertex's state on this shard at the named point.
static void debug_watch(Ctx& c, const char* where) {
  static const char* e = std::getenv("PM_DEBUG_WATCH_ID");
  if (!e || c.perm_host.empty()) return;
  const uint64_t id = std::strtoull(e, nullptr, 10);
  uint32_t p = 0;
  PM_HIP_CHECK(hipMemcpy(&p, c.d_pos + id, 4, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  uint16_t t0 = 0, t1 = 0, ts = 0;
  uint32_t ml = 0, ma = 0, ns = 0;
  PM_HIP_CHECK(hipMemcpy(&t0, c.d_tpub[0] + p, 2, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipMemcpy(&t1, c.d_tpub[1] + p, 2, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipMemcpy(&ts, c.d_tst + p, 2, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipMemcpy(&ml, c.d_mlen + p, 4, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipMemcpy(&ma, c.d_malive + p, 4, hipMemcpyDeviceToHost));
  PM_HIP_CHECK(hipMemcpy(&ns, c.d_nS, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> sl(ns);
  if (ns) PM_HIP_CHECK(hipMemcpy(sl.data(), c.d_slist, ns * 4, hipMemcpyDeviceToHost));
  int at = -1;
  for (uint32_t i = 0; i < ns; ++i)
    if (sl[i] == p) at = static_cast<int>(i);
  std::fprintf(stderr, "[pm watch] shard %u %-22s id %llu pos %u: tpub %u/%u (cur %d) tst %u mlen %u malive %u, slist[%d] of %u\n",
               c.shard, where, static_cast<unsigned long long>(id), p, t0, t1, c.cur, ts, ml, ma, at, ns);
}

// Pinned host staging of at least `words` u64 (read-backs of the driver loop).
uint64_t* pinned(Ctx& c, size_t words) {
  if (c.h_pin_words < words) {
    if (c.h_pin) (void)hipHostFree(c.h_pin);
    c.h_pin = nullptr;
    const size_t w = std::max<size_t>(words, 1 << 15);
    PM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c.h_pin), w * sizeof(uint64_t), hipHostMallocDefault));
    c.h_pin_words = w;
  }
  return c.h_pin;
}

static void ensure_counts(Ctx& c, size_t slots) {
  if (c.counts_slots >= slots) return;
  if (c.d_counts) (void)hipFree(c.d_counts);
  c.d_counts = dalloc<uint64_t>(slots * slot_words(c));
  c.counts_slots = slots;
}

// label_propagation_pattern_matching_bsp (nonunique_ee.hpp:1033-1153).
static LccOut lcc_call(Ctx& c, bool init_step) {
  const uint64_t D = c.pattern.graph.diameter;
  const uint64_t W = slot_words(c);
  const uint64_t P = c.nranks <= 1 ? 1 : c.nranks;
  ensure_counts(c, D);
  while (c.events.size() < D + 3) {
    hipEvent_t e;
    PM_HIP_CHECK(hipEventCreate(&e));
    c.events.push_back(e);
  }
  std::vector<hipEvent_t>& ev = c.events;  // [0..D] superstep bounds, [D+1], [D+2] superstep-0 kernel
  // (a dense superstep-0 state is never packed: with D >= 2 the hand-off follows a later superstep)
  const uint64_t handoff_ss = D == 1 ? 0 : std::max<uint64_t>(1, std::min<uint64_t>(c.handoff_ss, D - 1));
  zero_later(c, c.d_counts, D * W * sizeof(uint64_t));  // kernels add into the slots
  // the search's reset fills go with superstep 0's own (one launch, before the call's timing event)
  if (init_step) queue_lcc_first_fills(c);
  flush_zero(c);
  c.probe("zero flushed");
  PM_HIP_CHECK(hipEventRecord(ev[0], c.stream));
  bool k_timed = false, handed_off = false;
  // diagnostics: PM_DEBUG_LCC_STOP=k -- the first call runs supersteps 0..k-1 only
  static const uint64_t stop_at = std::getenv("PM_DEBUG_LCC_STOP") ? std::strtoull(std::getenv("PM_DEBUG_LCC_STOP"), nullptr, 10) : 0;
  // sharded: the state became the replica (the sharded part of the search ends here)
  auto handoff = [&] {
    if (!c.comm) return;
    if (!c.ev_handoff) PM_HIP_CHECK(hipEventCreate(&c.ev_handoff));
    PM_HIP_CHECK(hipEventRecord(c.ev_handoff, c.stream));
    c.comm_wall_handoff = c.comm->wall;
    handed_off = true;
  };
  for (uint64_t ss = 0; ss < D; ++ss) {
    if (init_step && stop_at && ss >= stop_at) {
      PM_HIP_CHECK(hipEventRecord(ev[D], c.stream));
      break;
    }
    uint64_t* slot = c.d_counts + ss * W;
    if (ss == 0 && init_step) {
      if (c.lcc_started) throw std::runtime_error("init_step LCC after the state map was built");
      // (the call's start event ev[0] directly precedes the kernel -- the search's fills were flushed before it --
      // so it also opens the kernel's own interval: one event record less before superstep 0)
      launch_lcc_first(c, slot, nullptr, ev[D + 2]);
      c.probe("superstep 0 launched");
      debug_point(c, "superstep 0"); debug_watch(c, "superstep 0");
      k_timed = true;
      // |slist| is read back with the counters at the end of the call; until
      // then later supersteps size their grids by its upper bound
      c.nS_host = static_cast<uint32_t>(std::min<uint64_t>(c.ss0_rows, 0xFFFFFFFFull));
      c.lcc_started = true;
      // sharded: the delegates' shares meet at their controllers; the survivors' codes of every shard
      // for the next superstep's pulls; a one-superstep pattern goes to the replica at once
      if (c.split_hubs) shard_hub_combine(c, slot);
      debug_point(c, "delegate combine"); debug_watch(c, "delegate combine");
      if (handoff_ss > 0) shard_codes_after_first(c);
      else {
        shard_replicate(c);
        handoff();
      }
      debug_point(c, "code exchange / replica"); debug_watch(c, "code exchange / replica");
    } else {
      if (!c.lcc_started) throw std::runtime_error("LCC without an initial step: state map is empty");
      // pull form while M is known symmetric (the first call on a symmetric
      // graph: no cycle flag set yet); push form otherwise
      if (!c.force_pull && (!c.symmetric || !init_step)) launch_lcc_push(c, slot);
      else {
        // S collapses in the first later supersteps (S=28 tree: 9.8 M -> 0.8 M -> 26 k): the next
        // supersteps, the NLC lines and the next reset walk the live entries only.  (Appending the live
        // entries inside the superstep, one counter reservation per 64-entry chunk, measured 1.2 ms slower
        // at S=28: 153 k atomics on one address serialise.)
        c.cur_ss = init_step ? ss : 0;
        launch_lcc_step(c, slot, init_step && ss == 1, ss + 1 == D, init_step);
        debug_point(c, "pull superstep"); debug_watch(c, "pull superstep");
        if (init_step && (ss == 1 || ss == 2) && ss + 1 < D) launch_compact_slist(c);
        // the codes' clear for the next search (their last reader was the first later superstep), beside the
        // latency-bound small supersteps after the second compaction rather than beside the first
        if (init_step && (ss == 2 || (ss == 1 && D == 2))) side_clear_codes(c);
        debug_point(c, "list compaction"); debug_watch(c, "list compaction");
      }
      // sharded: the state of S goes to the replica after superstep handoff_ss; before, the supersteps run
      // over each shard's own rows, and after the first the shards' new T_pub are exchanged
      if (init_step && ss == handoff_ss) {
        shard_replicate(c);
        handoff();
      } else if (init_step && ss < handoff_ss) {
        shard_tpub_exchange(c);
      }
      debug_point(c, "superstep end"); debug_watch(c, "superstep end");
    }
    if (c.fine_timing || ss + 1 == D) PM_HIP_CHECK(hipEventRecord(ev[ss + 1], c.stream));
  }
  // rows with dead entries compacted for the lines and the next call (k_compact_rows)
  const uint32_t stamp = ++c.lcc_calls;
  if (!c.no_row_compaction) launch_compact_rows(c, stamp);
  debug_point(c, "row compaction");
  c.probe("lcc issued");
  // read-back through pinned memory: [nS | local counts | summed counts]
  uint64_t* pin = pinned(c, 1 + 2 * D * W);
  // sharded: the supersteps before the replica counted this shard's rows only: their slots are summed
  // over the shards (the replica's supersteps count the whole state on every shard)
  const uint64_t sharded_slots = c.comm && init_step ? handoff_ss + 1 : 0;
  // one context with prelaunched lines: the read-back copies go on a side stream ordered after the call's last
  // kernel, so they run beside the lines instead of in front of them (the lines read neither the list count nor
  // the counters, and the host waits for both)
  const bool side = c.prelaunch_lines && !sharded_slots;
  hipStream_t rs = c.stream;
  if (side) {
    if (!c.rstream) {
      PM_HIP_CHECK(hipStreamCreateWithFlags(&c.rstream, hipStreamNonBlocking));
      PM_HIP_CHECK(hipEventCreateWithFlags(&c.ev_rb, hipEventDisableTiming));
    }
    PM_HIP_CHECK(hipEventRecord(c.ev_rb, c.stream));
    PM_HIP_CHECK(hipStreamWaitEvent(c.rstream, c.ev_rb, 0));
    rs = c.rstream;
    prelaunch_lines_fused(c);  // the device goes on with the lines while the host parses
  }
  PM_HIP_CHECK(hipMemcpyAsync(pin, c.d_nS, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, rs));  // + stamp
  if (sharded_slots) {  // this shard's counts, then the sums over the shards
    PM_HIP_CHECK(hipMemcpyAsync(pin + 1, c.d_counts, D * W * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.comm->allreduce_sum_u64(c.d_counts, sharded_slots * W, c.stream);
  }
  PM_HIP_CHECK(hipMemcpyAsync(pin + 1 + D * W, c.d_counts, D * W * sizeof(uint64_t), hipMemcpyDeviceToHost, rs));
  if (c.prelaunch_lines && !side) prelaunch_lines_fused(c);
  // (with the read-back on the side stream the host parses the counters while the prelaunched lines run; the
  // lines' own read-back waits for the stream in run_lines_fused)
  if (side) stream_wait(c.rstream);
  debug_point(c, "counters + prelaunched lines");
  if (!side) stream_wait(c.stream);
  c.probe("lcc synced");
  std::vector<uint64_t> host(pin + 1 + D * W, pin + 1 + 2 * D * W);
  std::vector<uint64_t> local = sharded_slots ? std::vector<uint64_t>(pin + 1, pin + 1 + D * W) : host;
  const uint32_t nS = static_cast<uint32_t>(pin[0] & 0xFFFFFFFFull);
  c.nS_host = nS;
  c.push_long = c.no_row_compaction || !nS || static_cast<uint32_t>(pin[0] >> 32) == stamp;
  LccOut out;
  bool asym = false;
  {
    const uint64_t* h = local.data() + (D - 1) * W;
    out.loc_vc.assign(h, h + c.nranks);
    out.loc_ec.assign(h + P, h + P + c.nranks);
  }
  for (uint64_t ss = 0; ss < D; ++ss) {
    const uint64_t* h = host.data() + ss * W;
    std::vector<uint64_t> vc(c.nranks), ec(c.nranks);
    for (uint32_t r = 0; r < c.nranks; ++r) {
      vc[r] = h[r];
      ec[r] = h[P + r];
    }
    out.vcount.push_back(vc);
    out.ecount.push_back(ec);
    out.trav.push_back(h[2 * P]);
    if (ss == 0 && init_step) {
      // superstep 0 visits only label-matching rows; their adjacency size is
      // a property of the layout (build_tiling), identical to the reference's count
      out.trav.back() = c.ss0_trav_all;
      out.matching_rows = c.ss0_rows;
      for (uint32_t r = 0; r < c.nranks; ++r) {  // this shard's survivors (roofline bytes)
        out.loc_surv += local[r];
        out.loc_edges += local[P + r];
      }
    }
    if (init_step && ss > 0) {  // pull supersteps that deferred long rows (the next search's pieces launches)
      if (c.long_seen.size() < D) c.long_seen.assign(D, 1);
      c.long_seen[ss] = h[2 * P + 4] != 0;
    }
    if (init_step) {  // the survivors' mean |M| per superstep (the next search's entries in flight)
      uint64_t v = 0, e = 0;
      for (uint32_t r = 0; r < c.nranks; ++r) {
        v += h[r];
        e += h[P + r];
      }
      if (c.m_per_row.size() < D) c.m_per_row.resize(D, 0.0);
      c.m_per_row[ss] = v ? double(e) / double(v) : 0.0;
    }
    if (h[2 * P + 2]) out.not_finished = true;
    if (h[2 * P + 3]) asym = true;
    float ms = 0.f;
    if (c.fine_timing) PM_HIP_CHECK(hipEventElapsedTime(&ms, ev[ss], ev[ss + 1]));
    out.seconds.push_back(ms * 1e-3);
    c.device_seconds += ms * 1e-3;
  }
  if (!c.fine_timing) {  // one interval for the whole call
    float ms = 0.f;
    PM_HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[D]));
    c.device_seconds += ms * 1e-3;
  }
  if (k_timed) {
    float ms = 0.f;
    PM_HIP_CHECK(hipEventElapsedTime(&ms, ev[0], ev[D + 2]));
    c.lcc_first_ms = ms;
  }
  if (handed_off) {  // minus the collectives' host time, during which the stream idles (in-process shards wait
                     // for each other there): the shard's own device work and launch gaps
    float ms = 0.f;
    PM_HIP_CHECK(hipEventElapsedTime(&ms, ev[0], c.ev_handoff));
    c.sharded_ms = static_cast<float>(std::max(0.0, ms - (c.comm_wall_handoff - c.comm_wall0) * 1e3));
  }
  c.probe("lcc parsed");
  if (asym)
    throw std::runtime_error(
        "active-edge map became asymmetric (a cycle-marked edge outlived its neighbour's message) in a pull-form "
        "superstep (PM_FORCE_PULL=1)");
  return out;
}

// Algorithmic bytes of the fused superstep-0 kernel (DESIGN.md
// roofline): 4 B neighbour id per scanned adjacency entry, 12 B per scanned
// (label-matching) row (8 B row offset + 2 B T + 2 B TN), 12 B of state per
// survivor (T_state, T_pub, |M| written, mlen) and 4 B per kept M entry.  The
// 2 B neighbour-T gather of the survey's model is not counted: the label-major
// layout derives a neighbour's template bits from its position, no load.
static uint64_t lcc_first_bytes(const Ctx& c, uint64_t scanned, uint64_t survivors, uint64_t edges,
                                uint64_t matching_rows) {
  (void)c;
  return scanned * 4 + matching_rows * 12 + survivors * 12 + edges * 4;
}

struct DriverFiles {
  std::vector<std::string> superstep, step, iteration;
  std::vector<std::vector<std::string>> vcount, ecount, mcount;  // per rank
};

static void add_count_lines(Ctx& c, DriverFiles& f, uint64_t itr, const char* tag, uint64_t idx,
                            const std::vector<uint64_t>& vc, const std::vector<uint64_t>& ec, uint64_t msgs) {
  for (uint32_t r = 0; r < c.nranks; ++r) {
    const std::string pre = std::to_string(itr) + ", " + tag + ", " + std::to_string(idx) + ", ";
    f.vcount[r].push_back(pre + std::to_string(vc[r]));
    f.ecount[r].push_back(pre + std::to_string(ec[r]));
    f.mcount[r].push_back(pre + std::to_string(r == 0 ? msgs : 0));
  }
}

static void count_state(Ctx& c, std::vector<uint64_t>& vc, std::vector<uint64_t>& ec) {
  ensure_counts(c, 1);
  const uint64_t W = slot_words(c);
  const uint64_t P = c.nranks <= 1 ? 1 : c.nranks;
  PM_HIP_CHECK(hipMemsetAsync(c.d_counts, 0, W * sizeof(uint64_t), c.stream));
  if (c.nS_host) launch_count_state(c, c.d_counts);
  std::vector<uint64_t> host(W);
  PM_HIP_CHECK(hipMemcpyAsync(host.data(), c.d_counts, host.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  vc.assign(c.nranks, 0);
  ec.assign(c.nranks, 0);
  for (uint32_t r = 0; r < c.nranks; ++r) {
    vc[r] = host[r];
    ec[r] = host[P + r];
  }
}

static uint32_t owner_host(const Ctx& c, uint64_t v) {
  if (c.nranks <= 1) return 0;
  if (!c.hubs_host.empty()) {
    auto it = std::lower_bound(c.hubs_host.begin(), c.hubs_host.end(), v);
    if (it != c.hubs_host.end() && *it == v) return static_cast<uint32_t>((it - c.hubs_host.begin()) % c.nranks);
  }
  return static_cast<uint32_t>(v % c.nranks);
}

// State by vertex id: T_pub, |M[v]| and the alive M entries (neighbour ids,
// rows in vertex-id order, entries in the row's order: neighbour-id order).
// The rows of S are packed on the device (pack_state: every member of S is an
// slist entry with T_pub != 0), so only the state map crosses PCIe.  A sharded
// context holds the replica of the whole state after its first superstep pair,
// so every shard exports everything.
static void export_state(Ctx& c, std::vector<uint16_t>& tpub, std::vector<uint32_t>& mdeg,
                         std::vector<uint32_t>& nbrs) {
  const uint64_t n = c.n;
  tpub.assign(n, 0);
  mdeg.assign(n, 0);
  nbrs.clear();
  if (!c.lcc_started || !c.nS_host) return;
  if (c.comm && !c.replicated) throw std::runtime_error("pm_export_state: the sharded state is not replicated yet");
  const uint64_t ne = pack_state_entry_bound(c);
  const uint64_t nr = pinned(c, 2)[0];
  uint32_t *d_rec = nullptr, *d_ent = nullptr;
  PM_HIP_CHECK(hipMalloc(&d_rec, std::max<uint64_t>(c.nS_host, 1) * 16));
  if (hipMalloc(&d_ent, std::max<uint64_t>(ne, 1) * 4) != hipSuccess) {
    (void)hipFree(d_rec);
    throw std::runtime_error("pm_export_state: out of device memory");
  }
  std::vector<uint32_t> rec(nr * 4), ent(ne);
  try {
    pack_state(c, d_rec, d_ent, ne, c.d_xcnt + 2);
    if (nr) PM_HIP_CHECK(hipMemcpyAsync(rec.data(), d_rec, nr * 16, hipMemcpyDeviceToHost, c.stream));
    if (ne) PM_HIP_CHECK(hipMemcpyAsync(ent.data(), d_ent, ne * 4, hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  } catch (...) {
    (void)hipFree(d_rec);
    (void)hipFree(d_ent);
    throw;
  }
  (void)hipFree(d_rec);
  (void)hipFree(d_ent);
  std::vector<uint64_t> at(n, ~0ull);
  for (uint64_t i = 0; i < nr; ++i) {
    const uint32_t v = c.perm_host[rec[4 * i]];
    tpub[v] = static_cast<uint16_t>(rec[4 * i + 1]);
    mdeg[v] = rec[4 * i + 2];
    at[v] = i;
  }
  for (uint64_t v = 0; v < n; ++v) {
    if (at[v] == ~0ull) continue;
    const uint32_t* r = rec.data() + 4 * at[v];
    for (uint32_t k = 0; k < r[2]; ++k) nbrs.push_back(c.perm_host[ent[r[3] + k] & kPosMask]);
  }
}

static void export_state_all(Ctx& c, std::vector<uint16_t>& tpub, std::vector<uint32_t>& mdeg,
                             std::vector<uint32_t>& nbrs) {
  export_state(c, tpub, mdeg, nbrs);
}

static void write_lines(const std::string& path, const std::vector<std::string>& lines) {
  std::ofstream f(path, std::ofstream::out);
  if (!f) throw std::runtime_error("cannot write " + path);
  for (const auto& l : lines) f << l << "\n";
}

// Subgraph lines "[r], w0, ..., wk, [wk]" of kept TDS walks (positions, `stride` per walk), into the file of
// the owner of the last vertex (tds_batch_1.hpp:739-743).
static void add_walk_lines(const Ctx& c, std::vector<std::vector<std::string>>& files, const uint32_t* walks,
                           uint64_t n, uint32_t stride) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t* w = walks + i * stride;
    const uint32_t last = c.perm_host[w[stride - 1]];
    const uint32_t r = owner_host(c, last);
    std::string l = "[" + std::to_string(r) + "], ";
    for (uint32_t p = 0; p < stride; ++p) l += std::to_string(c.perm_host[w[p]]) + ", ";
    l += "[" + std::to_string(last) + "]";
    files[r].push_back(std::move(l));
  }
}

// run_pattern_matching_beta.cpp:539-1425
// (diagnostics, PM_HOST_PROBES=1: the host's time between searches -- from the previous run_beta's return to
// this one's entry, its setup before the first launch, and its end after the last sync -- on stderr)
static std::chrono::steady_clock::time_point g_last_return{};
static double g_last_tail_us = 0;  // the previous search: its last probe ("end") to its return
static void run_beta(Ctx& c, const std::string& out_dir, uint64_t max_iterations, pm_run_stats* st) {
  const auto t_entry = std::chrono::steady_clock::now();
  static const bool host_probes = std::getenv("PM_HOST_PROBES") != nullptr;
  c.probes.clear();
  c.probing = host_probes || std::getenv("PM_PHASE_TIMES") != nullptr;
  c.probe("entry");
  const Pattern& P = c.pattern;
  const bool files = !out_dir.empty();
  static const bool build_lines_anyway = std::getenv("PM_BUILD_LINES") != nullptr;  // diagnostics (A/B)
  const bool lines_on = files || build_lines_anyway;
  reset_state(c, true);  // flushed with superstep 0's fills
  c.probe("reset");
  DriverFiles f;
  f.vcount.assign(c.nranks, {});
  f.ecount.assign(c.nranks, {});
  f.mcount.assign(c.nranks, {});
  std::vector<std::vector<std::vector<std::string>>> subgraphs(P.lines.size(),
                                                               std::vector<std::vector<std::string>>(c.nranks));
  pm_run_stats s{};
  const uint64_t comm_calls0 = c.comm ? c.comm->calls : 0, comm_bytes0 = c.comm ? c.comm->bytes : 0;
  if (c.comm) c.comm_wall0 = c.comm->wall;
  c.device_seconds = 0.0;
  c.lines_seconds = 0.0;
  // pattern_time_start (beta.cpp:539): the reset above is only enqueued; the
  // search's kernels follow it on the stream without a host round trip
  const auto t_pattern = std::chrono::steady_clock::now();
  c.probe("start");
  auto since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
  };
  bool init_step = true, nf = false, terminated = true;
  // PM_PHASE_TIMES=1: per-phase host wall time on stderr (diagnostics)
  const bool phase_times = std::getenv("PM_PHASE_TIMES") != nullptr;
  c.fine_timing = files || phase_times;
  c.probing = phase_times || host_probes;
  double ph_lcc = 0, ph_tp = 0, ph_post = 0, ph_count = 0;
  auto tick = [] { return std::chrono::steady_clock::now(); };
  uint64_t itr = 0;
  uint64_t first_scanned = 0, first_surv = 0, first_edges = 0, first_matching = 0;
  uint64_t last_v = 0, last_e = 0;
  auto totals = [&](const std::vector<uint64_t>& vc, const std::vector<uint64_t>& ec) {
    last_v = 0;
    last_e = 0;
    for (auto x : vc) last_v += x;
    for (auto x : ec) last_e += x;
  };
  // active vertex / edge counts per rank after the latest step
  std::vector<uint64_t> cur_vc(c.nranks, 0), cur_ec(c.nranks, 0);
  std::vector<uint64_t> loc_vc(c.nranks, 0), loc_ec(c.nranks, 0);  // this shard's share (sharded)
  auto record_lcc = [&](const LccOut& lo, uint64_t itr_) {
    loc_vc = lo.loc_vc;
    loc_ec = lo.loc_ec;
    c.live_hint = 0;
    for (auto x : loc_vc) c.live_hint += x;
    for (size_t ss = 0; ss < lo.seconds.size(); ++ss) {
      if (lines_on) {  // (result-file lines are built only when they are written)
        f.superstep.push_back(std::to_string(itr_) + ", LP, " + std::to_string(ss) + ", " + fmt_double(lo.seconds[ss]));
        add_count_lines(c, f, itr_, "LP", ss, lo.vcount[ss], lo.ecount[ss], lo.trav[ss]);
      }
      if (phase_times) {
        uint64_t sv = 0, se = 0;
        for (auto x : lo.vcount[ss]) sv += x;
        for (auto x : lo.ecount[ss]) se += x;
        std::fprintf(stderr, "[pm] LP itr %llu superstep %zu: |S| %llu, |M| %llu, traversed %llu, %.1f us\n",
                     static_cast<unsigned long long>(itr_), ss, static_cast<unsigned long long>(sv),
                     static_cast<unsigned long long>(se), static_cast<unsigned long long>(lo.trav[ss]),
                     lo.seconds[ss] * 1e6);
      }
      s.lcc_edges += lo.trav[ss];
      totals(lo.vcount[ss], lo.ecount[ss]);
      cur_vc = lo.vcount[ss];
      cur_ec = lo.ecount[ss];
    }
  };
  do {
    if (max_iterations && itr >= max_iterations) {
      terminated = false;
      break;
    }
    nf = false;
    const auto t_itr = std::chrono::steady_clock::now();
    const auto t_lp = std::chrono::steady_clock::now();
    const bool was_init = init_step;
    auto t0 = tick();
    // iteration 0 always runs the lines (beta.cpp:686-688): one shard enqueues them behind the LCC
    c.prelaunch_lines = itr == 0 && c.fused_lines && !P.lines.empty();
    LccOut lo = lcc_call(c, init_step);
    c.prelaunch_lines = false;
    ph_lcc += since(t0);
    if (was_init) {  // this shard's superstep-0 kernel (roofline bytes)
      first_scanned = c.ss0_trav;
      first_matching = lo.matching_rows;
      first_surv = lo.loc_surv;
      first_edges = lo.loc_edges;
    }
    record_lcc(lo, itr);
    if (was_init && c.shard == 0 && std::getenv("PM_DEBUG_STATE_DUMP")) {  // diagnostics: the state after it
      std::vector<uint16_t> tp;
      std::vector<uint32_t> md, nb;
      export_state(c, tp, md, nb);
      std::ofstream f(std::getenv("PM_DEBUG_STATE_DUMP"));
      uint64_t at = 0;
      for (uint64_t v = 0; v < c.n; ++v) {
        if (!tp[v]) continue;
        std::vector<uint32_t> row(nb.begin() + at, nb.begin() + at + md[v]);
        std::sort(row.begin(), row.end());
        f << v << " " << tp[v] << " :";
        for (auto x : row) f << " " << x;
        f << "\n";
        at += md[v];
      }
    }
    nf = nf || lo.not_finished;
    if (lines_on) f.step.push_back(std::to_string(itr) + ", LP, " + fmt_double(since(t_lp)));
    init_step = false;
    if (itr == 0) nf = true;  // forced token passing (beta.cpp:686-688)
    if (nf) {
      nf = false;
      // fused lines run in batches (one launch for consecutive lines, see
      // run_lines_fused); a line whose batch overflowed runs on the exact path
      std::vector<FusedLineOut> batch;
      size_t batch_pl0 = 0, exact_at = SIZE_MAX;
      for (size_t pl = 0; pl < P.lines.size(); ++pl) {
        const NlcLine& line = P.lines[pl];
        for (auto& r : subgraphs[pl]) r.clear();  // reopened with truncation (beta.cpp:713-717)
        const auto t_tp = std::chrono::steady_clock::now();
        TpResult tr;
        uint32_t deleted = 0;
        std::vector<uint64_t> vc, ec;
        std::vector<uint32_t> walks;
        uint32_t stride = 0;
        FusedLineOut fo;
        bool fused = false;
        auto t1 = tick();
        if (c.comm && !c.replicated) throw std::runtime_error("internal: NLC line before the sharded state was replicated");
        if (c.fused_lines && pl != exact_at) {
          if (pl < batch_pl0 || pl >= batch_pl0 + batch.size()) {
            for (;;) {
              bool overflow = false;
              const size_t n = run_lines_fused(c, pl, files, batch, overflow);
              s.line_overflows += overflow ? 1 : 0;
              batch_pl0 = pl;
              const bool regrown = c.hash_regrown;
              c.hash_regrown = false;
              if (overflow && !regrown) {  // (walk storage, or no room to grow the table)
                // one context: the line's sources in parts on the fused kernel (local_split_line), else the
                // exact path
                FusedLineOut lo;
                static const bool no_local = std::getenv("PM_LOCAL_SPLIT") && std::string(std::getenv("PM_LOCAL_SPLIT")) == "0";
                if (!no_local && !c.comm && pl + n < P.lines.size() && local_split_line(c, pl + n, files, lo)) {
                  if (phase_times)
                    std::fprintf(stderr, "[pm] line %zu: local split in %u parts\n", pl + n, c.local_split_parts);
                  batch.push_back(std::move(lo));
                } else {
                  exact_at = pl + n;
                }
              }
              if (!(overflow && regrown && n == 0)) break;   // the overflowed line reruns with the grown table
            }
          }
          if (pl >= batch_pl0 && pl < batch_pl0 + batch.size()) {
            fo = std::move(batch[pl - batch_pl0]);
            fused = true;
          }
        }
        if (fused) {
          tr = fo.tr;
          deleted = fo.deleted;
          s.split_lines += fo.split ? 1 : 0;
          vc = cur_vc;
          ec = cur_ec;
          for (uint32_t r = 0; r < c.nranks; ++r) {
            vc[r] -= fo.rm_v[r];
            ec[r] -= fo.rm_e[r];
          }
          walks.swap(fo.walks);
          stride = fo.stride;
          ph_tp += since(t1);
        } else {
          // exact-count path (one launch + sync per position)
          ++s.exact_lines;
          if (pl >= 4) {  // beta.cpp:762-767
            // the kept walks become subgraph lines chunk by chunk (the chunked enumeration bounds the device
            // memory, the lines are all the host keeps)
            tr = run_tds_line(c, line, stride, [&](const uint32_t* w, uint64_t nk) {
              if (lines_on) add_walk_lines(c, subgraphs[pl], w, nk, stride);
            });
            s.tds_chunks += c.last_tds_chunks;
          } else {
            tr = run_path_line(c, line);
            s.path_batches += tr.batches;
          }
          ph_tp += since(t1);
          auto t2 = tick();
          deleted = launch_post_tp(c, line);
          ph_post += since(t2);
          auto t3 = tick();
          count_state(c, vc, ec);
          ph_count += since(t3);
          c.lines_seconds += since(t1);
        }
        if (pl >= 4) {
          s.tds_edges += tr.edges;
          s.walks = tr.walks;
          if (stride) add_walk_lines(c, subgraphs[pl], walks.data(), walks.size() / stride, stride);
        } else {
          s.nlcc_edges += tr.edges;
        }
        if (deleted) nf = true;
        if (lines_on) {
          f.superstep.push_back(std::to_string(itr) + ", TP, " + std::to_string(pl) + ", " + fmt_double(since(t_tp)));
          add_count_lines(c, f, itr, "TP", pl, vc, ec, tr.edges);
        }
        totals(vc, ec);
        cur_vc = vc;
        cur_ec = ec;
        if (deleted && line.interleave_lp) {  // beta.cpp:1163-1197
          const auto t_lpi = std::chrono::steady_clock::now();
          LccOut li = lcc_call(c, false);
          record_lcc(li, itr);
          nf = nf || li.not_finished;
          if (lines_on) f.step.push_back(std::to_string(itr) + ", LP, " + fmt_double(since(t_lpi)));
        }
      }
    } else {
      nf = false;
    }
    if (lines_on) f.iteration.push_back(std::to_string(itr) + ", " + fmt_double(since(t_itr)));
    ++itr;
  } while (nf);
  c.probe("iterations done");
  stream_wait(c.stream);
  c.probe("end");
  const double secs = since(t_pattern);
  if (phase_times)
    std::fprintf(stderr, "[pm] run_beta %.3f ms: lcc %.3f, token passing %.3f, post %.3f, counts %.3f, device %.3f\n",
                 secs * 1e3, ph_lcc * 1e3, ph_tp * 1e3, ph_post * 1e3, ph_count * 1e3, c.device_seconds * 1e3);
  if ((phase_times || host_probes) && !c.probes.empty()) {
    std::string line = "[pm] host:";
    if (g_last_return.time_since_epoch().count()) {
      char buf[128];
      std::snprintf(buf, sizeof(buf), " (previous end to return %.1f, return to entry %.1f, entry to start %.1f)",
                    g_last_tail_us, std::chrono::duration<double>(t_entry - g_last_return).count() * 1e6,
                    (c.probes[0].second - std::chrono::duration<double>(t_entry.time_since_epoch()).count()) * 1e6);
      line += buf;
    }
    double prev = c.probes[0].second;
    for (const auto& pr : c.probes) {
      char buf[96];
      std::snprintf(buf, sizeof(buf), " %s +%.1f", pr.first, (pr.second - prev) * 1e6);
      line += buf;
      prev = pr.second;
    }
    std::fprintf(stderr, "%s us\n", line.c_str());
  }
  s.iterations = itr;
  s.terminated = terminated ? 1 : 0;
  s.hubs = static_cast<uint32_t>(c.hubs_host.size());
  s.nlcc_seconds = c.lines_seconds;
  s.seconds = secs;
  s.device_seconds = c.device_seconds;
  s.lcc_first_kernel_ms = c.lcc_first_ms;
  c.lcc_first_bytes = lcc_first_bytes(c, first_scanned, first_surv, first_edges, first_matching);
  s.lcc_first_bytes = c.lcc_first_bytes;
  s.final_vertices = last_v;
  s.final_edges = last_e;
  s.shard_entries = c.nnz;
  s.shard_rows = c.held_rows;
  s.shard_hub_entries = c.held_hub_entries;
  for (uint64_t j = c.shard; c.split_hubs && j < c.hubs_host.size(); j += c.nshards) ++s.shard_hubs_controlled;
  s.shard_ss0_entries = first_scanned;
  s.shard_ss0_survivors = first_surv;
  s.shard_sharded_ms = c.comm ? c.sharded_ms : 0.0;
  if (c.comm) {
    s.comm_calls = c.comm->calls - comm_calls0;
    s.comm_bytes = c.comm->bytes - comm_bytes0;
    s.comm_seconds = c.comm->wall - c.comm_wall0;
  }
  s.replica_rows = c.replica_rows;
  s.replica_entries = c.replica_entries;
  if (files) {
    // result dump (beta.cpp:1370-1425) -- after pattern_time_end, as in the reference
    std::vector<uint16_t> tpub;
    std::vector<uint32_t> mdeg, nbrs;
    export_state_all(c, tpub, mdeg, nbrs);
    if (c.shard != 0) {  // shard 0 writes every rank's files
      if (st) *st = s;
      return;
    }
    const std::string d = out_dir + "/0";
    const char* subdirs[] = {"all_ranks_active_vertices_count", "all_ranks_active_edges_count", "all_ranks_messages",
                             "all_ranks_active_vertices", "all_ranks_active_edges", "all_ranks_subgraphs",
                             "all_ranks_vertex_data"};
    for (auto sd : subdirs) mkdir_p(d + "/" + sd);
    write_lines(out_dir + "/result_pattern_set",
                {"0, " + std::to_string(c.nranks) + ", " + std::to_string(itr) + ", " + fmt_double(secs) + ", " +
                 std::to_string(P.graph.edge_count) + ", " + std::to_string(P.graph.vertex_count) + ", " +
                 std::to_string(P.lines.size())});
    write_lines(d + "/result_iteration", f.iteration);
    write_lines(d + "/result_step", f.step);
    write_lines(d + "/result_superstep", f.superstep);
    std::vector<std::vector<std::string>> av(c.nranks), ae(c.nranks);
    uint64_t pos = 0;
    for (uint64_t v = 0; v < c.n; ++v) {
      if (!tpub[v]) continue;
      const uint32_t r = owner_host(c, v);
      av[r].push_back(std::to_string(r) + ", " + std::to_string(v) + ", 0, " + std::to_string(c.labels_host[v]) + ", " +
                      std::bitset<16>(tpub[v]).to_string());
      for (uint32_t k = 0; k < mdeg[v]; ++k)
        ae[r].push_back(std::to_string(r) + ", " + std::to_string(v) + ", " + std::to_string(nbrs[pos + k]));
      pos += mdeg[v];
    }
    for (uint32_t r = 0; r < c.nranks; ++r) {
      const std::string rs = std::to_string(r);
      write_lines(d + "/all_ranks_active_vertices_count/active_vertices_" + rs, f.vcount[r]);
      write_lines(d + "/all_ranks_active_edges_count/active_edges_" + rs, f.ecount[r]);
      write_lines(d + "/all_ranks_messages/messages_" + rs, f.mcount[r]);
      write_lines(d + "/all_ranks_active_vertices/active_vertices_" + rs, av[r]);
      write_lines(d + "/all_ranks_active_edges/active_edges_" + rs, ae[r]);
      for (size_t pl = 0; pl < P.lines.size(); ++pl)
        write_lines(d + "/all_ranks_subgraphs/subgraphs_" + std::to_string(pl) + "_" + rs, subgraphs[pl][r]);
    }
  }
  if (st) *st = s;
  if (host_probes) {
    g_last_return = std::chrono::steady_clock::now();
    g_last_tail_us = c.probes.empty() ? 0.0
                                      : (std::chrono::duration<double>(g_last_return.time_since_epoch()).count() -
                                         c.probes.back().second) * 1e6;
  }
}

}  // namespace pm


extern "C" {

pm_ctx* pm_create(const pm_graph_desc* graph, const char* pattern_dir, int device) {
  try {
    return pm::create_ctx(graph, pattern_dir, device);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return nullptr;
  }
}

void pm_destroy(pm_ctx* ctx) {
  pm::gather_floor_forget(ctx ? static_cast<const void*>(static_cast<pm::Ctx*>(ctx)) : nullptr);
  pm::destroy_ctx(ctx);
}

const char* pm_last_error(const pm_ctx* ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return pm::g_last_error.c_str();
}

#define PM_API_BODY(ctx, ...)             \
  do {                                    \
    if (!(ctx)) return -1;                \
    try {                                 \
      (void)hipSetDevice((ctx)->device);  \
      __VA_ARGS__;                        \
      return 0;                           \
    } catch (const std::exception& e) {   \
      (ctx)->err = e.what();              \
      pm::g_last_error = e.what();        \
      return -1;                          \
    }                                     \
  } while (0)

int pm_vertex_data_degree(pm_ctx* ctx) {
  PM_API_BODY(ctx, {
    pm::set_degree_labels(*ctx);
    pm::relayout(*ctx);
  });
}

int pm_vertex_data_set(pm_ctx* ctx, const uint64_t* labels) {
  PM_API_BODY(ctx, {
    if (!labels) throw std::runtime_error("null labels");
    ctx->labels_host.assign(labels, labels + ctx->n);
    pm::relayout(*ctx);
  });
}

int pm_vertex_data_files(pm_ctx* ctx, const char* prefix) {
  PM_API_BODY(ctx, {
    if (!prefix) throw std::runtime_error("null label prefix");
    const std::vector<std::string> files = pm::vertex_label_files(prefix);
    uint64_t* d_labels = nullptr;  // (parsed on the device, kept on the host: the layout's input)
    PM_HIP_CHECK(hipMalloc(&d_labels, std::max<uint64_t>(ctx->n, 1) * sizeof(uint64_t)));
    try {
      pm::labels_from_files_device(files, ctx->n, d_labels, ctx->stream);
      ctx->labels_host.resize(ctx->n);
      PM_HIP_CHECK(hipMemcpyAsync(ctx->labels_host.data(), d_labels, ctx->n * sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, ctx->stream));
      PM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    } catch (...) {
      (void)hipFree(d_labels);
      throw;
    }
    (void)hipFree(d_labels);
    pm::relayout(*ctx);
  });
}

int pm_reset(pm_ctx* ctx) {
  PM_API_BODY(ctx, {
    pm::reset_state(*ctx);
  });
}

int pm_lcc_bsp(pm_ctx* ctx, int init_step, uint64_t itr, pm_lcc_stats* out) {
  (void)itr;
  PM_API_BODY(ctx, {
    pm::LccOut lo = pm::lcc_call(*ctx, init_step != 0);
    if (out) {
      *out = pm_lcc_stats{};
      out->supersteps = lo.seconds.size();
      for (auto t : lo.trav) out->edges_traversed += t;
      for (auto x : lo.vcount.back()) out->active_vertices += x;
      for (auto x : lo.ecount.back()) out->active_edges += x;
      out->not_finished = lo.not_finished ? 1 : 0;
    }
  });
}

int pm_token_passing(pm_ctx* ctx, uint32_t pl, pm_tp_stats* out) {
  PM_API_BODY(ctx, {
    if (ctx->comm) throw std::runtime_error("pm_token_passing: sharded contexts run lines through pm_run_beta");
    if (pl >= ctx->pattern.lines.size()) throw std::runtime_error("NLC line index out of range");
    const auto& line = ctx->pattern.lines[pl];
    pm::TpResult r;
    if (pl >= 4) {
      std::vector<uint32_t> walks;
      uint32_t stride = 0;
      r = pm::run_tds_line(*ctx, line, walks, stride);
    } else {
      r = pm::run_path_line(*ctx, line);
    }
    if (out) {
      out->sources = r.sources;
      out->acked_sources = 0;
      out->edges_traversed = r.edges;
      out->tokens = r.tokens;
      out->walks = r.walks;
    }
  });
}

int pm_tds(pm_ctx* ctx, uint32_t pl, pm_path_sink sink, void* user, pm_tp_stats* out) {
  PM_API_BODY(ctx, {
    if (ctx->comm) throw std::runtime_error("pm_tds: sharded contexts run lines through pm_run_beta");
    if (pl >= ctx->pattern.lines.size()) throw std::runtime_error("NLC line index out of range");
    if (pl < 4) throw std::runtime_error("pm_tds: line index below 4 is a path / cycle line (pm_token_passing)");
    // kept walks reach the sink chunk by chunk, in the enumeration's order
    uint32_t stride = 0;
    std::vector<uint32_t> ids;
    const pm::TpResult r = pm::run_tds_line(*ctx, ctx->pattern.lines[pl], stride,
                                            [&](const uint32_t* w, uint64_t n) {
                                              if (!sink) return;
                                              ids.resize(stride);
                                              for (uint64_t i = 0; i < n; ++i) {
                                                for (uint32_t p = 0; p < stride; ++p)
                                                  ids[p] = ctx->perm_host[w[i * stride + p]];
                                                sink(user, pm::owner_host(*ctx, ids[stride - 1]), ids.data(), stride);
                                              }
                                            });
    if (out) {
      out->sources = r.sources;
      out->acked_sources = 0;
      out->edges_traversed = r.edges;
      out->tokens = r.tokens;
      out->walks = r.walks;
    }
  });
}

int pm_post_token_passing(pm_ctx* ctx, uint32_t pl, uint32_t* deleted) {
  PM_API_BODY(ctx, {
    if (pl >= ctx->pattern.lines.size()) throw std::runtime_error("NLC line index out of range");
    const uint32_t d = pm::launch_post_tp(*ctx, ctx->pattern.lines[pl]);
    if (deleted) *deleted = d;
  });
}

int pm_run_beta(pm_ctx* ctx, const char* result_dir, uint64_t max_iterations, pm_run_stats* out) {
  PM_API_BODY(ctx, { pm::run_beta(*ctx, result_dir ? result_dir : "", max_iterations, out); });
}

int pm_export_state(pm_ctx* ctx, uint16_t* tpub, uint32_t* mdeg, uint32_t* nbrs, uint64_t* n_edges) {
  PM_API_BODY(ctx, {
    std::vector<uint16_t> t;
    std::vector<uint32_t> d, nb;
    pm::export_state_all(*ctx, t, d, nb);
    if (tpub) std::copy(t.begin(), t.end(), tpub);
    if (mdeg) std::copy(d.begin(), d.end(), mdeg);
    if (nbrs) std::copy(nb.begin(), nb.end(), nbrs);
    if (n_edges) *n_edges = nb.size();
  });
}

int pm_comm_unique_id(uint8_t* out, uint64_t len) {
  try {
    return static_cast<int>(pm::rccl_unique_id(out, len));
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_debug_rccl_selftest(int device, uint64_t bytes, int op) {
  try {
    return pm::rccl_selftest(device, bytes, op);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

pm_ctx* pm_create_shard(const pm_shard_desc* d, const char* pattern_dir, int device, const uint8_t* unique_id) {
  try {
    if (!d || !unique_id) throw std::runtime_error("pm_create_shard: null argument");
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    pm::CtxInput in;
    in.n = d->n;
    in.off = d->off;
    in.col = d->col;
    in.gdeg = d->degree;
    if (!in.gdeg) throw std::runtime_error("pm_create_shard: null degree array");
    in.symmetric = d->symmetric != 0;
    in.nranks = d->nranks;
    in.hub_threshold = d->hub_threshold;
    in.nshards = d->nshards;
    in.shard = d->shard;
    // the exchanges run whenever a communicator is present (also for one shard)
    in.comm = pm::make_rccl_comm(unique_id, static_cast<int>(d->nshards), static_cast<int>(d->shard));
    return pm::create_ctx(in, pattern_dir, device);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return nullptr;
  }
}

pm_ctx* pm_create_shard_host_comm(const pm_shard_desc* d, const char* pattern_dir, int device,
                                  const pm_host_comm* comm) {
  try {
    if (!d || !comm) throw std::runtime_error("pm_create_shard_host_comm: null argument");
    if (comm->nshards != d->nshards || comm->shard != d->shard)
      throw std::runtime_error("pm_create_shard_host_comm: communicator and shard disagree on nshards / shard");
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    pm::CtxInput in;
    in.n = d->n;
    in.off = d->off;
    in.col = d->col;
    in.gdeg = d->degree;
    if (!in.gdeg) throw std::runtime_error("pm_create_shard_host_comm: null degree array");
    in.symmetric = d->symmetric != 0;
    in.nranks = d->nranks;
    in.hub_threshold = d->hub_threshold;
    in.nshards = d->nshards;
    in.shard = d->shard;
    in.comm = pm::make_host_comm(*comm);
    return pm::create_ctx(in, pattern_dir, device);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return nullptr;
  }
}

// Every failed shard's message (a device fault is seen by whichever shard calls the runtime next; the shard
// whose work faulted names it in its own message).
static void throw_shard_errors(const std::vector<std::string>& errs) {
  std::string msg;
  for (size_t q = 0; q < errs.size(); ++q)
    if (!errs[q].empty() && errs[q] != "another shard failed")
      msg += (msg.empty() ? "" : " | ") + ("shard " + std::to_string(q) + ": " + errs[q]);
  if (msg.empty())
    for (size_t q = 0; q < errs.size() && msg.empty(); ++q)
      if (!errs[q].empty()) msg = "shard " + std::to_string(q) + ": " + errs[q];
  if (!msg.empty()) throw std::runtime_error(msg);
}

// PM_SEGV_TRACE=1: backtrace of a host crash inside the shard threads (diagnostics)
static void pm_segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "[pm] fatal signal, backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int pm_run_beta_local_shards2(const pm_graph_desc* g, const char* pattern_dir, int device, uint32_t nshards,
                              const uint64_t* labels, const char* label_prefix, const char* result_dir,
                              uint64_t max_iterations, uint32_t repeats, pm_run_stats* per_shard) {
  try {
    if (!g || !g->off || !g->col) throw std::runtime_error("pm_run_beta_local_shards: null graph");
    if (nshards == 0 || nshards > 64) throw std::runtime_error("pm_run_beta_local_shards: 1..64 shards");
    pm::require_gfx950(device);
    const uint64_t n = g->n;
    std::vector<uint32_t> gdeg(n);
    for (uint64_t v = 0; v < n; ++v) {
      const uint64_t d = g->off[v + 1] - g->off[v];
      if (d > 0xFFFFFFFFull) throw std::runtime_error("degree above 2^32");
      gdeg[v] = static_cast<uint32_t>(d);
    }
    // -v files: parsed on the device once, the same labels for every shard
    std::vector<uint64_t> file_labels;
    if (label_prefix) {
      PM_HIP_CHECK(hipSetDevice(device));
      const std::vector<std::string> files = pm::vertex_label_files(label_prefix);
      hipStream_t s = nullptr;
      uint64_t* d_labels = nullptr;
      try {
        PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        PM_HIP_CHECK(hipMalloc(&d_labels, std::max<uint64_t>(n, 1) * sizeof(uint64_t)));
        pm::labels_from_files_device(files, n, d_labels, s);
        file_labels.resize(n);
        if (n) PM_HIP_CHECK(hipMemcpyAsync(file_labels.data(), d_labels, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        PM_HIP_CHECK(hipStreamSynchronize(s));
      } catch (...) {
        if (d_labels) (void)hipFree(d_labels);
        if (s) (void)hipStreamDestroy(s);
        throw;
      }
      (void)hipFree(d_labels);
      (void)hipStreamDestroy(s);
      labels = file_labels.data();
    }
    if (std::getenv("PM_SEGV_TRACE")) signal(SIGSEGV, pm_segv_trace);
    pm::ThreadGroup grp(static_cast<int>(nshards));
    std::vector<pm_run_stats> st(nshards);
    std::vector<std::string> errs(nshards);
    const std::string dir = result_dir ? result_dir : "";
    auto work = [&](uint32_t q) {
      pm_ctx* ctx = nullptr;
      try {
        // this shard's rows, built on the host by every shard thread at once: shard q holds the rows of ids
        // v % nshards == q; a delegate's row (degree >= the hub threshold) is split by target owner -- shard q
        // holds its entries u with u % nshards == q (delegate_partitioned_graph.ipp:818-969, 1402-1648)
        std::vector<uint64_t> off(n + 1, 0);
        const bool split = nshards > 1;
        for (uint64_t v = 0; v < n; ++v) {
          uint64_t k = 0;
          if (split && gdeg[v] >= g->hub_threshold) {
            for (uint64_t e = g->off[v]; e < g->off[v + 1]; ++e) k += g->col[e] % nshards == q;
          } else if (v % nshards == q) {
            k = gdeg[v];
          }
          off[v + 1] = off[v] + k;
        }
        std::vector<uint32_t> col(std::max<uint64_t>(off[n], 1), 0);
        for (uint64_t v = 0; v < n; ++v) {
          if (off[v + 1] == off[v]) continue;
          uint32_t* out = col.data() + off[v];
          if (split && gdeg[v] >= g->hub_threshold) {
            for (uint64_t e = g->off[v]; e < g->off[v + 1]; ++e)
              if (g->col[e] % nshards == q) *out++ = g->col[e];
          } else {
            std::copy(g->col + g->off[v], g->col + g->off[v + 1], out);
          }
        }
        std::unique_lock<std::mutex> dev(grp.device);
        PM_HIP_CHECK(hipSetDevice(device));
        pm::CtxInput in;
        in.n = n;
        in.off = off.data();
        in.col = col.data();
        in.gdeg = gdeg.data();
        in.symmetric = g->symmetric != 0;
        in.nranks = g->nranks;
        in.hub_threshold = g->hub_threshold;
        in.nshards = nshards;
        in.shard = q;
        in.comm = pm::make_thread_comm(&grp, static_cast<int>(q));
        in.inprocess_shards = nshards;
        ctx = pm::create_ctx(in, pattern_dir, device);
        std::vector<uint64_t>().swap(off);  // (the context holds its copy)
        std::vector<uint32_t>().swap(col);
        if (labels) {
          ctx->labels_host.assign(labels, labels + n);
          pm::relayout(*ctx);
        }
        for (uint32_t r = 0; r < std::max<uint32_t>(repeats, 1); ++r)
          pm::run_beta(*ctx, r == 0 ? dir : std::string(), max_iterations, &st[q]);
        pm::destroy_ctx(ctx);  // (the device lock still held)
        ctx = nullptr;
      } catch (const std::exception& e) {
        errs[q] = e.what();
        grp.abort();
      }
      if (ctx) {
        std::lock_guard<std::mutex> dev(grp.device);
        pm::destroy_ctx(ctx);
      }
    };
    std::vector<std::thread> pool;
    for (uint32_t q = 0; q < nshards; ++q) pool.emplace_back(work, q);
    for (auto& t : pool) t.join();
    throw_shard_errors(errs);
    if (per_shard) std::copy(st.begin(), st.end(), per_shard);
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_run_beta_local_shards(const pm_graph_desc* g, const char* pattern_dir, int device, uint32_t nshards,
                             const uint64_t* labels, const char* result_dir, uint64_t max_iterations,
                             pm_run_stats* out) {
  if (nshards == 0 || nshards > 64) {
    pm::g_last_error = "pm_run_beta_local_shards: 1..64 shards";
    return -1;
  }
  std::vector<pm_run_stats> st(nshards);
  const int rc = pm_run_beta_local_shards2(g, pattern_dir, device, nshards, labels, nullptr, result_dir,
                                           max_iterations, 1, st.data());
  if (rc == 0 && out) *out = st[0];
  return rc;
}

int pm_rmat_edges(uint64_t scale, uint64_t p_gen, uint64_t first, uint64_t stride, uint32_t** src, uint32_t** dst,
                  uint64_t* m) {
  try {
    if (stride == 0) throw std::runtime_error("pm_rmat_edges: stride 0");
    std::vector<uint64_t> vr;
    for (uint64_t r = first; r < p_gen; r += stride) vr.push_back(r);
    if (p_gen == 0) throw std::runtime_error("P_gen must be positive");
    const uint64_t total = 2 * pm::rmat_edges_per_rank(scale, p_gen) * vr.size();
    uint32_t* s = static_cast<uint32_t*>(std::malloc(std::max<uint64_t>(1, total) * sizeof(uint32_t)));
    uint32_t* d = static_cast<uint32_t*>(std::malloc(std::max<uint64_t>(1, total) * sizeof(uint32_t)));
    if (!s || !d) {
      std::free(s);
      std::free(d);
      throw std::runtime_error("pm_rmat_edges: out of host memory");
    }
    try {
      *m = pm::rmat_stream_of(scale, p_gen, vr, [&](uint64_t i, uint32_t u, uint32_t v) {
        s[i] = u;
        d[i] = v;
      });
    } catch (...) {
      std::free(s);
      std::free(d);
      throw;
    }
    *src = s;
    *dst = d;
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_rmat_csr(uint64_t scale, uint64_t p_gen, uint64_t** off, uint32_t** col, uint64_t* n) {
  try {
    pm::Csr g = pm::build_rmat_csr(scale, p_gen);
    *n = g.n;
    *off = static_cast<uint64_t*>(std::malloc(g.off.size() * sizeof(uint64_t)));
    *col = static_cast<uint32_t*>(std::malloc(std::max<size_t>(1, g.col.size()) * sizeof(uint32_t)));
    std::memcpy(*off, g.off.data(), g.off.size() * sizeof(uint64_t));
    std::memcpy(*col, g.col.data(), g.col.size() * sizeof(uint32_t));
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

// GPU generator (pm_rmat.hip): the same CSR as pm_rmat_csr, built on `device`.
int pm_rmat_csr_gpu(uint64_t scale, uint64_t p_gen, int device, uint64_t** off, uint32_t** col, uint64_t* n) {
  hipStream_t s = nullptr;
  pm::DevCsr g;
  try {
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g = pm::rmat_csr_device(scale, p_gen, s);
    uint64_t* o = static_cast<uint64_t*>(std::malloc((g.n + 1) * sizeof(uint64_t)));
    uint32_t* c = static_cast<uint32_t*>(std::malloc(std::max<uint64_t>(1, g.nnz) * sizeof(uint32_t)));
    if (!o || !c) {
      std::free(o);
      std::free(c);
      throw std::runtime_error("pm_rmat_csr_gpu: out of host memory");
    }
    PM_HIP_CHECK(hipMemcpy(o, g.d_off, (g.n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (g.nnz) PM_HIP_CHECK(hipMemcpy(c, g.d_col, g.nnz * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *off = o;
    *col = c;
    *n = g.n;
    (void)hipFree(g.d_off);
    (void)hipFree(g.d_col);
    (void)hipStreamDestroy(s);
    return 0;
  } catch (const std::exception& e) {
    if (g.d_off) (void)hipFree(g.d_off);
    if (g.d_col) (void)hipFree(g.d_col);
    if (s) (void)hipStreamDestroy(s);
    pm::g_last_error = e.what();
    return -1;
  }
}

// Context over an R-MAT graph generated on the device itself (no host copy of
// the adjacency): the north_star S=28 one-GPU configuration.
pm_ctx* pm_create_rmat(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nranks,
                       uint64_t hub_threshold, double* gen_seconds) {
  hipStream_t s = nullptr;
  pm::DevCsr g;
  try {
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const auto t0 = std::chrono::steady_clock::now();
    g = pm::rmat_csr_device(scale, p_gen, s);
    if (gen_seconds) *gen_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<uint64_t> off(g.n + 1);
    PM_HIP_CHECK(hipMemcpy(off.data(), g.d_off, off.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    (void)hipFree(g.d_off);
    g.d_off = nullptr;
    pm::CtxInput in;
    in.n = g.n;
    in.off = off.data();
    in.col = g.d_col;
    in.col_on_device = true;
    in.col_release = true;  // the context frees the generated adjacency once it holds its copy
    g.d_col = nullptr;
    in.symmetric = true;
    in.nranks = nranks;
    in.hub_threshold = hub_threshold;
    pm_ctx* c = pm::create_ctx(in, pattern_dir, device);
    (void)hipStreamDestroy(s);
    return c;
  } catch (const std::exception& e) {
    if (g.d_off) (void)hipFree(g.d_off);
    if (g.d_col) (void)hipFree(g.d_col);
    if (s) (void)hipStreamDestroy(s);
    pm::g_last_error = e.what();
    return nullptr;
  }
}

}  // extern "C"

namespace pm {
// HBM copy bandwidth (the measured ceiling beside the 8 TB/s datasheet peak): 16-B nontemporal loads
// and stores, four in flight per lane, a grid of resident blocks.
typedef uint32_t cp_u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void k_copy16(const cp_u32x4* __restrict__ src, cp_u32x4* __restrict__ dst,
                                                uint64_t n) {
  const uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
  else dst[i] = src[i];
}
}  // namespace pm

extern "C" {
int pm_debug_copy_gbs(int device, uint64_t bytes, int reps, double* gbs) {
  void *a = nullptr, *b = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  try {
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    const uint64_t n = std::max<uint64_t>(bytes / 16, 1);
    PM_HIP_CHECK(hipMalloc(&a, n * 16));
    PM_HIP_CHECK(hipMalloc(&b, n * 16));
    PM_HIP_CHECK(hipMemset(a, 1, n * 16));
    PM_HIP_CHECK(hipEventCreate(&e0));
    PM_HIP_CHECK(hipEventCreate(&e1));
    // one 16-B element per thread, the whole buffer in one grid; the faster of plain and nontemporal
    const unsigned grid = static_cast<unsigned>((n + 255) / 256);
    float best = 0.f;
    for (int nt = 0; nt < 2; ++nt) {
      auto launch = [&] {
        if (nt)
          hipLaunchKernelGGL(pm::k_copy16<true>, dim3(grid), dim3(256), 0, 0, static_cast<const pm::cp_u32x4*>(a),
                             static_cast<pm::cp_u32x4*>(b), n);
        else
          hipLaunchKernelGGL(pm::k_copy16<false>, dim3(grid), dim3(256), 0, 0, static_cast<const pm::cp_u32x4*>(a),
                             static_cast<pm::cp_u32x4*>(b), n);
      };
      launch();  // warm
      PM_HIP_CHECK(hipEventRecord(e0, 0));
      for (int r = 0; r < std::max(reps, 1); ++r) launch();
      PM_HIP_CHECK(hipEventRecord(e1, 0));
      PM_HIP_CHECK(hipEventSynchronize(e1));
      float t = 0.f;
      PM_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
      if (best == 0.f || t < best) best = t;
    }
    const float ms = best;
    if (gbs) *gbs = 2.0 * n * 16 * std::max(reps, 1) / (ms * 1e-3) / 1e9;  // read + write bytes
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
  } catch (const std::exception& e) {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    pm::g_last_error = e.what();
    return -1;
  }
}
}  // extern "C"

namespace pm {
// One shard of the R-MAT graph built on the device (pm_rmat.hip rmat_shard_device) and its context;
// the communicator passes to the context.
static pm_ctx* create_rmat_shard_ctx(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device,
                                     uint32_t nranks, uint64_t hub_threshold, uint32_t nshards, uint32_t shard,
                                     Comm* comm, uint32_t inprocess, double* gen_seconds) {
  std::unique_ptr<Comm> owned(comm);
  hipStream_t s = nullptr;
  DevCsr g;
  try {
    require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> gdeg;
    g = rmat_shard_device(scale, p_gen, hub_threshold, *comm, nshards, shard, gdeg, s);
    if (gen_seconds) *gen_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<uint64_t> off(g.n + 1);
    PM_HIP_CHECK(hipMemcpy(off.data(), g.d_off, off.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    (void)hipFree(g.d_off);
    g.d_off = nullptr;
    CtxInput in;
    in.n = g.n;
    in.off = off.data();
    in.col = g.d_col;
    in.col_on_device = true;
    in.col_release = true;  // freed by the context once copied (in-process shards: before the next shard builds)
    g.d_col = nullptr;
    in.gdeg = gdeg.data();
    in.symmetric = true;
    in.nranks = nranks;
    in.hub_threshold = hub_threshold;
    in.nshards = nshards;
    in.shard = shard;
    in.comm = owned.release();
    in.inprocess_shards = inprocess;
    pm_ctx* c = create_ctx(in, pattern_dir, device);
    (void)hipStreamDestroy(s);
    return c;
  } catch (...) {
    if (g.d_off) (void)hipFree(g.d_off);
    if (g.d_col) (void)hipFree(g.d_col);
    if (s) (void)hipStreamDestroy(s);
    throw;
  }
}
}  // namespace pm

extern "C" {
pm_ctx* pm_create_rmat_shard(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nranks,
                             uint64_t hub_threshold, uint32_t nshards, uint32_t shard, const uint8_t* unique_id,
                             double* gen_seconds) {
  try {
    if (!unique_id) throw std::runtime_error("pm_create_rmat_shard: null communicator id");
    PM_HIP_CHECK(hipSetDevice(device));
    pm::Comm* comm = pm::make_rccl_comm(unique_id, static_cast<int>(nshards), static_cast<int>(shard));
    return pm::create_rmat_shard_ctx(scale, p_gen, pattern_dir, device, nranks, hub_threshold, nshards, shard, comm, 1,
                                     gen_seconds);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return nullptr;
  }
}

int pm_run_rmat_local_shards2(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nshards,
                              uint32_t nranks, uint64_t hub_threshold, const uint64_t* labels, const char* result_dir,
                              uint64_t max_iterations, uint32_t repeats, pm_run_stats* per_shard) {
  try {
    if (nshards == 0 || nshards > 64) throw std::runtime_error("pm_run_rmat_local_shards: 1..64 shards");
    pm::ThreadGroup grp(static_cast<int>(nshards));
    std::vector<pm_run_stats> st(nshards);
    std::vector<std::string> errs(nshards);
    const std::string dir = result_dir ? result_dir : "";
    auto work = [&](uint32_t q) {
      std::unique_lock<std::mutex> dev(grp.device);
      pm_ctx* ctx = nullptr;
      try {
        PM_HIP_CHECK(hipSetDevice(device));
        ctx = pm::create_rmat_shard_ctx(scale, p_gen, pattern_dir, device, nranks, hub_threshold, nshards, q,
                                        pm::make_thread_comm(&grp, static_cast<int>(q)), nshards, nullptr);
        if (labels) {
          ctx->labels_host.assign(labels, labels + ctx->n);
          pm::relayout(*ctx);
        }
        for (uint32_t r = 0; r < std::max<uint32_t>(repeats, 1); ++r)
          pm::run_beta(*ctx, r == 0 ? dir : std::string(), max_iterations, &st[q]);
      } catch (const std::exception& e) {
        errs[q] = e.what();
        grp.abort();
      }
      if (ctx) pm::destroy_ctx(ctx);
    };
    std::vector<std::thread> pool;
    for (uint32_t q = 0; q < nshards; ++q) pool.emplace_back(work, q);
    for (auto& t : pool) t.join();
    throw_shard_errors(errs);
    if (per_shard) std::copy(st.begin(), st.end(), per_shard);
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_run_rmat_local_shards(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nshards,
                             uint32_t nranks, uint64_t hub_threshold, const char* result_dir, uint64_t max_iterations,
                             pm_run_stats* out) {
  if (nshards == 0 || nshards > 64) {
    pm::g_last_error = "pm_run_rmat_local_shards: 1..64 shards";
    return -1;
  }
  std::vector<pm_run_stats> st(nshards);
  const int rc = pm_run_rmat_local_shards2(scale, p_gen, pattern_dir, device, nshards, nranks, hub_threshold, nullptr,
                                           result_dir, max_iterations, 1, st.data());
  if (rc == 0 && out) *out = st[0];
  return rc;
}

static std::vector<std::string> file_list(const char* const* files, uint32_t nfiles) {
  if (nfiles && !files) throw std::runtime_error("null file list");
  std::vector<std::string> v;
  for (uint32_t i = 0; i < nfiles; ++i) {
    if (!files[i]) throw std::runtime_error("null file name");
    v.emplace_back(files[i]);
  }
  return v;
}

static void free_dev_csr(pm::DevCsr& g) {
  if (g.d_off) (void)hipFree(g.d_off);
  if (g.d_col) (void)hipFree(g.d_col);
  g.d_off = nullptr;
  g.d_col = nullptr;
}

// GPU text ingest (pm_ingest.hip): the CSR ingest_edge_list builds, returned to the host.
int pm_ingest_edge_list_gpu(const char* const* files, uint32_t nfiles, int undirected, int device, uint64_t** off,
                            uint32_t** col, uint64_t* n, int* symmetric) {
  hipStream_t s = nullptr;
  pm::IngestCsr g;
  try {
    if (!off || !col || !n) throw std::runtime_error("null output");
    const std::vector<std::string> fl = file_list(files, nfiles);
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g = pm::ingest_edges_device(fl, undirected != 0, false, s);
    uint64_t* o = static_cast<uint64_t*>(std::malloc((g.fwd.n + 1) * sizeof(uint64_t)));
    uint32_t* c = static_cast<uint32_t*>(std::malloc(std::max<uint64_t>(1, g.fwd.nnz) * sizeof(uint32_t)));
    if (!o || !c) {
      std::free(o);
      std::free(c);
      throw std::runtime_error("pm_ingest_edge_list_gpu: out of host memory");
    }
    PM_HIP_CHECK(hipMemcpy(o, g.fwd.d_off, (g.fwd.n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (g.fwd.nnz) PM_HIP_CHECK(hipMemcpy(c, g.fwd.d_col, g.fwd.nnz * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *off = o;
    *col = c;
    *n = g.fwd.n;
    if (symmetric) *symmetric = g.symmetric ? 1 : 0;
    free_dev_csr(g.fwd);
    free_dev_csr(g.rev);
    (void)hipStreamDestroy(s);
    return 0;
  } catch (const std::exception& e) {
    free_dev_csr(g.fwd);
    free_dev_csr(g.rev);
    if (s) (void)hipStreamDestroy(s);
    pm::g_last_error = e.what();
    return -1;
  }
}

// Context over a graph ingested from text on the device (the adjacency never
// leaves HBM; a directed graph's in-rows come from the same sort).
pm_ctx* pm_create_edge_list(const char* const* files, uint32_t nfiles, int undirected, const char* pattern_dir,
                            int device, uint32_t nranks, uint64_t hub_threshold, double* ingest_seconds) {
  hipStream_t s = nullptr;
  pm::IngestCsr g;
  try {
    const std::vector<std::string> fl = file_list(files, nfiles);
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const auto t0 = std::chrono::steady_clock::now();
    g = pm::ingest_edges_device(fl, undirected != 0, true, s);
    if (ingest_seconds)
      *ingest_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<uint64_t> off(g.fwd.n + 1), roff;
    PM_HIP_CHECK(hipMemcpy(off.data(), g.fwd.d_off, off.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    pm::CtxInput in;
    in.n = g.fwd.n;
    in.off = off.data();
    in.col = g.fwd.d_col;
    in.col_on_device = true;
    in.symmetric = g.symmetric;
    in.nranks = nranks;
    in.hub_threshold = hub_threshold;
    if (!g.symmetric) {
      roff.resize(g.rev.n + 1);
      PM_HIP_CHECK(hipMemcpy(roff.data(), g.rev.d_off, roff.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      in.in_off = roff.data();
      in.in_col = g.rev.d_col;
    }
    pm_ctx* c = pm::create_ctx(in, pattern_dir, device);
    free_dev_csr(g.fwd);
    free_dev_csr(g.rev);
    (void)hipStreamDestroy(s);
    return c;
  } catch (const std::exception& e) {
    free_dev_csr(g.fwd);
    free_dev_csr(g.rev);
    if (s) (void)hipStreamDestroy(s);
    pm::g_last_error = e.what();
    return nullptr;
  }
}

int pm_graph_size(const pm_ctx* ctx, uint64_t* n, uint64_t* nnz, int* symmetric) {
  if (!ctx) return -1;
  if (n) *n = ctx->n;
  if (nnz) *nnz = ctx->nnz;
  if (symmetric) *symmetric = ctx->symmetric ? 1 : 0;
  return 0;
}

// Host check of the MT19937 jump-ahead machinery (host/mt_jump.hpp): the
// first `count` outputs of std::mt19937(seed) after skipping `skip` outputs,
// obtained by one polynomial jump instead of stepping.
int pm_mt19937_jump_outputs(uint32_t seed, uint64_t skip, uint32_t* out, uint64_t count) {
  try {
    uint32_t w[pm::mtj::kN], wj[pm::mtj::kN];
    pm::mtj::seed_window(seed, w);
    pm::mtj::apply(pm::mtj::jump_poly(skip), w, wj);
    std::vector<uint32_t> seq(pm::mtj::kN + count);
    pm::mtj::extend(wj, seq.data(), seq.size());
    for (uint64_t i = 0; i < count; ++i) out[i] = pm::mtj::temper(seq[pm::mtj::kN + i]);
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

void pm_free_host(void* p) { std::free(p); }

int pm_write_graph(const char* base, uint64_t n, const uint64_t* off, const uint32_t* col, int symmetric,
                   uint32_t nranks, uint64_t hub_threshold) {
  try {
    pm::Csr g;
    g.n = n;
    g.off.assign(off, off + n + 1);
    g.col.assign(col, col + off[n]);
    g.symmetric = symmetric != 0;
    pm::write_graph_files(base, g, nranks, hub_threshold);
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_read_graph(const char* base, uint64_t** off, uint32_t** col, uint64_t* n, int* symmetric, uint32_t* nranks,
                  uint64_t* hub_threshold) {
  try {
    uint32_t p = 1;
    uint64_t h = 0;
    pm::Csr g = pm::read_graph_files(base, &p, &h);
    *n = g.n;
    *off = static_cast<uint64_t*>(std::malloc(g.off.size() * sizeof(uint64_t)));
    *col = static_cast<uint32_t*>(std::malloc(std::max<size_t>(1, g.col.size()) * sizeof(uint32_t)));
    std::memcpy(*off, g.off.data(), g.off.size() * sizeof(uint64_t));
    std::memcpy(*col, g.col.data(), g.col.size() * sizeof(uint32_t));
    if (symmetric) *symmetric = g.symmetric ? 1 : 0;
    if (nranks) *nranks = p;
    if (hub_threshold) *hub_threshold = h;
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_graph_partitions(const char* base) {
  try {
    if (!base) throw std::runtime_error("pm_graph_partitions: null base");
    const uint32_t p = pm::graph_file_partitions(base);
    if (p == 0) throw std::runtime_error(std::string("no graph files found for base ") + base);
    return static_cast<int>(p);
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_read_graph_shard(const char* base, uint32_t nshards, uint32_t shard, uint64_t** off, uint32_t** col,
                        uint32_t** degree, uint64_t* n, int* symmetric, uint32_t* nranks, uint64_t* hub_threshold) {
  try {
    if (!base || !off || !col || !degree || !n) throw std::runtime_error("pm_read_graph_shard: null argument");
    pm::ShardCsr s = pm::read_graph_shard(base, nshards, shard);
    auto* o = static_cast<uint64_t*>(std::malloc(s.off.size() * sizeof(uint64_t)));
    auto* c = static_cast<uint32_t*>(std::malloc(s.col.size() * sizeof(uint32_t)));
    auto* d = static_cast<uint32_t*>(std::malloc(std::max<size_t>(1, s.degree.size()) * sizeof(uint32_t)));
    if (!o || !c || !d) {
      std::free(o);
      std::free(c);
      std::free(d);
      throw std::runtime_error("pm_read_graph_shard: out of host memory");
    }
    std::memcpy(o, s.off.data(), s.off.size() * sizeof(uint64_t));
    std::memcpy(c, s.col.data(), s.col.size() * sizeof(uint32_t));
    std::memcpy(d, s.degree.data(), s.degree.size() * sizeof(uint32_t));
    *off = o;
    *col = c;
    *degree = d;
    *n = s.n;
    if (symmetric) *symmetric = s.symmetric ? 1 : 0;
    if (nranks) *nranks = s.nranks;
    if (hub_threshold) *hub_threshold = s.hub_threshold;
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_device_count(void) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return count;
}

int pm_comm_info(const pm_ctx* ctx, uint32_t* nshards, uint32_t* shard, int32_t* comm_ranks, int32_t* transport) {
  if (!ctx) return -1;
  try {
    if (nshards) *nshards = ctx->nshards;
    if (shard) *shard = ctx->shard;
    if (comm_ranks) *comm_ranks = ctx->comm ? ctx->comm->ranks() : 0;
    if (transport) *transport = ctx->comm ? ctx->comm->transport() : PM_TRANSPORT_NONE;
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

const char* pm_build_arch(void) { return "gfx950"; }

}  // extern "C"

namespace {

// Decimal text of x at p (no terminator); returns the end.
inline char* put_u64(char* p, uint64_t x) {
  char tmp[20];
  int k = 0;
  do {
    tmp[k++] = static_cast<char>('0' + x % 10);
    x /= 10;
  } while (x);
  while (k) *p++ = tmp[--k];
  return p;
}

// Lines "a[i] b[i]\n" (b == nullptr: "i a[i]\n") for i in [0, n), formatted by host threads into
// per-chunk buffers and written in order to f.
uint64_t write_pairs_text(std::FILE* f, const uint64_t* a, const uint64_t* b, uint64_t n, uint64_t id0) {
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  constexpr uint64_t kChunk = 1ull << 22;  // lines per chunk (<= 42 bytes each)
  uint64_t total = 0;
  std::vector<std::vector<char>> buf(T, std::vector<char>(kChunk * 42));
  std::vector<uint64_t> len(T);
  for (uint64_t c0 = 0; c0 < n; c0 += kChunk * T) {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        const uint64_t b0 = c0 + t * kChunk, e0 = std::min(n, b0 + kChunk);
        char* p = buf[t].data();
        for (uint64_t i = b0; i < e0; ++i) {
          p = put_u64(p, b ? a[i] : id0 + i);
          *p++ = ' ';
          p = put_u64(p, b ? b[i] : a[i]);
          *p++ = '\n';
        }
        len[t] = b0 < e0 ? static_cast<uint64_t>(p - buf[t].data()) : 0;
      });
    for (auto& x : th) x.join();
    for (unsigned t = 0; t < T; ++t) {
      if (len[t] && std::fwrite(buf[t].data(), 1, len[t], f) != len[t]) throw std::runtime_error("text write failed");
      total += len[t];
    }
  }
  return total;
}

}  // namespace

extern "C" {

int pm_write_rmat_text(uint64_t scale, uint64_t p_gen, int device, const char* base, uint64_t* bytes_out) {
  hipStream_t s = nullptr;
  uint64_t* d_keys = nullptr;
  try {
    if (!base || !p_gen || scale == 0 || scale > 32) throw std::runtime_error("pm_write_rmat_text: bad arguments");
    pm::require_gfx950(device);
    PM_HIP_CHECK(hipSetDevice(device));
    PM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const pm::RmatPlan plan = pm::rmat_plan(scale, p_gen);
    PM_HIP_CHECK(hipMalloc(&d_keys, std::max<uint64_t>(2 * plan.per_rank, 1) * sizeof(uint64_t)));
    std::vector<uint64_t> keys(2 * plan.per_rank), u(plan.per_rank), v(plan.per_rank);
    const uint64_t mask = (uint64_t(1) << scale) - 1;
    uint64_t total = 0;
    for (uint64_t r = 0; r < p_gen; ++r) {
      pm::rmat_keys_device(plan, {r}, d_keys, s);  // keys 2k = (u << S | v), 2k + 1 = (v << S | u)
      PM_HIP_CHECK(hipMemcpy(keys.data(), d_keys, keys.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      for (uint64_t k = 0; k < plan.per_rank; ++k) {
        u[k] = keys[2 * k] >> scale;
        v[k] = keys[2 * k] & mask;
      }
      const std::string path = std::string(base) + "." + std::to_string(r);
      std::FILE* f = std::fopen(path.c_str(), "wb");
      if (!f) throw std::runtime_error("cannot write " + path);
      try {
        total += write_pairs_text(f, u.data(), v.data(), plan.per_rank, 0);
      } catch (...) {
        std::fclose(f);
        throw;
      }
      if (std::fclose(f) != 0) throw std::runtime_error("cannot close " + path);
    }
    (void)hipFree(d_keys);
    (void)hipStreamDestroy(s);
    if (bytes_out) *bytes_out = total;
    return 0;
  } catch (const std::exception& e) {
    if (d_keys) (void)hipFree(d_keys);
    if (s) (void)hipStreamDestroy(s);
    pm::g_last_error = e.what();
    return -1;
  }
}

int pm_write_label_text(const uint64_t* labels, uint64_t n, const char* prefix, uint32_t nfiles, uint64_t* bytes_out) {
  try {
    if (!labels || !prefix || !nfiles) throw std::runtime_error("pm_write_label_text: bad arguments");
    uint64_t total = 0;
    const uint64_t per = (n + nfiles - 1) / nfiles;
    for (uint32_t i = 0; i < nfiles; ++i) {
      const uint64_t b = std::min<uint64_t>(n, uint64_t(i) * per), e = std::min<uint64_t>(n, b + per);
      const std::string path = std::string(prefix) + "." + std::to_string(i);
      std::FILE* f = std::fopen(path.c_str(), "wb");
      if (!f) throw std::runtime_error("cannot write " + path);
      try {
        total += write_pairs_text(f, labels + b, nullptr, e - b, b);
      } catch (...) {
        std::fclose(f);
        throw;
      }
      if (std::fclose(f) != 0) throw std::runtime_error("cannot close " + path);
    }
    if (bytes_out) *bytes_out = total;
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

// Diagnostics: times `reps` launches of the superstep-0 kernel on the current
// labels (state is reset first).  variant & 0xFFFF: the kernel variant (0 the
// product; diagnostic MODEs and register / pairing variants in libpm_diag.so),
// dense M whenever light tiles run, as in the product; variant >> 16: the grid
// in blocks (0: the product grid).
int pm_debug_time_lcc_first(pm_ctx* ctx, int variant, int reps, float* ms_out) {
  PM_API_BODY(ctx, {
    pm::reset_state(*ctx);
    hipEvent_t a, b;
    PM_HIP_CHECK(hipEventCreate(&a));
    PM_HIP_CHECK(hipEventCreate(&b));
    // variant = kernel variant | grid << 16 (grid 0: the product grid)
    const unsigned grid = (variant >> 16) ? std::min<unsigned>(static_cast<unsigned>(variant >> 16), pm::kPartGridMax)
                                          : ctx->k1_grid;
    const int mode = variant & 0xFFFF;
    const bool dense = !(mode & 2);
    pm::ensure_counts(*ctx, 1);
    pm::lcc_first_prepare(*ctx);
    // the product launch writes dense M when the search would
    if (dense) pm::lcc_first_set_dense(*ctx);
    pm::launch_lcc_first_kernel(*ctx, mode, grid, ctx->d_counts);  // warm (partials not reduced)
    // each timed launch starts from cleared heavy-row tickets (the last segment of a heavy row runs its
    // verify), the memsets outside the events
    float total = 0.f;
    for (int i = 0; i < reps; ++i) {
      pm::lcc_first_prepare(*ctx);
      PM_HIP_CHECK(hipMemsetAsync(ctx->d_tcode, 0, pm::tcode_words(ctx->lr) * sizeof(uint32_t), ctx->stream));
      if (dense) pm::lcc_first_set_dense(*ctx);
      PM_HIP_CHECK(hipEventRecord(a, ctx->stream));
      pm::launch_lcc_first_kernel(*ctx, mode, grid, ctx->d_counts);
      PM_HIP_CHECK(hipEventRecord(b, ctx->stream));
      PM_HIP_CHECK(hipEventSynchronize(b));
      float ms = 0.f;
      PM_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    if (ms_out) *ms_out = total / std::max(1, reps);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    ctx->k1_dense = false;
    ctx->tpub_clean = false;  // the timed launches wrote T_pub outside any search
    pm::reset_state(*ctx);
  });
}

// Diagnostics: superstep-0 tiling of the current labels: out[0] real adjacency
// entries of the scanned runs, [1] slots loaded (padding included), [2]
// scanned rows, [3] tiles, [4] ranges, [5] heavy rows, [6] microseconds of
// the last label-major layout + tiling build (one-time, outside any search).
int pm_debug_layout_stats(pm_ctx* ctx, uint64_t* out, uint64_t n) {
  PM_API_BODY(ctx, {
    uint64_t st[7] = {0, 0, 0, ctx->ntiles, ctx->ktab.empty() ? 0 : ctx->ktab.size() - 1, ctx->nheavy,
                      static_cast<uint64_t>(ctx->layout_seconds * 1e6)};
    std::vector<uint64_t> offp(ctx->n + 1), offr(ctx->n + 1);
    PM_HIP_CHECK(hipMemcpy(offp.data(), ctx->d_offp, offp.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    PM_HIP_CHECK(hipMemcpy(offr.data(), ctx->d_offr, offr.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (size_t i = 0; i + 1 < ctx->ktab.size(); ++i) {
      const pm::KRange& R = ctx->ktab[i];
      st[0] += offr[R.end] - offr[R.start];
      st[1] += offp[R.end] - offp[R.start];
      st[2] += R.end - R.start;
    }
    for (uint64_t i = 0; i < n && i < 7; ++i) out[i] = st[i];
  });
}

int pm_debug_tpub_census(pm_ctx* ctx, int deferred_reset, uint64_t* out) {
  PM_API_BODY(ctx, {
    if (!out) throw std::runtime_error("null output");
    if (deferred_reset) {
      pm::reset_state(*ctx, true);
      pm::flush_zero(*ctx);
    }
    const uint64_t n = ctx->n;
    std::vector<uint16_t> t0(n), t1(n);
    uint32_t ns = 0;
    PM_HIP_CHECK(hipMemcpyAsync(t0.data(), ctx->d_tpub[0], n * sizeof(uint16_t), hipMemcpyDeviceToHost, ctx->stream));
    PM_HIP_CHECK(hipMemcpyAsync(t1.data(), ctx->d_tpub[1], n * sizeof(uint16_t), hipMemcpyDeviceToHost, ctx->stream));
    PM_HIP_CHECK(hipMemcpyAsync(&ns, ctx->d_nS, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
    PM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    std::vector<uint32_t> sl(ns);
    if (ns) PM_HIP_CHECK(hipMemcpy(sl.data(), ctx->d_slist, ns * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint8_t> in(n, 0);
    for (uint32_t p : sl)
      if (p < n) in[p] = 1;
    out[0] = out[1] = out[2] = 0;
    for (uint64_t p = 0; p < n; ++p) {
      out[0] += t0[p] != 0;
      out[1] += t1[p] != 0;
      out[2] += (t0[p] || t1[p]) && !in[p];
    }
  });
}

int pm_pattern_summary(const char* pattern_dir, char* buf, uint64_t buflen) {
  try {
    const pm::Pattern p = pm::load_pattern_dir(pattern_dir);
    std::ostringstream o;
    auto vec = [&o](const std::vector<uint64_t>& v) {
      o << "[";
      for (size_t i = 0; i < v.size(); ++i) o << (i ? "," : "") << v[i];
      o << "]";
    };
    o << "{\"vertex_count\":" << p.graph.vertex_count << ",\"edge_count\":" << p.graph.edge_count
      << ",\"diameter\":" << p.graph.diameter << ",\"vertices\":";
    vec(p.graph.vertices);
    o << ",\"edges\":";
    vec(p.graph.edges);
    o << ",\"vertex_data\":";
    vec(p.graph.vertex_data);
    o << ",\"adj\":[";
    for (size_t t = 0; t < p.graph.vertex_data.size(); ++t) o << (t ? "," : "") << p.graph.adj[t];
    o << "],\"lines\":[";
    for (size_t i = 0; i < p.lines.size(); ++i) {
      const auto& l = p.lines[i];
      o << (i ? "," : "") << "{\"labels\":";
      vec(l.labels);
      o << ",\"indices\":";
      vec(l.indices);
      o << ",\"C\":" << l.cycle_length << ",\"VC\":" << l.valid_cycle << ",\"IL\":" << l.interleave_lp
        << ",\"SV\":" << l.selected_vertices << ",\"enumeration\":";
      vec(l.enumeration);
      o << "}";
    }
    o << "]}";
    const std::string s = o.str();
    if (s.size() + 1 > buflen) throw std::runtime_error("summary buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return 0;
  } catch (const std::exception& e) {
    pm::g_last_error = e.what();
    return -1;
  }
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------------------
// Diagnostics: the floor of the first later superstep's neighbour-T_pub gathers.  The gathers
// of the S=28 first later superstep: one 2-bit code per alive M entry of the superstep-0 survivors, read from the
// code array (tcode, ~22 MB) at the entry's code index.  pm_debug_gather_floor runs superstep 0 (product kernel,
// dense M + records), collects the light survivors' M entries as code indices in record order (the order the
// superstep reads them), and times gather-only kernels over them:
//   0  record order: the entry's index read (coalesced) + its code word gathered, 4 entries in flight per lane
//   1  the index stream alone (no gather)
//   2  XCD-sliced: entries bucketed (untimed) into eight code ranges of an eighth of the entries each; workgroup b
//      takes bucket b % 8 (workgroups are dealt to the 8 XCDs round-robin), so each XCD's gathers stay inside its
//      own range of the code array
//   3  the same buckets, each spread over every XCD (bucket (b / 8) % 8): the XCD placement alone
//   4  the same number of gathers, uniformly random over the code array (index hashed, no index stream)
//   5  the entries sorted by code index (every line fetched once, in order)
//   6  calibration: one 4-B load from each of n distinct 128-B lines of a 4 GiB buffer (every load a miss beyond
//      the Infinity Cache), for FETCH_SIZE per narrow gather
//   7  a bucketing pass (the preparation a sliced gather needs on the device; eight equal code ranges): per
//      workgroup LDS counts, one reservation per bucket and workgroup, every entry written to its bucket
// info[0] entries (heavy rows' entries, read from their padded rows by the superstep, are not collected),
// [1] checksum of the gathered codes (equal for 0, 2, 3, 5), [2] code array bytes.
namespace pm {
template <int V>
__global__ __launch_bounds__(256) void k_gather_floor(const uint32_t* __restrict__ idx, uint64_t n,
                                                      const uint32_t* __restrict__ tab, uint64_t ncode,
                                                      const uint64_t* __restrict__ boff,
                                                      unsigned long long* __restrict__ sink,
                                                      uint32_t* __restrict__ bout, unsigned int* __restrict__ bcnt) {
  uint64_t lo = 0, hi = n, start, stride;
  if (V == 2 || V == 3) {
    // 2: bucket b % 8 on XCD b % 8 (member b / 8); 3: bucket (b / 8) % 8, its members on every XCD
    const uint32_t b = V == 2 ? (blockIdx.x & 7u) : ((blockIdx.x >> 3) & 7u);
    const uint32_t mem = V == 2 ? (blockIdx.x >> 3) : ((blockIdx.x & 7u) | ((blockIdx.x >> 6) << 3));
    lo = boff[b];
    hi = boff[b + 1];
    start = lo + (uint64_t(mem) * blockDim.x + threadIdx.x);
    stride = uint64_t(gridDim.x >> 3) * blockDim.x;
  } else {
    start = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    stride = uint64_t(gridDim.x) * blockDim.x;
  }
  uint64_t acc = 0;
  for (uint64_t i0 = start; i0 < hi; i0 += 4 * stride) {
    uint32_t ci[4];
    bool ok[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t i = i0 + q * stride;
      ok[q] = i < hi;
      if (V == 4) ci[q] = ok[q] ? static_cast<uint32_t>((i * 0x9E3779B97F4A7C15ull >> 29) % ncode) : 0u;
      else if (V == 6) ci[q] = ok[q] ? static_cast<uint32_t>(((i * 2654435761ull) & (ncode - 1)) << 5) : 0u;
      else ci[q] = ok[q] ? idx[i] : 0u;
    }
    if (V == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += ci[q];
    } else if (V == 7) {
      // (the bucketing pass is k_bucket_floor)
    } else if (V == 6) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = ok[q] ? tab[ci[q]] : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += w[q];
    } else {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = ok[q] ? tab[ci[q] >> 4] : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += (w[q] >> ((ci[q] & 15u) << 1)) & 3u;
    }
  }
  acc = wave_sum(acc);
  if (lane_id() == 0) atomicAdd(sink, static_cast<unsigned long long>(acc));
}

// the light survivors' alive M entries as code indices, in record order: pass 0 counts per wave slice, pass 1
// writes at the slice's offset (one thread per superstep-0 wave slice)
template <int PASS>
__global__ __launch_bounds__(256) void k_collect_entries(const uint4* __restrict__ rarea,
                                                         const uint64_t* __restrict__ rbase,
                                                         const uint32_t* __restrict__ rcnt, uint32_t nw,
                                                         const uint32_t* __restrict__ mcol, uint64_t dbase,
                                                         LabelRuns lr, uint64_t* __restrict__ cnt,
                                                         uint32_t* __restrict__ out) {
  const uint32_t gw = blockIdx.x * blockDim.x + threadIdx.x;
  if (gw >= nw) return;
  uint64_t k = PASS ? cnt[gw] : 0;
  for (uint32_t r = 0; r < rcnt[gw]; ++r) {
    const uint4 rec = rarea[rbase[gw] + r];
    if (rec.z == kNone) continue;
    const uint32_t len = (rec.y >> 16) & 0x1FFu;
    for (uint32_t j = 0; j < len; ++j) {
      const uint32_t m = mcol[dbase + rec.z + j];
      if (!(m & kAlive)) continue;
      const uint32_t p = m & kPosMask;
      uint32_t ci = kNone;
      for (int l = 0; l < lr.n; ++l)
        if (p - lr.lo[l] < lr.len[l]) ci = p + lr.cd[l];
      if (ci == kNone) continue;
      if (PASS) out[k] = ci;
      ++k;
    }
  }
  if (!PASS) cnt[gw] = k;
}

// a bucketing pass (variant 7): each workgroup takes a contiguous range of the index stream, counts its entries
// per bucket in LDS, reserves its bucket ranges with one global atomic per bucket, then re-reads the range and
// writes every entry to its bucket (two reads and one write of the stream)
__global__ __launch_bounds__(256) void k_bucket_floor(const uint32_t* __restrict__ idx, uint64_t n, uint64_t ncode,
                                                      const uint64_t* __restrict__ boff, uint32_t* __restrict__ bout,
                                                      unsigned int* __restrict__ bcnt) {
  __shared__ unsigned int s_cnt[8], s_at[8];
  if (threadIdx.x < 8) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = min<uint64_t>(n, uint64_t(blockIdx.x) * per), hi = min<uint64_t>(n, lo + per);
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
    atomicAdd(&s_cnt[(uint64_t(idx[i]) * 8) / ncode], 1u);
  __syncthreads();
  if (threadIdx.x < 8) {
    s_at[threadIdx.x] = atomicAdd(&bcnt[threadIdx.x], s_cnt[threadIdx.x]);
    s_cnt[threadIdx.x] = 0;
  }
  __syncthreads();
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t ci = idx[i];
    const uint32_t b = static_cast<uint32_t>((uint64_t(ci) * 8) / ncode);
    const unsigned k = atomicAdd(&s_cnt[b], 1u);
    const uint64_t at = boff[b] + s_at[b] + k;
    if (at < boff[b + 1]) bout[at] = ci;
  }
}

struct GfArgs {
  const uint32_t* idx;
  uint64_t n;
  const uint32_t* tab;
  uint64_t ncode;
  const uint64_t* boff;
  unsigned long long* sink;
  uint32_t* bout;
  unsigned int* bcnt;
};
template <int V>
static void launch_gather_floor(const GfArgs& g, unsigned grid, hipStream_t s) {
  if (V == 7) {
    hipLaunchKernelGGL(k_bucket_floor, dim3(grid), dim3(256), 0, s, g.idx, g.n, g.ncode, g.boff, g.bout, g.bcnt);
    return;
  }
  hipLaunchKernelGGL(k_gather_floor<V>, dim3(grid), dim3(256), 0, s, g.idx, g.n, g.tab, g.ncode, g.boff, g.sink,
                     g.bout, g.bcnt);
}

struct GatherFloor {
  const void* owner = nullptr;
  uint64_t n = 0;
  uint32_t *d_idx = nullptr, *d_bkt = nullptr, *d_sorted = nullptr, *d_big = nullptr, *d_bout = nullptr;
  uint64_t* d_boff = nullptr;
  unsigned long long* d_sink = nullptr;
  unsigned int* d_bcnt = nullptr;
  void release() {
    for (void* p : {static_cast<void*>(d_idx), static_cast<void*>(d_bkt), static_cast<void*>(d_sorted),
                    static_cast<void*>(d_big), static_cast<void*>(d_bout), static_cast<void*>(d_boff),
                    static_cast<void*>(d_sink), static_cast<void*>(d_bcnt)})
      if (p) (void)hipFree(p);
    *this = GatherFloor{};
  }
};
static GatherFloor g_gather;
void gather_floor_forget(const void* owner) {
  if (owner && g_gather.owner == owner) g_gather.release();
}

static void gather_floor_build(Ctx& c) {
  g_gather.release();
  reset_state(c);
  ensure_counts(c, 1);
  lcc_first_prepare(c);
  lcc_first_set_dense(c);
  if (!c.k1_dense || !c.d_rarea) throw std::runtime_error("gather floor: superstep 0 writes no dense M records here");
  launch_lcc_first_kernel(c, 0, c.k1_grid, c.d_counts);
  const uint32_t nw = c.rwaves;
  uint64_t* d_cnt = dalloc<uint64_t>(nw + 1);
  const unsigned g = (nw + 255) / 256;
  hipLaunchKernelGGL(k_collect_entries<0>, dim3(g), dim3(256), 0, c.stream, c.d_rarea, c.d_rbase, c.d_rcnt, nw,
                     c.d_mcol, c.dbase, c.lr, d_cnt, nullptr);
  std::vector<uint64_t> cnt(nw);
  PM_HIP_CHECK(hipMemcpyAsync(cnt.data(), d_cnt, nw * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  uint64_t n = 0;
  for (auto& x : cnt) {
    const uint64_t v = x;
    x = n;
    n += v;
  }
  PM_HIP_CHECK(hipMemcpy(d_cnt, cnt.data(), nw * sizeof(uint64_t), hipMemcpyHostToDevice));
  g_gather.d_idx = dalloc<uint32_t>(n + 1);
  hipLaunchKernelGGL(k_collect_entries<1>, dim3(g), dim3(256), 0, c.stream, c.d_rarea, c.d_rbase, c.d_rcnt, nw,
                     c.d_mcol, c.dbase, c.lr, d_cnt, g_gather.d_idx);
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  (void)hipFree(d_cnt);
  std::vector<uint32_t> idx(n);
  PM_HIP_CHECK(hipMemcpy(idx.data(), g_gather.d_idx, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  // buckets: eight code ranges holding an eighth of the entries each (the R-MAT skew puts most entries on low
  // positions), entries in record order inside a bucket; and a fully sorted copy
  std::vector<uint32_t> sorted(idx);
  std::sort(sorted.begin(), sorted.end());
  uint32_t cut[8];
  for (int b = 0; b < 8; ++b) cut[b] = n ? sorted[std::min<uint64_t>(n - 1, (uint64_t(b) + 1) * n / 8)] : 0u;
  cut[7] = kNone;
  auto bucket = [&](uint32_t ci) {
    int b = 0;
    while (b < 7 && ci >= cut[b]) ++b;
    return b;
  };
  std::vector<uint64_t> roff(9, 0);  // (variant 7: eight equal code ranges)
  for (uint32_t ci : idx) ++roff[(uint64_t(ci) * 8) / c.lr.ncode + 1];
  for (int b = 0; b < 8; ++b) roff[b + 1] += roff[b];
  std::vector<uint64_t> boff(9, 0);
  for (uint32_t ci : idx) ++boff[bucket(ci) + 1];
  for (int b = 0; b < 8; ++b) boff[b + 1] += boff[b];
  std::vector<uint32_t> bkt(n);
  {
    std::vector<uint64_t> at(boff.begin(), boff.end() - 1);
    for (uint32_t ci : idx) bkt[at[bucket(ci)]++] = ci;
  }
  idx.swap(sorted);
  g_gather.d_bkt = dalloc<uint32_t>(n + 1);
  g_gather.d_sorted = dalloc<uint32_t>(n + 1);
  g_gather.d_bout = dalloc<uint32_t>(n + 1);
  g_gather.d_boff = dalloc<uint64_t>(18);
  g_gather.d_sink = dalloc<unsigned long long>(1);
  g_gather.d_bcnt = dalloc<unsigned int>(8);
  PM_HIP_CHECK(hipMemcpy(g_gather.d_bkt, bkt.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMemcpy(g_gather.d_sorted, idx.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMemcpy(g_gather.d_boff, boff.data(), 9 * sizeof(uint64_t), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMemcpy(g_gather.d_boff + 9, roff.data(), 9 * sizeof(uint64_t), hipMemcpyHostToDevice));
  // 4 GiB calibration buffer: 2^25 lines of 128 B
  g_gather.d_big = dalloc<uint32_t>(uint64_t(1) << 30);
  PM_HIP_CHECK(hipMemset(g_gather.d_big, 1, uint64_t(4) << 30));
  g_gather.n = n;
  g_gather.owner = &c;
  reset_state(c);
  c.k1_dense = false;
  c.tpub_clean = false;
}
}  // namespace pm

extern "C" int pm_debug_gather_floor(pm_ctx* ctx, int variant, int reps, float* ms_out, uint64_t* info) {
  PM_API_BODY(ctx, {
    if (variant < 0 || variant > 7) throw std::runtime_error("gather floor: variant 0..7");
    if (pm::g_gather.owner != static_cast<const void*>(static_cast<pm::Ctx*>(ctx))) pm::gather_floor_build(*ctx);
    auto& G = pm::g_gather;
    // the code array as superstep 0 leaves it (the codes of this launch)
    pm::reset_state(*ctx);
    pm::ensure_counts(*ctx, 1);
    pm::lcc_first_prepare(*ctx);
    pm::lcc_first_set_dense(*ctx);
    pm::launch_lcc_first_kernel(*ctx, 0, ctx->k1_grid, ctx->d_counts);
    const uint64_t ncode = variant == 6 ? (uint64_t(1) << 25) : ctx->lr.ncode;
    const uint32_t* idx = variant == 5 ? G.d_sorted : (variant == 2 || variant == 3) ? G.d_bkt : G.d_idx;
    const uint32_t* tab = variant == 6 ? G.d_big : ctx->d_tcode;
    const unsigned grid = 2048;  // 8 waves per SIMD, a multiple of 8 (the XCD round-robin)
    auto launch = [&] {
      pm::GfArgs g{idx, G.n, tab, ncode, variant == 7 ? G.d_boff + 9 : G.d_boff, G.d_sink, G.d_bout, G.d_bcnt};
      switch (variant) {
        case 0: pm::launch_gather_floor<0>(g, grid, ctx->stream); break;
        case 1: pm::launch_gather_floor<1>(g, grid, ctx->stream); break;
        case 2: pm::launch_gather_floor<2>(g, grid, ctx->stream); break;
        case 3: pm::launch_gather_floor<3>(g, grid, ctx->stream); break;
        case 4: pm::launch_gather_floor<4>(g, grid, ctx->stream); break;
        case 5: pm::launch_gather_floor<5>(g, grid, ctx->stream); break;
        case 6: pm::launch_gather_floor<6>(g, grid, ctx->stream); break;
        default: pm::launch_gather_floor<7>(g, grid, ctx->stream); break;
      }
    };
    hipEvent_t a, b;
    PM_HIP_CHECK(hipEventCreate(&a));
    PM_HIP_CHECK(hipEventCreate(&b));
    PM_HIP_CHECK(hipMemsetAsync(G.d_bcnt, 0, 8 * sizeof(unsigned int), ctx->stream));
    launch();  // warm
    float total = 0.f;
    for (int i = 0; i < std::max(reps, 1); ++i) {
      // the sink reset outside the events
      PM_HIP_CHECK(hipMemsetAsync(G.d_sink, 0, sizeof(unsigned long long), ctx->stream));
      if (variant == 7) PM_HIP_CHECK(hipMemsetAsync(G.d_bcnt, 0, 8 * sizeof(unsigned int), ctx->stream));
      PM_HIP_CHECK(hipEventRecord(a, ctx->stream));
      launch();
      PM_HIP_CHECK(hipEventRecord(b, ctx->stream));
      PM_HIP_CHECK(hipEventSynchronize(b));
      float ms = 0.f;
      PM_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    unsigned long long sum = 0;
    PM_HIP_CHECK(hipMemcpy(&sum, G.d_sink, sizeof(sum), hipMemcpyDeviceToHost));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms_out) *ms_out = total / std::max(1, reps);
    if (info) {
      info[0] = G.n;
      info[1] = sum;
      info[2] = pm::tcode_words(ctx->lr) * sizeof(uint32_t);
    }
    ctx->k1_dense = false;
    ctx->tpub_clean = false;
    pm::reset_state(*ctx);
  });
}
