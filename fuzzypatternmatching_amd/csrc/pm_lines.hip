// Fused token passing: one persistent grid-synchronised kernel per run of NLC lines.
//
// The level-synchronous formulation of pm_kernels.hip ("Token passing")
// executed as a single grid-wide kernel whose phases are separated by grid
// barriers, so a line costs one launch and one host synchronisation instead of
// a launch + sync per position:
//   P1 source selection over slist (nem_1.hpp:387-479 / tds_batch_1.hpp:1067-1135)
//      fused with the position-1 tokens of each selected source
//   P2.. one phase per walk position (nem_1.hpp:131-297, :540-791 /
//      tds_batch_1.hpp:284-302, :622-758)
//   Pp post-processing of unacked sources (beta.cpp:964-1000), reporting the
//      vertices / edges that leave S per rank (the active counts after the
//      line follow from the counts before it), and hash-slot cleanup
// Barriers: C + 1 per path line, C + 2 per TDS line (tree_barrier: a
// two-level arrival counter, ~6 us at one 1024-thread block per CU against
// ~30 us for cooperative_groups grid.sync, tools/ubench_src/coop_barrier.hip).
//
// Path / cycle lines (nem_1) deduplicate (source, vertex) arrivals in an
// open-addressing hash table: value = (position << 32) | parent, the parent
// turning into kMulti when a second distinct parent arrives at the same
// position -- the rule of the sort-based path (lowest position wins; a single
// parent is excluded from forwarding, several parents exclude none).
// Capacities are fixed per call; an overflow is detected before any terminal
// effect and the caller reruns the line through the exact-count path.
// Stale token-source-map entries need no cleanup: only sources are read in
// post-processing and P1 resets every source's entry.
//
// Memory ordering: phases exchange data through global memory across CUs.
// Reads of data written by another CU in an earlier phase whose cache line
// this CU may already hold (frontier lists, hash slots, source list) go
// through ld_dev (L1-bypassing atomic loads); TDS walk regions are fresh,
// 128-B aligned memory per position.
//
// Launch: at most one 1024-thread block per CU (hipOccupancyMaxActiveBlocksPerMultiprocessor >= 1 checked).
// Round 6: an ordinary launch when the context is alone on its device (Ctx::coop false): the grid fits, and what
// runs beside it on the context's side stream (read-back copies, a fill) finishes without waiting for it, so every
// block becomes resident.  In-process shards sharing a device take hipLaunchCooperativeKernel, whose guarantee
// covers their concurrent grids; it costs ~28 us per launch (tools/gpu_coop_ab.sh: 2.484 vs 2.397 ms per S=28
// step with the compaction scans' two launches).  The cooperative queue also crashes libhsa-runtime's exit-time
// teardown under rocprofv3 (tools/rp_exit.py beta vs beta_nocoop), hence PM_LINES_NOCOOP=1 for profiled runs.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "pm_device.hpp"
#include "pm_internal.hpp"

namespace pm {

static constexpr unsigned long long kEmpty = ~0ull;
static constexpr uint32_t kMulti = 0xFFFFFFFEu;
static constexpr int kMaxProbe = 128;

// Relaxed device-scope atomic load: bypasses this CU's L1 so a value written by
// another CU before the last grid barrier is seen; the ordering itself comes
// from the barrier's release / acquire fences (tree_barrier).
template <typename T>
__device__ __forceinline__ T ld_dev(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct LineKernelArgs {
  // graph / state (positions)
  const uint64_t* offp;
  uint32_t* mcol;
  const uint32_t* mlen;
  const uint32_t* malive;
  uint16_t* tpub;
  const uint32_t* perm;
  uint8_t* tsm;
  const uint32_t* slist;
  const uint32_t* nS;
  const unsigned long long* smask;  // live mask of slist per 64 entries (null: all live)
  uint32_t* sources;
  OwnerArgs oa;
  const LineArgs* la;  // current line (global memory: indexed at run time)
  int i0;  // pattern_indices[0] (post-processing bit)
  unsigned* gbar;  // grid barrier state
  // hash table (path lines), persistent, clean between lines
  unsigned long long* hkey;
  unsigned long long* hval;
  uint64_t hmask;
  uint32_t* front;  // inserted slots, position segments
  uint64_t fcap;
  // walk storage (TDS lines): positions laid out one after the other
  uint32_t* wbuf;
  uint64_t wcap;  // u32 slots
  uint32_t* kept;  // kept walks of the launch (stride C+2 of their line)
  uint64_t kept_cap;
  unsigned long long* kept_ctr;  // u32 slots used in kept
  LineStats* st;   // per line (indexed by pl)
  const LineDesc* lines;
  int pl_begin, pl_end;
  unsigned* done;  // lines processed by the launch
  uint32_t* act;   // S members at launch start (slist entries with T_pub != 0), built by k_lines
  unsigned long long* nact;
  uint64_t small_line;  // single-block threshold (kSmallLine)
  int stamps;           // per-position time stamps (PM_PHASE_TIMES)
  // sharded replica: lines whose census reaches split_min run split by owner (so: the shard owner rule)
  OwnerArgs so;
  uint32_t shard;
  uint64_t split_min;
  int split;                      // the current line runs split: own sources, post-processing deferred
  unsigned long long* xflag;      // split cycle lines: M entries this shard's terminals flagged
  unsigned long long* nxflag;
  uint64_t xflag_cap;
  // long rows (hubs) of a position: cut into kLineLong-entry pieces that the whole grid works through after
  // the position's other items (a wave walking a hub row of 10^5..10^6 entries alone held up the line)
  unsigned long long* lpieces;
  uint64_t lp_cap;
  // PM_DEBUG_SYNC (diagnostics): every row a line reads is checked against the vertex count and the M
  // buffer first; the first bad one is recorded in dbg[0..3] (flag, vertex, row start, length) and skipped
  unsigned long long* dbg;
  uint64_t n, mcap;
};

// The current line's constants, copied into LDS at the line's start by k_lines (read at every entry of the
// walks: from global memory they were vector loads -- the kernel writes global memory, so they cannot go
// through the scalar cache -- each a round trip in the walks' dependent chains).
__shared__ LineArgs s_la;
static_assert(sizeof(LineArgs) % sizeof(uint32_t) == 0, "LineArgs is copied in words");

// (diagnostics) false when the row (b, L) of vertex u lies outside the M buffer: recorded, not read
__device__ __forceinline__ bool row_ok(const LineKernelArgs& a, uint32_t u, uint64_t b, uint64_t L) {
  if (!a.dbg) return true;
  if (u < a.n && b <= a.mcap && L <= a.mcap - b) return true;
  if (atomicCAS(&a.dbg[0], 0ull, 1ull) == 0ull) {
    a.dbg[1] = u;
    a.dbg[2] = b;
    a.dbg[3] = L;
  }
  return false;
}

__device__ __forceinline__ void wave_add(unsigned long long* ctr, uint64_t x) {
  x = wave_sum(x);
  if (lane_id() == 0 && x) atomicAdd(ctr, static_cast<unsigned long long>(x));
}

// Value update of hash slot h for an arrival at position `level` from
// `parent`; true for the first arrival (the slot joins the position's frontier).
__device__ __forceinline__ bool ht_arrive(unsigned long long* hval, uint64_t h, uint32_t level, uint32_t parent) {
  const unsigned long long want = (static_cast<unsigned long long>(level) << 32) | parent;
  unsigned long long old = ld_dev(&hval[h]);
  while (true) {
    if (old == kEmpty) {
      const unsigned long long prev = atomicCAS(&hval[h], kEmpty, want);
      if (prev == kEmpty) return true;
      old = prev;
      continue;
    }
    if ((old >> 32) < level) return false;  // reached at a lower position: dropped
    const uint32_t par = static_cast<uint32_t>(old);
    if (par == parent || par == kMulti) return false;
    const unsigned long long prev =
        atomicCAS(&hval[h], old, (static_cast<unsigned long long>(level) << 32) | kMulti);
    if (prev == old) return false;
    old = prev;
  }
}

// Insert (s, u) at `level` from `parent`; returns the slot on a first
// arrival, kEmpty otherwise (and on overflow, flagged in st).
__device__ __forceinline__ uint64_t ht_insert(const LineKernelArgs& a, uint32_t s, uint32_t u, uint32_t level,
                                              uint32_t parent) {
  const unsigned long long key = (static_cast<unsigned long long>(s) << 32) | u;
  uint64_t h = mix64(key) & a.hmask;
  for (int probe = 0; probe < kMaxProbe; ++probe) {
    unsigned long long k = ld_dev(&a.hkey[h]);
    if (k == kEmpty) {
      const unsigned long long prev = atomicCAS(&a.hkey[h], kEmpty, key);
      k = prev == kEmpty ? key : prev;
    }
    if (k == key) return ht_arrive(a.hval, h, level, parent) ? h : kEmpty;
    h = (h + 1) & a.hmask;
  }
  atomicOr(&a.st->overflow, 1u);
  return kEmpty;
}

// Index of vertex v in the row [b, e) (rows hold positions in neighbour-id order, one entry per neighbour), e
// when absent.
__device__ __forceinline__ uint64_t row_find(const LineKernelArgs& a, uint64_t b, uint64_t e, uint32_t v) {
  const uint32_t pid = a.perm[v];
  uint64_t lo = b, hi = e;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a.perm[a.mcol[mid] & kPosMask] < pid) lo = mid + 1; else hi = mid;
  }
  return lo < e && (a.mcol[lo] & kPosMask) == v ? lo : e;
}
__device__ __forceinline__ bool row_has_alive(const LineKernelArgs& a, uint64_t b, uint64_t e, uint32_t v) {
  const uint64_t i = row_find(a, b, e, v);
  return i < e && (a.mcol[i] & kAlive);
}

// Terminal position C+1 of a path / cycle line (nem_1.hpp:661-791).
__device__ __forceinline__ void tp_terminal(const LineKernelArgs& a, uint32_t u, uint32_t s, uint32_t p) {
  const LineArgs& la = s_la;
  if (!pos_ok(a.tpub[u], la.C + 1, la)) return;
  if (!la.VC) {
    if (u == s) return;
    if (a.tpub[s]) a.tsm[s] = 2;  // ack visitor needs an active source (nem_1.hpp:101, :326-336)
  } else {
    if (u != s) return;
    a.tsm[s] = 2;
    // mark M[s][p]
    const uint64_t b = a.offp[s], e = b + a.mlen[s];
    const uint64_t lo = row_find(a, b, e, p);
    if (lo < e && (a.mcol[lo] & kAlive)) {
      if (!a.split) {
        a.mcol[lo] |= kFlag;
      } else if (!(atomicOr(&a.mcol[lo], kFlag) & kFlag) && a.xflag) {  // newly flagged: the other replicas too
        const unsigned long long at = atomicAdd(a.nxflag, 1ull);
        if (at < a.xflag_cap) a.xflag[at] = lo;
        else atomicOr(&a.st->overflow, 1u);
      }
    }
  }
}

// Per-wave staging of the rows a wave expands (flattened expansion: the
// wave's 64 rows are concatenated and every lane takes every 64th entry, so a
// long row costs one pass over the wave instead of a serial walk by one lane).
static constexpr int kLineWaves = 16;  // kLineBlock / kWave
static constexpr int kStage = 10;      // TDS walks of up to kStage positions are staged in LDS
struct WaveRows {
  uint64_t beg[kLineWaves][kWave];
  uint32_t end[kLineWaves][kWave];  // inclusive scan of the row lengths
  union {
    struct {
      uint32_t s[kLineWaves][kWave], u[kLineWaves][kWave], x[kLineWaves][kWave];
    } t;                                          // token rows (path lines, TDS sources)
    uint32_t walk[kLineWaves][kWave * kStage];    // the wave's walks (TDS positions)
  };
  unsigned long long wn[20];  // walks per position of a single-block TDS line
  unsigned lpany[20];         // a row of this position went to the piece list (single-block lines: no global read)
};

// Lane owning concatenated entry t (end[] inclusive scan of the wave's rows).
__device__ __forceinline__ int row_of(const uint32_t* end, uint32_t t) {
  int lo = 0, hi = kWave - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (end[mid] > t) hi = mid; else lo = mid + 1;
  }
  return lo;
}

struct GridIdx {
  uint64_t tid, nth, gw, nw;
};

static constexpr uint32_t kLineLong = 2048;
static constexpr int kUnroll = 4;  // entry groups in flight per wave in the flattened row loops

// Appends the pieces of a long row (item id of position k, len entries) to the position's list; false when it
// is full (the caller's wave then walks the row itself).  Piece word: q << 32 | item.
__device__ __forceinline__ bool line_pieces(const LineKernelArgs& a, int k, uint32_t item, uint32_t len,
                                            unsigned* lpany) {
  lpany[k] = 1u;
  const uint32_t np = (len + kLineLong - 1) / kLineLong;
  const unsigned long long b = atomicAdd(&a.st->lp[k], static_cast<unsigned long long>(np));
  if (b + np > a.lp_cap) {
    for (uint64_t q = b; q < a.lp_cap && q < b + np; ++q) a.lpieces[q] = ~0ull;
    return false;
  }
  for (uint32_t q = 0; q < np; ++q) a.lpieces[b + q] = (static_cast<unsigned long long>(q) << 32) | item;
  return true;
}

// Forwarding from u (token of source s at position k, excluded parent excl):
// every alive w in M[u] other than excl goes to position k + 1 (terminal
// action at C + 1, else arrival filter + hash insert).  All lanes of the wave
// must call it; returns the lane's share of the emitted token count.
__device__ __forceinline__ uint32_t tp_forward(const LineKernelArgs& a, WaveRows& wr, uint32_t u, uint32_t s,
                                               uint32_t excl, int k, bool active, uint32_t item) {
  uint32_t emitted = 0;
  const LineArgs& la = s_la;
  k = __builtin_amdgcn_readfirstlane(k);
  const int wv = threadIdx.x / kWave, lane = lane_id();
  uint64_t b = 0;
  uint32_t L = 0;
  const bool term = k == la.C;  // the row's entries reach the terminal position C + 1
  if (active) {
    b = a.offp[u];
    L = a.mlen[u];
    if (!row_ok(a, u, b, L)) L = 0;
    if (term && L) {
      // the token count of a terminal row is its alive entries other than excl, as the walk would count them;
      // only the terminal actions need the entries
      emitted = a.malive[u] - (excl != kNone && row_has_alive(a, b, b + L, excl) ? 1u : 0u);
      if (la.VC) {
        // cycle line: of the row's entries only w = s reaches the terminal action, so the row is searched for s
        if (s != excl && row_has_alive(a, b, b + L, s)) tp_terminal(a, s, s, u);
        L = 0;
      } else if (!a.tpub[s] || a.tsm[s] == 2) {
        L = 0;  // path line: the action acks an active source only, and s is inactive or acked already
      }
    }
    if (L > kLineLong && line_pieces(a, k, item, L, wr.lpany)) L = 0;  // (the pieces: tp_pieces)
  }
  const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(L));
  const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
  if (!total) return 0;
  wr.beg[wv][lane] = b;
  wr.end[wv][lane] = incl;
  wr.t.s[wv][lane] = s;
  wr.t.u[wv][lane] = u;
  wr.t.x[wv][lane] = excl;
  __builtin_amdgcn_wave_barrier();
  // kUnroll groups of 64 entries per round: their row searches and entry loads are independent (the loads
  // of one round are in flight together), their first arrivals share one frontier reservation
  for (uint32_t t0 = 0; t0 < total; t0 += kUnroll * kWave) {
    uint32_t mm[kUnroll];
    int rr[kUnroll];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const uint32_t t = t0 + j * kWave + lane;
      mm[j] = 0;
      rr[j] = 0;
      if (t < total) {
        const int r = row_of(wr.end[wv], t);
        const uint32_t first = r ? wr.end[wv][r - 1] : 0u;
        rr[j] = r;
        mm[j] = a.mcol[wr.beg[wv][r] + (t - first)];
      }
    }
    uint32_t slots[kUnroll];
    uint32_t nnew = 0;
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const uint32_t m = mm[j];
      const int r = rr[j];
      if ((m & kAlive) && (!a.dbg || row_ok(a, m & kPosMask, 0, 0))) {
        const uint32_t w = m & kPosMask, sr = wr.t.s[wv][r], ur = wr.t.u[wv][r];
        if (w != wr.t.x[wv][r]) {
          if (term) {
            tp_terminal(a, w, sr, ur);  // (counted above)
          } else {
            ++emitted;
            if (w != sr && pos_ok(a.tpub[w], k + 1, la)) {
              const uint64_t slot = ht_insert(a, sr, w, static_cast<uint32_t>(k + 1), ur);
              if (slot != kEmpty) slots[nnew++] = static_cast<uint32_t>(slot);
            }
          }
        }
      }
    }
    if (__ballot(nnew != 0)) {
      const uint64_t pos = wave_reserve(&a.st->ftotal, nnew);
      for (uint32_t j = 0; j < nnew; ++j) {
        if (pos + j < a.fcap) a.front[pos + j] = slots[j];
        else atomicOr(&a.st->overflow, 1u);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  return emitted;
}

// The long-row pieces of position k of a path / cycle line (items: the source at k = 0, the frontier's hash
// slot after): the entries [q kLineLong, (q + 1) kLineLong) of the item's row, one piece per wave and round,
// with tp_forward's per-entry rule.  Returns the lane's share of the emitted tokens.
__device__ __forceinline__ uint32_t tp_pieces(const LineKernelArgs& a, const GridIdx& g, int k) {
  const LineArgs& la = s_la;
  const int lane = lane_id();
  uint32_t emitted = 0;
  const uint64_t np = min<uint64_t>(ld_dev(&a.st->lp[k]), a.lp_cap);
  for (uint64_t pi = g.gw; pi < np; pi += g.nw) {
    const unsigned long long pc = ld_dev(&a.lpieces[pi]);
    if (pc == ~0ull) continue;
    const uint32_t item = static_cast<uint32_t>(pc), q = static_cast<uint32_t>(pc >> 32);
    uint32_t s, u, excl = kNone;
    if (k == 0) {
      s = u = item;
    } else {
      const unsigned long long key = ld_dev(&a.hkey[item]);
      const uint32_t par = static_cast<uint32_t>(ld_dev(&a.hval[item]));
      s = static_cast<uint32_t>(key >> 32);
      u = static_cast<uint32_t>(key);
      excl = par == kMulti ? kNone : par;
    }
    const uint64_t b = a.offp[u] + uint64_t(q) * kLineLong;
    const uint32_t len = min(kLineLong, a.mlen[u] - q * kLineLong);
    for (uint32_t t0 = 0; t0 < len; t0 += kWave) {
      const uint32_t t = t0 + lane;
      uint64_t slot = kEmpty;
      if (t < len) {
        const uint32_t m = a.mcol[b + t];
        if ((m & kAlive) && (!a.dbg || row_ok(a, m & kPosMask, 0, 0))) {
          const uint32_t w = m & kPosMask;
          if (w != excl) {
            if (k == la.C) {
              tp_terminal(a, w, s, u);  // (the token count was taken when the row was listed)
            } else {
              ++emitted;
              if (w != s && pos_ok(a.tpub[w], k + 1, la)) slot = ht_insert(a, s, w, static_cast<uint32_t>(k + 1), u);
            }
          }
        }
      }
      const uint32_t is_new = slot != kEmpty ? 1u : 0u;
      if (__ballot(is_new)) {
        const uint64_t pos = wave_reserve(&a.st->ftotal, is_new);
        if (is_new) {
          if (pos < a.fcap) a.front[pos] = static_cast<uint32_t>(slot);
          else atomicOr(&a.st->overflow, 1u);
        }
      }
    }
  }
  return emitted;
}

// Grid barrier for co-resident blocks (see "Launch" above): blocks arrive on
// per-group counters (16 blocks, own 128-B lines), the last of a group on the
// top counter, the last group bumps the generation word everyone waits on.
// Counters reset themselves; the generation only grows.
__device__ __forceinline__ void tree_barrier(unsigned* bar) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x;
    const unsigned ngroups = (nb + 15) / 16;
    const unsigned grp = blockIdx.x / 16;
    const unsigned gsize = min(16u, nb - grp * 16);
    unsigned* gen = bar;
    unsigned* top = bar + 32;
    unsigned* gc = bar + 64 + grp * 32;
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (atomicAdd(gc, 1u) == gsize - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (atomicAdd(top, 1u) == ngroups - 1) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) __builtin_amdgcn_s_sleep(1);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}
static constexpr unsigned kGbarWords = 64 + 32 * 64;  // up to 1024 blocks

static constexpr int kLineBlock = 1024;
static_assert(kLineBlock / kWave == kLineWaves, "WaveRows is sized for kLineBlock");
__device__ __forceinline__ GridIdx grid_idx() {
  GridIdx g;
  const uint32_t wpb = blockDim.x / kWave;
  g.tid = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  g.nth = uint64_t(gridDim.x) * blockDim.x;
  g.gw = blockIdx.x * uint64_t(wpb) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  g.nw = uint64_t(gridDim.x) * wpb;
  return g;
}

// P1 for one entry of the active list: returns the lane's source (ok) after
// appending it to the source list and marking the token source map.  The
// list was built at launch start; a member whose T_pub became 0 since (post-
// processing of an earlier line) fails the T_pub test.
__device__ __forceinline__ bool select_source(const LineKernelArgs& a, uint64_t i, uint64_t nact, bool tds,
                                              uint32_t& s) {
  bool ok = false;
  s = 0;
  if (i < nact) {
    s = ld_dev(&a.act[i]);
    const uint16_t T = a.tpub[s];
    ok = T && pos_ok(T, 0, s_la);
    if (ok && !tds && !s_la.VC && !((T >> s_la.ilast) & 1u)) ok = false;
    if (ok && a.split && owner_of(s, a.so) != a.shard) ok = false;  // a split line: this shard's sources
  }
  const uint64_t pos = wave_reserve(&a.st->nsrc, ok ? 1u : 0u);
  if (ok) {
    a.sources[pos] = s;
    a.tsm[s] = 1;
  }
  return ok;
}

// Active list of the launch: the slist entries with T_pub != 0 (every later
// source is one of them: S only shrinks), found through the live masks of the
// last superstep, 64 mask words per wave (dead chunks cost one coalesced load).
__device__ __forceinline__ void build_active(const LineKernelArgs& a) {
  const GridIdx g = grid_idx();
  const int lane = lane_id();
  const uint32_t nS = *a.nS;
  const uint64_t nch = (uint64_t(nS) + kWave - 1) / kWave;
  if (nch <= uint64_t(g.nw) * 4) {
    // a short (compacted) list: one chunk per wave, so that the chunks' dependent
    // loads and reservations overlap across waves instead of queueing in one
    for (uint64_t ch = g.gw; ch < nch; ch += g.nw) {
      const uint64_t live = a.smask ? a.smask[ch] : ~0ull;  // wave-uniform
      if (!live) continue;
      const uint64_t i = ch * kWave + lane;
      uint32_t v = 0;
      bool ok = false;
      if (i < nS && ((live >> lane) & 1ull)) {
        v = a.slist[i];
        ok = a.tpub[v] != 0;
      }
      const uint64_t pos = wave_reserve(a.nact, ok ? 1u : 0u);
      if (ok) a.act[pos] = v;
    }
    return;
  }
  for (uint64_t c0 = g.gw * kWave; c0 < nch; c0 += g.nw * kWave) {
    const uint64_t ch = c0 + lane;
    const uint64_t lm = ch < nch ? (a.smask ? a.smask[ch] : ~0ull) : 0ull;
    uint64_t bal = __ballot(lm != 0);
    while (bal) {
      const int j = __ffsll(static_cast<long long>(bal)) - 1;
      bal &= bal - 1;
      const uint64_t live =
          (uint64_t(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(lm >> 32), j))) << 32) |
          static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(lm), j));
      const uint64_t i = (c0 + j) * kWave + lane;
      uint32_t v = 0;
      bool ok = false;
      if (i < nS && ((live >> lane) & 1ull)) {
        v = a.slist[i];
        ok = a.tpub[v] != 0;
      }
      const uint64_t pos = wave_reserve(a.nact, ok ? 1u : 0u);
      if (ok) a.act[pos] = v;
    }
  }
}

// Pp: post-processing of unacked sources (k_tp_post), reporting the vertices
// and edges (|M|) per rank whose T_pub becomes empty.
__device__ __forceinline__ void line_post(const LineKernelArgs& a, const GridIdx& g, unsigned long long* s_hist) {
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  const uint64_t nsrc = ld_dev(&a.st->nsrc);
  uint64_t acked = 0, deleted = 0, rv = 0, re = 0;
  for (uint64_t i = g.tid; i < nsrc; i += g.nth) {
    const uint32_t s = ld_dev(&a.sources[i]);
    if (ld_dev(&a.tsm[s]) == 2) {
      ++acked;
      continue;
    }
    uint16_t T = a.tpub[s];
    if (!T) continue;
    if ((T >> a.i0) & 1u) {
      T &= static_cast<uint16_t>(~(1u << a.i0));
      a.tpub[s] = T;  // T == 0: vertex_active = false and erased from the state map
      if (!T) {
        if (a.oa.nranks <= 1) {
          rv += 1;
          re += a.malive[s];
        } else {
          acc_owner(s_hist, a.oa, s, a.malive[s]);
        }
      }
    }
    ++deleted;
  }
  wave_add(&a.st->acked, acked);
  wave_add(&a.st->deleted, deleted);
  if (a.oa.nranks <= 1) {
    wave_add(&a.st->removed[0], rv);
    wave_add(&a.st->removed[1], re);
  } else {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 2 * a.oa.nranks; i += blockDim.x)
      if (s_hist[i]) atomicAdd(&a.st->removed[i], s_hist[i]);
  }
}

// ---- TDS lines (tds_batch_1) -------------------------------------------
// Walks of position L (L+1 vertices) are stored from st->wbase[L] on, stride
// C+2 u32, each position in fresh memory (no cache line is reused across
// phases).  Sender-side checks of a child nb of walk w at position k + 1
// (tds_batch_1.hpp:793-909), as in k_tds_expand.
__device__ __forceinline__ bool tds_child_ok(const uint32_t* w, int k, uint32_t nb, const LineArgs& la) {
  if (k == la.C) {
    if (la.VC) return nb == w[0];
    if (nb == w[0]) return false;
  }
  return enum_ok(w, k + 1, nb, la);
}

// Flattened expansion of the wave's walks at position k (rows b/L per lane,
// L = 0 for walks that fail the arrival checks): children are appended to
// region out through counter ctr.  The walks are read from the wave's LDS
// stage (stage) or from win[i0 ..].  All lanes must call it.
__device__ __forceinline__ void tds_expand_wave(const LineKernelArgs& a, WaveRows& wr, const uint32_t* win,
                                                uint64_t i0, int k, uint64_t b, uint32_t L, uint32_t* out,
                                                uint64_t out_room, int stride, bool stage,
                                                unsigned long long* ctr) {
  const LineArgs& la = *a.la;
  const int wv = threadIdx.x / kWave, lane = lane_id();
  const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(L));
  const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
  if (!total) return;
  wr.beg[wv][lane] = b;
  wr.end[wv][lane] = incl;
  __builtin_amdgcn_wave_barrier();
  // kUnroll groups of 64 entries per round (tp_forward); the round's children share one reservation
  for (uint32_t t0 = 0; t0 < total; t0 += kUnroll * kWave) {
    uint32_t mm[kUnroll];
    int rr[kUnroll];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const uint32_t t = t0 + j * kWave + lane;
      mm[j] = 0;
      rr[j] = 0;
      if (t < total) {
        const int r = row_of(wr.end[wv], t);
        const uint32_t first = r ? wr.end[wv][r - 1] : 0u;
        rr[j] = r;
        mm[j] = a.mcol[wr.beg[wv][r] + (t - first)];
      }
    }
    uint32_t cm = 0;  // children of the round (bit j)
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const uint32_t* w = stage ? wr.walk[wv] + rr[j] * stride : win + (i0 + rr[j]) * stride;
      if ((mm[j] & kAlive) && tds_child_ok(w, k, mm[j] & kPosMask, la)) cm |= 1u << j;
    }
    const uint32_t nc = __popc(cm);
    const uint64_t pos = wave_reserve(ctr, nc);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      if (!((cm >> j) & 1u)) continue;
      const uint32_t* w = stage ? wr.walk[wv] + rr[j] * stride : win + (i0 + rr[j]) * stride;
      if ((pos + c + 1) * stride <= out_room) {
        uint32_t* d = out + (pos + c) * stride;
        for (int p = 0; p <= k; ++p) d[p] = w[p];
        d[k + 1] = mm[j] & kPosMask;
      } else {
        atomicOr(&a.st->overflow, 1u);
      }
      ++c;
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// The long-row pieces of position k of a TDS line (items: the source at k = 0, the walk's index in win after):
// children of the entries [q kLineLong, (q + 1) kLineLong) of the row of the walk's last vertex, with
// tds_expand_wave's checks, appended through ctr.  The walk itself passed the arrival checks when its piece
// was listed.
__device__ __forceinline__ void tds_pieces(const LineKernelArgs& a, const GridIdx& g, int k, const uint32_t* win,
                                           uint32_t* out, uint64_t out_room, int stride, unsigned long long* ctr) {
  const LineArgs& la = s_la;
  const int lane = lane_id();
  const uint64_t np = min<uint64_t>(ld_dev(&a.st->lp[k]), a.lp_cap);
  for (uint64_t pi = g.gw; pi < np; pi += g.nw) {
    const unsigned long long pc = ld_dev(&a.lpieces[pi]);
    if (pc == ~0ull) continue;
    const uint32_t item = static_cast<uint32_t>(pc), q = static_cast<uint32_t>(pc >> 32);
    const uint32_t* w = k == 0 ? nullptr : win + uint64_t(item) * stride;
    const uint32_t u = k == 0 ? item : w[k];
    const uint64_t b = a.offp[u] + uint64_t(q) * kLineLong;
    const uint32_t len = min(kLineLong, a.mlen[u] - q * kLineLong);
    for (uint32_t t0 = 0; t0 < len; t0 += kWave) {
      const uint32_t t = t0 + lane;
      bool child = false;
      uint32_t nb = 0;
      if (t < len) {
        const uint32_t m = a.mcol[b + t];
        if (m & kAlive) {
          nb = m & kPosMask;
          child = k == 0 || tds_child_ok(w, k, nb, la);
        }
      }
      const uint64_t pos = wave_reserve(ctr, child ? 1u : 0u);
      if (child) {
        if ((pos + 1) * stride <= out_room) {
          uint32_t* d = out + pos * stride;
          if (k == 0) {
            d[0] = u;
          } else {
            for (int p = 0; p <= k; ++p) d[p] = w[p];
          }
          d[k + 1] = nb;
        } else {
          atomicOr(&a.st->overflow, 1u);
        }
      }
    }
  }
}

// Block-local index (single-block mode: block 0 finishes a small line alone).
__device__ __forceinline__ GridIdx block_idx() {
  GridIdx g;
  g.tid = threadIdx.x;
  g.nth = blockDim.x;
  g.gw = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  g.nw = blockDim.x / kWave;
  return g;
}

__device__ __forceinline__ void phase_sync(const LineKernelArgs& a, bool single) {
  if (single) __syncthreads();
  else tree_barrier(a.gbar);
}

// A line whose sources and position-1 frontier are at most this large starts on
// block 0 alone (block barriers instead of grid barriers) while the other blocks
// wait at a grid barrier; once a position's frontier outgrows it, block 0 stops
// and the whole grid continues from that position (escalation: R-MAT hubs make
// a small line's later positions explode).  LineKernelArgs::small_line,
// PM_SMALL_LINE overrides.  Round 5: with a position's items spread over every wave (16 to 64 per wave), the
// grid finishes a position of a few hundred walks sooner than block 0 does despite its barriers (the S=28 TDS
// line: 7 positions of 446-1693 walks, 85 us on the grid vs 125 us on block 0), so block 0 keeps only the
// tiny lines.
static constexpr uint64_t kSmallLine = 256;

// ---- path / cycle lines (nem_1) ----------------------------------------
// Positions 2..C+1 and post-processing; every participating wave calls it.
// Returns true when block 0 (single) handed the line to the grid at position esc_k.
__device__ __forceinline__ bool path_rest(const LineKernelArgs& a, const GridIdx& g, bool single,
                                          unsigned long long* s_hist, WaveRows& wr, int k0 = 1, uint64_t lo0 = 0) {
  LineStats* st = a.st;
  uint64_t trav = 0, tokens = 0, lo = lo0;
  if (single) {
    if (threadIdx.x < 20) wr.lpany[threadIdx.x] = 0u;
    __syncthreads();
  }
  // (the overflow flag and the frontier end read together after each position's barrier, as in tds_rest)
  unsigned ovf_next = ld_dev(&st->overflow);
  uint64_t hi_next = ld_dev(&st->ftotal);
  for (int k = k0; k <= s_la.C; ++k) {
    k = __builtin_amdgcn_readfirstlane(k);  // (uniform: the line's constants indexed by k load through the scalar cache)
    if (ovf_next) break;  // same value in every wave after the barrier
    const uint64_t hi = hi_next;
    if (single && hi - lo > a.small_line) {  // the frontier outgrew the block: the grid takes position k
      wave_add(&st->trav, trav);
      wave_add(&st->tokens, tokens);
      if (g.tid == 0) {
        st->esc_base = lo;
        st->esc_k = static_cast<unsigned>(k);
      }
      return true;
    }
    // frontier items per wave and pass: spread over every wave (16 to 64 each), as in tds_rest
    const uint64_t per = min<uint64_t>(kWave, max<uint64_t>(16, (hi - lo + g.nw - 1) / g.nw));
    for (uint64_t i0 = lo + g.gw * per; i0 < hi; i0 += g.nw * per) {
      const uint64_t i = i0 + lane_id();
      const bool act = static_cast<uint64_t>(lane_id()) < per && i < hi;
      uint32_t s = 0, u = 0, excl = kNone, h = 0;
      if (act) {
        h = ld_dev(&a.front[i]);
        const unsigned long long key = ld_dev(&a.hkey[h]);
        const uint32_t par = static_cast<uint32_t>(ld_dev(&a.hval[h]));
        s = static_cast<uint32_t>(key >> 32);
        u = static_cast<uint32_t>(key);
        excl = par == kMulti ? kNone : par;
        trav += a.malive[u];
      }
      tokens += tp_forward(a, wr, u, s, excl, k, act, h);
    }
    lo = hi;
    phase_sync(a, single);
    const bool pieces = single ? wr.lpany[k] != 0u : ld_dev(&st->lp[k]) != 0ull;
    ovf_next = ld_dev(&st->overflow);
    hi_next = ld_dev(&st->ftotal);
    if (pieces) {  // the position's long rows, over every wave
      tokens += tp_pieces(a, g, k);
      phase_sync(a, single);
      ovf_next = ld_dev(&st->overflow);
      hi_next = ld_dev(&st->ftotal);
    }
    if (a.stamps && g.tid == 0) st->ptime[k] = __builtin_amdgcn_s_memrealtime();
  }
  wave_add(&st->trav, trav);
  wave_add(&st->tokens, tokens);
  if (ld_dev(&st->overflow)) return false;  // the host clears the table and reruns the line
  if (!a.split) line_post(a, g, s_hist);  // (split: after the shards agreed on overflow, split_line_finish)
  // hash cleanup: no insert happens after the last position
  const uint64_t nf = ld_dev(&st->ftotal);
  for (uint64_t i = g.tid; i < nf; i += g.nth) {
    const uint32_t h = ld_dev(&a.front[i]);
    a.hkey[h] = kEmpty;
    a.hval[h] = kEmpty;
  }
  return false;
}

__device__ __forceinline__ void path_line(const LineKernelArgs& a, unsigned long long* s_hist, WaveRows& wr) {
  const GridIdx g = grid_idx();
  LineStats* st = a.st;
  uint64_t trav = 0, tokens = 0;
  // P1 + position 1: (v, s, parent = s) for v in M[s]
  const uint64_t nact = ld_dev(a.nact);
  for (uint64_t i0 = g.gw * kWave; i0 < nact; i0 += g.nw * kWave) {
    uint32_t s;
    const bool ok = select_source(a, i0 + lane_id(), nact, false, s);
    if (ok) trav += a.malive[s];
    tokens += tp_forward(a, wr, s, s, kNone, 0, ok, s);
  }
  tree_barrier(a.gbar);
  if (ld_dev(&st->lp[0])) {  // the sources' long rows, spread over every wave
    tokens += tp_pieces(a, g, 0);
    tree_barrier(a.gbar);
  }
  wave_add(&st->trav, trav);
  wave_add(&st->tokens, tokens);
  tree_barrier(a.gbar);
  if (blockIdx.x == 0 && threadIdx.x == 0) st->tstamp[1] = __builtin_amdgcn_s_memrealtime();
  const uint64_t nsrc = ld_dev(&st->nsrc);
  if (nsrc == 0) return;  // no tokens, nothing to post-process (every block agrees)
  const bool single = nsrc <= a.small_line && ld_dev(&st->ftotal) <= a.small_line;
  if (!single) {
    path_rest(a, g, false, s_hist, wr);
    return;
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) st->single = 1;
    path_rest(a, block_idx(), true, s_hist, wr);
  }
  tree_barrier(a.gbar);  // (the other blocks wait for block 0 here)
  const unsigned ek = ld_dev(&st->esc_k);
  if (ek) path_rest(a, g, false, s_hist, wr, static_cast<int>(ek), ld_dev(&st->esc_base));
}

// ---- TDS lines (tds_batch_1) -------------------------------------------
// Positions 2..C+1, terminal and post-processing.  Walks of position L are
// stored from wbase[L] on (fresh, 128-B aligned memory per position); kept
// walks are appended to the launch's kept buffer.
// Returns true when block 0 (single) handed the line to the grid at position esc_k.
__device__ __forceinline__ bool tds_rest(const LineKernelArgs& a, const GridIdx& g, bool single,
                                         unsigned long long* s_hist, WaveRows& wr, uint64_t kept_base,
                                         int k0 = 1, uint64_t in_base0 = 0) {
  LineStats* st = a.st;
  const LineArgs& la = s_la;
  const int stride = la.C + 2;
  uint64_t trav = 0, tokens = 0, in_base = in_base0;
  // single block: the walk counters live in LDS (no global atomic per wave and round)
  const bool stage = stride <= kStage;
  if (single) {
    if (threadIdx.x < 20) {
      wr.wn[threadIdx.x] = threadIdx.x == 1 ? ld_dev(&st->wn[1]) : 0ull;
      wr.lpany[threadIdx.x] = 0u;
    }
    __syncthreads();
  }
  const int wv = threadIdx.x / kWave, lane = lane_id();
  // the overflow flag and the next position's walk count, read together after each position's barrier (and
  // the long-row piece count with them): three independent loads instead of a chain across the boundary
  unsigned ovf_next = ld_dev(&st->overflow);
  uint64_t nin_next = single ? 0 : ld_dev(&st->wn[k0]);
  for (int k = k0; k <= la.C; ++k) {
    k = __builtin_amdgcn_readfirstlane(k);  // (uniform: the line's constants indexed by k load through the scalar cache)
    if (ovf_next) break;
    const uint64_t nin = single ? wr.wn[k] : nin_next;
    if (single && nin > a.small_line) {  // the walks outgrew the block: the grid takes position k
      if (threadIdx.x >= 2 && threadIdx.x <= static_cast<unsigned>(k)) st->wn[threadIdx.x] = wr.wn[threadIdx.x];
      wave_add(&st->trav, trav);
      wave_add(&st->tokens, tokens);
      if (g.tid == 0) {
        st->esc_base = in_base;
        st->esc_k = static_cast<unsigned>(k);
      }
      return true;
    }
    const uint64_t out_base = (in_base + nin * stride + 31) & ~uint64_t(31);
    tokens += g.tid == 0 ? nin : 0;
    const uint32_t* win = a.wbuf + in_base;
    unsigned long long* ctr = single ? &wr.wn[k + 1] : &st->wn[k + 1];
    const bool closing = k == la.C && la.VC;
    // walks per wave and pass: a position of a few hundred walks is spread over every wave (16 to 64 each), so
    // no wave walks the rows of 64 walks while others idle
    const uint64_t per = min<uint64_t>(kWave, max<uint64_t>(16, (nin + g.nw - 1) / g.nw));
    for (uint64_t i0 = g.gw * per; i0 < nin; i0 += g.nw * per) {
      const uint64_t i = i0 + lane;
      uint64_t b = 0;
      uint32_t L = 0;
      const uint32_t* cw = nullptr;
      if (static_cast<uint64_t>(lane) < per && i < nin) {
        const uint32_t* w = win + i * stride;
        uint32_t u;
        if (stage) {  // the walk's positions (independent loads) into the wave's stage
          uint32_t* sw = wr.walk[wv] + lane * stride;
#pragma unroll
          for (int p = 0; p < kStage; ++p)
            if (p <= k) sw[p] = w[p];
          u = sw[k];
          w = sw;
        } else {
          u = w[k];
        }
        // the row of u is fetched together with its T_pub (used if the arrival checks pass)
        const uint16_t T = a.tpub[u];
        const uint64_t ob = a.offp[u];
        uint32_t ml = a.mlen[u], ma = a.malive[u];
        if (!row_ok(a, u, ob, ml)) ml = 0;
        if (a.stamps && g.tid == 0 && i0 == g.gw * per) {  // (diagnostics: the first walks' state is in)
          __builtin_amdgcn_s_waitcnt(0);
          st->pmid[k][0] = __builtin_amdgcn_s_memrealtime() + (T & 0u) + (ml & 0u);
        }
        if (pos_ok(T, k, la) && enum_ok(w, k, u, la)) {
          b = ob;
          L = ml;
          trav += ma;
          if (closing) {
            // the closing step of a cycle walk: its only child is w[0] (tds_child_ok), searched for in the row
            L = row_has_alive(a, b, b + L, w[0]) ? 1u : 0u;
            cw = w;
          } else if (L > kLineLong && i <= 0xFFFFFFFFull && line_pieces(a, k, static_cast<uint32_t>(i), L, wr.lpany)) {
            L = 0;
          }
        }
      }
      if (closing) {
        const uint64_t pos = wave_reserve(ctr, L);
        if (L) {
          uint32_t* o = a.wbuf + out_base;
          if ((pos + 1) * stride <= (a.wcap > out_base ? a.wcap - out_base : 0)) {
            uint32_t* d = o + pos * stride;
            for (int p = 0; p <= k; ++p) d[p] = cw[p];
            d[k + 1] = cw[0];
          } else {
            atomicOr(&st->overflow, 1u);
          }
        }
        continue;
      }
      __builtin_amdgcn_wave_barrier();
      if (a.stamps && g.gw == 0) {  // (diagnostics: entries of thread 0's wave)
        const uint64_t tw = wave_sum(uint64_t(L));
        if (lane == 0) st->pmid[k][2] += tw;
      }
      tds_expand_wave(a, wr, win, i0, k, b, L, a.wbuf + out_base, a.wcap > out_base ? a.wcap - out_base : 0, stride,
                      stage, ctr);
    }
    if (a.stamps && g.tid == 0) st->pmid[k][1] = __builtin_amdgcn_s_memrealtime();
    phase_sync(a, single);
    const bool pieces = single ? wr.lpany[k] != 0u : ld_dev(&st->lp[k]) != 0ull;
    ovf_next = ld_dev(&st->overflow);
    nin_next = single ? 0 : ld_dev(&st->wn[k + 1]);
    if (pieces) {  // the position's long rows, over every wave
      tds_pieces(a, g, k, win, a.wbuf + out_base, a.wcap > out_base ? a.wcap - out_base : 0, stride, ctr);
      phase_sync(a, single);
      ovf_next = ld_dev(&st->overflow);
      nin_next = single ? 0 : ld_dev(&st->wn[k + 1]);
    }
    in_base = out_base;
    if (a.stamps && g.tid == 0) st->ptime[k] = __builtin_amdgcn_s_memrealtime();
  }
  // (diagnostics: a single block's walk counts, kept in LDS, for the phase-time print)
  if (single && a.stamps && threadIdx.x >= 2 && threadIdx.x < 20) st->wn[threadIdx.x] = wr.wn[threadIdx.x];
  // every final walk may be kept: its room must exist before any terminal effect
  const uint64_t nw = single ? wr.wn[la.C + 1] : ld_dev(&st->wn[la.C + 1]);
  // kept slots used by the launch's earlier lines (read at line start: the
  // terminal loop below adds to the counter while slower blocks still enter it)
  const uint64_t kept0 = kept_base;
  if (ld_dev(&st->overflow) || kept0 + nw * stride > a.kept_cap) {
    if (g.tid == 0) atomicOr(&st->overflow, 1u);
    wave_add(&st->trav, trav);
    return false;
  }
  // terminal position C+1 (tds_batch_1.hpp:641-758)
  {
    const int k = la.C + 1;
    tokens += g.tid == 0 ? nw : 0;
    if (g.tid == 0) st->wbase[0] = kept0;  // this line's kept walks start here (u32 slots)
    uint64_t kept = 0;
    for (uint64_t i0 = g.gw * kWave; i0 < nw; i0 += g.nw * kWave) {
      const uint64_t i = i0 + lane_id();
      bool kp = false;
      const uint32_t* w = a.wbuf + in_base + (i < nw ? i : 0) * stride;
      if (i < nw) {
        const uint32_t u = w[k], s = w[0];
        if (pos_ok(a.tpub[u], k, la)) {
          if (!la.VC) {
            if (u != s) {
              kp = true;
              if (a.tpub[s]) a.tsm[s] = 2;
            }
          } else if (u == s) {
            kp = true;
            a.tsm[s] = 2;
          }
        }
      }
      const uint64_t pos = wave_reserve(a.kept_ctr, kp ? static_cast<uint32_t>(stride) : 0u);
      if (kp) {
        uint32_t* d = a.kept + pos;
        for (int p = 0; p < stride; ++p) d[p] = w[p];
      }
      kept += kp;
    }
    wave_add(&st->walks, kept);
  }
  wave_add(&st->trav, trav);
  wave_add(&st->tokens, tokens);
  phase_sync(a, single);
  if (!a.split) line_post(a, g, s_hist);
  return false;
}

__device__ __forceinline__ void tds_line(const LineKernelArgs& a, unsigned long long* s_hist, WaveRows& wr) {
  const GridIdx g = grid_idx();
  LineStats* st = a.st;
  const int stride = s_la.C + 2;
  uint64_t trav = 0;
  // P1 + position 1 walks [s, w]; region 1 starts at slot 0
  const uint64_t kept_base = ld_dev(a.kept_ctr);  // no kept walk of this line exists yet
  const uint64_t nact = ld_dev(a.nact);
  for (uint64_t i0 = g.gw * kWave; i0 < nact; i0 += g.nw * kWave) {
    uint32_t s;
    const bool ok = select_source(a, i0 + lane_id(), nact, true, s);
    uint64_t b = 0;
    uint32_t L = 0;
    if (ok) {
      b = a.offp[s];
      L = a.mlen[s];
      trav += a.malive[s];
      if (!row_ok(a, s, b, L)) L = 0;
      if (L > kLineLong && line_pieces(a, 0, s, L, wr.lpany)) L = 0;  // (the pieces: tds_pieces)
    }
    // walks [s, w] for every alive w in M[s] (flattened over the wave's sources)
    const int wv = threadIdx.x / kWave, lane = lane_id();
    const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(L));
    const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
    if (!total) continue;
    wr.beg[wv][lane] = b;
    wr.end[wv][lane] = incl;
    wr.t.s[wv][lane] = s;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t t0 = 0; t0 < total; t0 += kWave) {
      const uint32_t t = t0 + lane;
      uint32_t m = 0, sr = 0;
      if (t < total) {
        const int r = row_of(wr.end[wv], t);
        const uint32_t first = r ? wr.end[wv][r - 1] : 0u;
        m = a.mcol[wr.beg[wv][r] + (t - first)];
        sr = wr.t.s[wv][r];
      }
      const bool alive = (m & kAlive) != 0;
      const uint64_t pos = wave_reserve(&st->wn[1], alive ? 1u : 0u);
      if (alive) {
        if ((pos + 1) * stride <= a.wcap) {
          a.wbuf[pos * stride + 0] = sr;
          a.wbuf[pos * stride + 1] = m & kPosMask;
        } else {
          atomicOr(&st->overflow, 1u);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  wave_add(&st->trav, trav);
  tree_barrier(a.gbar);
  if (ld_dev(&st->lp[0])) {  // the sources' long rows, spread over every wave
    tds_pieces(a, g, 0, nullptr, a.wbuf, a.wcap, stride, &st->wn[1]);
    tree_barrier(a.gbar);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) st->tstamp[1] = __builtin_amdgcn_s_memrealtime();
  const uint64_t nsrc = ld_dev(&st->nsrc);
  if (nsrc == 0) return;  // no walks, nothing to post-process (every block agrees)
  const bool single = nsrc <= a.small_line && ld_dev(&st->wn[1]) <= a.small_line;
  if (!single) {
    tds_rest(a, g, false, s_hist, wr, kept_base);
    return;
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) st->single = 1;
    tds_rest(a, block_idx(), true, s_hist, wr, kept_base);
  }
  tree_barrier(a.gbar);  // (the other blocks wait for block 0 here)
  const unsigned ek = ld_dev(&st->esc_k);
  if (ek) tds_rest(a, g, false, s_hist, wr, kept_base, static_cast<int>(ek), ld_dev(&st->esc_base));
}

// NLC lines [pl_begin, pl_end) in order, one grid barrier at each line end
// (the next line's sources see its post-processing).  Stops after a line
// that overflowed or that deleted with interleave_lp set (the host runs the
// interleaved LCC, beta.cpp:1163-1197, then relaunches).
__global__ __launch_bounds__(kLineBlock) void k_lines(LineKernelArgs a) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ WaveRows wr;
  unsigned long long* kst = reinterpret_cast<unsigned long long*>(a.gbar + kGbarWords + 8);  // diagnostics
  if (blockIdx.x == 0 && threadIdx.x == 0) kst[0] = __builtin_amdgcn_s_memrealtime();
  build_active(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) kst[1] = __builtin_amdgcn_s_memrealtime();
  tree_barrier(a.gbar);
  // Source census of every line of the launch on the state as it stands (select_source's test, counted only):
  // a line that finds no source changes nothing, so the census stays exact up to the first line that has
  // sources, and the lines before it are skipped without their selection pass and two grid barriers each.
  {
    const GridIdx g = grid_idx();
    const uint64_t nact = ld_dev(a.nact);
    for (int pl = a.pl_begin; pl < a.pl_end; ++pl) {
      const LineArgs& la = a.lines[pl].la;
      const bool tds = a.lines[pl].tds != 0;
      uint64_t cnt = 0, tok = 0;
      for (uint64_t i0 = g.gw * kWave; i0 < nact; i0 += g.nw * kWave) {
        const uint64_t i = i0 + lane_id();
        if (i < nact) {
          const uint32_t s = ld_dev(&a.act[i]);
          const uint16_t T = a.tpub[s];
          bool ok = T && pos_ok(T, 0, la);
          if (ok && !tds && !la.VC && !((T >> la.ilast) & 1u)) ok = false;
          cnt += ok ? 1u : 0u;
          tok += ok ? a.malive[s] : 0u;
        }
      }
      wave_add(&a.st[pl].census, cnt);
      if (a.split_min) wave_add(&a.st[pl].census_tok, tok);
    }
    tree_barrier(a.gbar);
  }
  bool fresh = true;  // no line of this launch has changed the state yet
  for (int pl = a.pl_begin; pl < a.pl_end; ++pl) {
    const LineDesc& d = a.lines[pl];
    const unsigned long long cen = ld_dev(&a.st[pl].census);
    if (fresh && cen == 0) {
      if (blockIdx.x == 0 && threadIdx.x == 0) *a.done = static_cast<unsigned>(pl + 1);
      continue;
    }
    // a split line is decided on an exact census only -- the replica's sources, identical on every shard --
    // so every shard splits the same lines: after a line of this launch changed the state the census is a
    // bound, and a line it would split ends the launch unprocessed (the next launch counts again)
    const bool split = a.split_min && a.so.nranks > 1 && ld_dev(&a.st[pl].census_tok) >= a.split_min;
    if (split && !fresh) break;
    fresh = false;
    __syncthreads();  // (every wave is done with the previous line's constants)
    if (threadIdx.x < sizeof(LineArgs) / sizeof(uint32_t))
      reinterpret_cast<uint32_t*>(&s_la)[threadIdx.x] = reinterpret_cast<const uint32_t*>(&d.la)[threadIdx.x];
    __syncthreads();
    LineKernelArgs b = a;
    b.la = &d.la;
    b.i0 = d.i0;
    b.st = a.st + pl;
    b.split = split ? 1 : 0;
    if (b.split && blockIdx.x == 0 && threadIdx.x == 0) b.st->split = 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) b.st->tstamp[0] = __builtin_amdgcn_s_memrealtime();
    if (d.tds) tds_line(b, s_hist, wr);
    else path_line(b, s_hist, wr);
    if (blockIdx.x == 0 && threadIdx.x == 0) b.st->tstamp[2] = __builtin_amdgcn_s_memrealtime();
    tree_barrier(a.gbar);
    if (blockIdx.x == 0 && threadIdx.x == 0) b.st->tstamp[3] = __builtin_amdgcn_s_memrealtime();
    // a split line ends the launch: the shards exchange its effects before the next line selects sources
    const bool stop = ld_dev(&b.st->overflow) || (d.il && ld_dev(&b.st->deleted)) || b.split;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.done = static_cast<unsigned>(pl + 1);
    if (stop) break;
  }
}

// ---------------------------------------------------------------------------
// host side
template <typename T>
static T* dmalloc(uint64_t n) {
  T* p = nullptr;
  PM_HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(1, n) * sizeof(T)));
  return p;
}

static void ensure_hash(Ctx& c, uint64_t want) {
  uint64_t cap = 1ull << 10;
  while (cap < want && cap < (1ull << 31)) cap <<= 1;
  if (c.hcap >= cap) return;
  if (c.d_hkey) (void)hipFree(c.d_hkey);
  if (c.d_hval) (void)hipFree(c.d_hval);
  if (c.d_front) (void)hipFree(c.d_front);
  c.d_hkey = dmalloc<unsigned long long>(cap);
  c.d_hval = dmalloc<unsigned long long>(cap);
  c.d_front = dmalloc<uint32_t>(cap / 2);
  PM_HIP_CHECK(hipMemsetAsync(c.d_hkey, 0xFF, cap * sizeof(unsigned long long), c.stream));
  PM_HIP_CHECK(hipMemsetAsync(c.d_hval, 0xFF, cap * sizeof(unsigned long long), c.stream));
  c.hcap = cap;
}

// After a path / cycle line overflowed the (source, vertex) table: partial inserts are not all recorded in the
// frontier list, so the table is cleared; it grows 4x while the device has room (c.hash_regrown: the caller
// reruns the line on the fused path), else the line goes to the exact per-position path.
// Sharded replica: every shard overflows the same line (the table and the arena have one size on every shard and
// the frontier count that overflows is order independent), so every shard is here; the room is agreed over the
// shards, so that all of them rerun the line fused (a split line: its collectives) or all take the exact path.
static void regrow_hash(Ctx& c) {
  PM_HIP_CHECK(hipMemsetAsync(c.d_hkey, 0xFF, c.hcap * sizeof(unsigned long long), c.stream));
  PM_HIP_CHECK(hipMemsetAsync(c.d_hval, 0xFF, c.hcap * sizeof(unsigned long long), c.stream));
  const uint64_t grow = c.hcap * 4;
  constexpr uint64_t kSlotBytes = 2 * sizeof(unsigned long long) + sizeof(uint32_t) / 2;  // key, value, frontier
  size_t free_b = 0, total_b = 0;
  PM_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
  bool room = grow <= (1ull << 31) && grow * kSlotBytes + (size_t(2) << 30) <= free_b + c.hcap * kSlotBytes;
  if (c.nogrow_shard == static_cast<int64_t>(c.shard) && (c.comm || c.nogrow_shard == 0))
    room = false;  // (PM_DEBUG_NOGROW_SHARD, tests; 0 on one context: its local split lines)
  room = shard_agree_min(c, room ? 1 : 0) != 0;
  if (!room) return;
  ensure_hash(c, grow);
  c.hash_regrown = true;
}

void free_line_buffers(Ctx& c) {
  void* ptrs[] = {c.d_hkey, c.d_hval, c.d_front, c.d_gbar, c.d_ldesc};  // (d_lstats lives in d_gbar)
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  c.d_lstats = nullptr;
  c.d_hkey = c.d_hval = nullptr;
  c.d_front = nullptr;
  c.d_gbar = nullptr;
  c.d_ldesc = nullptr;
  c.hcap = 0;
}

static void upload_lines(Ctx& c) {
  if (c.d_ldesc) return;
  const size_t nl = c.pattern.lines.size();
  std::vector<LineDesc> h(std::max<size_t>(nl, 1));
  for (size_t pl = 0; pl < nl; ++pl) {
    const NlcLine& line = c.pattern.lines[pl];
    h[pl] = LineDesc{};
    h[pl].la = make_line_args(c, line);
    h[pl].tds = pl >= 4 ? 1 : 0;
    h[pl].i0 = static_cast<int32_t>(line.indices[0]);
    h[pl].il = line.interleave_lp ? 1 : 0;
  }
  c.d_ldesc = dmalloc<LineDesc>(h.size());
  PM_HIP_CHECK(hipMemcpy(c.d_ldesc, h.data(), h.size() * sizeof(LineDesc), hipMemcpyHostToDevice));
  c.d_lstats_n = nl;
}

// Enqueues lines [pl0, nl) and the read-back of their results into the lines'
// pinned buffer; returns nl (pl0 >= nl: nothing launched).
static size_t launch_lines(Ctx& c, size_t pl0, size_t max_lines, uint32_t*& kept_out) {
  if (c.comm && !c.replicated) throw std::runtime_error("internal: fused lines before the sharded state was replicated");
  c.probe("lines entry");
  const size_t nl_all = c.pattern.lines.size();
  const size_t nl = pl0 < nl_all && max_lines < nl_all - pl0 ? pl0 + max_lines : nl_all;
  kept_out = nullptr;
  if (pl0 >= nl) return nl;
  for (size_t pl = pl0; pl < nl; ++pl) {
    const NlcLine& line = c.pattern.lines[pl];
    const size_t stride = line.cycle_length + 2;
    if (pl >= 4 && line.enumeration.size() < stride)
      throw std::runtime_error("pattern_non_local_constraint enumeration shorter than the TDS walk");
    if (stride > 18) throw std::runtime_error("NLC line longer than 16 positions");
  }
  upload_lines(c);
  // one buffer: grid barrier state | 64 control words (lines done, kept-walk counter, ...) | LineStats per
  // line -- the control words and the stats are cleared by one fill and read back by one copy
  static_assert(((kGbarWords + 64) * sizeof(unsigned)) % alignof(LineStats) == 0, "LineStats alignment");
  static_assert(sizeof(LineStats) % sizeof(unsigned) == 0, "LineStats size");
  if (!c.d_lstats) {
    const size_t words = kGbarWords + 64 + std::max<size_t>(nl_all, 1) * (sizeof(LineStats) / sizeof(unsigned)) + 16;
    c.d_gbar = dmalloc<unsigned>(words);
    PM_HIP_CHECK(hipMemsetAsync(c.d_gbar, 0, words * sizeof(unsigned), c.stream));
    c.d_lstats = reinterpret_cast<LineStats*>(c.d_gbar + kGbarWords + 64);
    c.lines_ctl_clean = true;
  }
  if (!c.line_grid) {
    int per_cu = 0;
    PM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lines, kLineBlock, 0));
    hipDeviceProp_t prop;
    PM_HIP_CHECK(hipGetDeviceProperties(&prop, c.device));
    if (per_cu < 1) throw std::runtime_error("fused line kernel cannot be resident");
    // one block per CU: the barrier cost grows with the number of blocks
    c.line_grid = static_cast<unsigned>(std::min<int>(prop.multiProcessorCount, 1024));
  }
  // the table is sized from the superstep-0 matching rows (upper bound of |S|); a replica by its rows, the same
  // on every shard
  // (PM_HASH_SLOTS, diagnostics: the first table of the context has that many slots -- tests force overflows)
  ensure_hash(c, c.hash_slots ? c.hash_slots
                              : std::max<uint64_t>(1ull << 20, 4 * (c.replicated ? uint64_t(c.nS_host) : c.ss0_rows)));
  unsigned* d_done = c.d_gbar + kGbarWords;                                   // [0] lines done
  auto* d_kept_ctr = reinterpret_cast<unsigned long long*>(c.d_gbar + kGbarWords + 2);
  const size_t ctl_bytes = 64 * sizeof(unsigned) + nl * sizeof(LineStats);  // control words + stats of lines < nl
  // (the fill rounded up to 64 B -- the buffer has the slack: one fill kernel instead of an aligned part and a tail)
  // The search's first launch finds them cleared by the search's zero batch (queue_lines_ctl_clear)
  if (!c.lines_ctl_clean) PM_HIP_CHECK(hipMemsetAsync(d_done, 0, (ctl_bytes + 63) & ~size_t(63), c.stream));
  c.lines_ctl_clean = false;
  LineKernelArgs a{};
  a.offp = m_off(c);
  a.mcol = m_col(c);
  a.mlen = c.d_mlen;
  a.malive = c.d_malive;
  a.tpub = c.d_tpub[c.cur];
  a.perm = c.d_perm;
  a.tsm = c.d_tsm;
  a.slist = c.d_slist;
  a.nS = c.d_nS;
  a.smask = c.smask_valid ? reinterpret_cast<const unsigned long long*>(c.d_smask[c.smask_cur]) : nullptr;
  a.sources = c.d_sources;
  a.oa.hubs = c.d_hubs;
  a.oa.perm = c.d_perm;
  a.oa.nhubs = static_cast<uint32_t>(c.hubs_host.size());
  a.oa.nranks = c.nranks;
  a.gbar = c.d_gbar;
  a.hkey = c.d_hkey;
  a.hval = c.d_hval;
  a.hmask = c.hcap - 1;
  a.front = c.d_front;
  a.fcap = c.hcap / 2;
  a.st = c.d_lstats;
  a.lines = c.d_ldesc;
  static const uint64_t small_line =
      std::getenv("PM_SMALL_LINE") ? std::strtoull(std::getenv("PM_SMALL_LINE"), nullptr, 10) : kSmallLine;
  a.small_line = small_line;
  static const bool phase_stamps = std::getenv("PM_PHASE_TIMES") != nullptr;
  a.stamps = phase_stamps ? 1 : 0;
  // split lines (sharded replica): owner rule of the shards, the flag list
  a.so.hubs = c.d_hubs;
  a.so.perm = c.d_perm;
  a.so.nhubs = static_cast<uint32_t>(c.hubs_host.size());
  a.so.nranks = c.comm ? c.nshards : 1;
  a.shard = c.shard;
  a.split_min = c.comm && c.nshards > 1 && c.pattern.lines.size() && !c.any_sv ? c.split_min : 0;
  if (c.lsplit_parts > 1) {  // one context, a local split line's part (local_split_line): flags set in place
    a.so.nranks = c.lsplit_parts;
    a.shard = c.lsplit_part;
    a.split_min = 1;
    a.xflag = nullptr;
    a.xflag_cap = 0;
  } else if (a.split_min) {
    const uint64_t want = m_cap(c) + c.nS_host + 2;
    if (c.xsplit_cap < want) {
      if (c.d_xsplit) (void)hipFree(c.d_xsplit);
      c.d_xsplit = nullptr;
      PM_HIP_CHECK(hipMalloc(&c.d_xsplit, want * sizeof(unsigned long long)));
      c.xsplit_cap = want;
    }
    a.xflag = c.d_xsplit;
    a.xflag_cap = m_cap(c);
    a.nxflag = reinterpret_cast<unsigned long long*>(c.d_gbar + kGbarWords + 6);  // zeroed with d_done
  }
  static const bool dbg_rows = std::getenv("PM_DEBUG_SYNC") != nullptr;
  a.dbg = dbg_rows ? reinterpret_cast<unsigned long long*>(c.d_gbar + kGbarWords + 16) : nullptr;  // zeroed below
  a.n = c.n;
  a.mcap = m_cap(c);
  a.pl_begin = static_cast<int>(pl0);
  a.pl_end = static_cast<int>(nl);
  a.done = d_done;
  a.kept_ctr = d_kept_ctr;
  a.nact = reinterpret_cast<unsigned long long*>(c.d_gbar + kGbarWords + 4);  // zeroed with d_done
  c.arena.reset();
  a.act = static_cast<uint32_t*>(c.arena.get(std::max<uint64_t>(c.nS_host, 1) * sizeof(uint32_t)));
  // long-row pieces of one position (a full list leaves the rest of the rows to their waves)
  a.lp_cap = std::min<uint64_t>(1ull << 22, std::max<uint64_t>(1024, m_cap(c) / kLineLong * 4));
  a.lpieces = static_cast<unsigned long long*>(c.arena.get(a.lp_cap * sizeof(unsigned long long)));
  const uint64_t room = (c.arena.cap - c.arena.used - 8192) / sizeof(uint32_t);
  a.kept_cap = room / 4;
  a.kept = static_cast<uint32_t*>(c.arena.get(a.kept_cap * sizeof(uint32_t)));
  a.wcap = (c.arena.cap - c.arena.used - 4096) / sizeof(uint32_t);
  // PM_TDS_CAP (tests): the fused walk storage is bounded too, so that a larger enumeration overflows into the
  // exact path's chunked enumeration
  if (const char* e = std::getenv("PM_TDS_CAP")) a.wcap = std::min<uint64_t>(a.wcap, std::strtoull(e, nullptr, 10));
  // PM_FUSED_WCAP (tests): the fused walk storage alone bounded (a TDS line then overflows into a local split)
  if (const char* e = std::getenv("PM_FUSED_WCAP")) a.wcap = std::min<uint64_t>(a.wcap, std::strtoull(e, nullptr, 10));
  a.wbuf = static_cast<uint32_t*>(c.arena.get(a.wcap * sizeof(uint32_t)));
  void* args[] = {&a};
  c.probe("lines launch");
  // few state-map members: a smaller grid (dispatching the full one costs ~50 us
  // before the first grid barrier completes)
  // (live_hint ~0: unknown after a relayout -- the full grid; the rounding must not wrap)
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(
      16, c.live_hint == ~0ull ? c.line_grid : std::min<uint64_t>(c.line_grid, c.live_hint / 256 + 1)));
  if (!c.coop)  // (one context on the device, Ctx::coop)
    PM_HIP_CHECK(hipLaunchKernel(reinterpret_cast<const void*>(k_lines), dim3(grid), dim3(kLineBlock), args, 0,
                                 c.stream));
  else
    PM_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_lines), dim3(grid), dim3(kLineBlock), args,
                                            0, c.stream));
  c.probe("lines launched");
  debug_point(c, "NLC line kernel");
  // read-back through pinned memory, one copy: [done | . | kept slots | ... (64 words) | line stats]
  static_assert(sizeof(LineStats) % 8 == 0, "LineStats is read back as u64 words");
  const size_t words = ctl_bytes / 8;
  if (c.h_pin_lines_words < words) {
    if (c.h_pin_lines) (void)hipHostFree(c.h_pin_lines);
    c.h_pin_lines = nullptr;
    const size_t w = std::max<size_t>(words, 1 << 12);
    PM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c.h_pin_lines), w * sizeof(uint64_t), hipHostMallocDefault));
    c.h_pin_lines_words = w;
  }
  uint64_t* pin = c.h_pin_lines;
  PM_HIP_CHECK(hipMemcpyAsync(pin, d_done, ctl_bytes, hipMemcpyDeviceToHost, c.stream));
  kept_out = a.kept;
  return nl;
}

// The control words and line statistics of a search's first line launch, cleared with the search's other fills
// (one batched launch at its start instead of a fill in front of the lines).
void queue_lines_ctl_clear(Ctx& c) {
  if (!c.d_gbar || c.pattern.lines.empty()) return;
  const size_t ctl_bytes = 64 * sizeof(unsigned) + c.pattern.lines.size() * sizeof(LineStats);
  zero_later(c, c.d_gbar + kGbarWords, (ctl_bytes + 63) & ~size_t(63));
  c.lines_ctl_clean = true;
}

LineStats run_line_part(Ctx& c, size_t pl, uint32_t parts, uint32_t part, uint32_t*& kept_dev) {
  if (c.comm || c.lines_prelaunched) throw std::runtime_error("internal: local split line on a sharded or busy context");
  c.lsplit_parts = parts;
  c.lsplit_part = part;
  try {
    launch_lines(c, pl, 1, kept_dev);
  } catch (...) {
    c.lsplit_parts = 0;
    throw;
  }
  c.lsplit_parts = 0;
  stream_wait(c.stream);
  LineStats st;
  std::memcpy(&st, reinterpret_cast<const char*>(c.h_pin_lines) + 64 * sizeof(unsigned) + pl * sizeof(LineStats),
              sizeof(LineStats));
  if (st.overflow) {  // (partial inserts are not all in the frontier list: the table is cleared)
    PM_HIP_CHECK(hipMemsetAsync(c.d_hkey, 0xFF, c.hcap * sizeof(unsigned long long), c.stream));
    PM_HIP_CHECK(hipMemsetAsync(c.d_hval, 0xFF, c.hcap * sizeof(unsigned long long), c.stream));
  }
  return st;
}

void prelaunch_lines_fused(Ctx& c) {
  c.pre_pl0 = 0;
  c.pre_nl = launch_lines(c, 0, SIZE_MAX, c.pre_kept);
  c.lines_prelaunched = true;
}

size_t run_lines_fused(Ctx& c, size_t pl0, bool want_walks, std::vector<FusedLineOut>& outs, bool& overflow,
                       size_t max_lines) {
  overflow = false;
  outs.clear();
  size_t nl;
  uint32_t* kept_dev = nullptr;
  if (c.lines_prelaunched && pl0 == c.pre_pl0 && max_lines == SIZE_MAX) {
    nl = c.pre_nl;
    kept_dev = c.pre_kept;
  } else {
    if (c.lines_prelaunched) throw std::runtime_error("internal: prelaunched NLC lines not consumed in order");
    nl = launch_lines(c, pl0, max_lines, kept_dev);
  }
  c.lines_prelaunched = false;
  if (pl0 >= nl) return 0;
  uint64_t* pin = c.h_pin_lines;
  stream_wait(c.stream);
  c.probe("lines synced");
  std::vector<LineStats> hs(nl - pl0);
  std::memcpy(hs.data(), reinterpret_cast<const char*>(pin) + 64 * sizeof(unsigned) + pl0 * sizeof(LineStats),
              hs.size() * sizeof(LineStats));
  const unsigned done = static_cast<unsigned>(pin[0] & 0xFFFFFFFFull);
  const unsigned long long kept_slots = pin[1];
  if (pin[8])  // (PM_DEBUG_SYNC row checks, control words 16-23)
    throw std::runtime_error("NLC line kernel: row of vertex " + std::to_string(pin[9]) + " at " +
                             std::to_string(pin[10]) + " + " + std::to_string(pin[11]) + " outside the M buffer (" +
                             std::to_string(m_cap(c)) + " entries, shard " + std::to_string(c.shard) +
                             (c.replicated ? ", replica)" : ")"));
  {  // device time of the launch: its start stamp (kst[0], control word 4) to the last processed line's end
    unsigned long long end = pin[5];
    for (unsigned j = 0; j + pl0 < done; ++j) end = std::max(end, hs[j].tstamp[3]);
    if (pin[4] && end > pin[4]) c.lines_seconds += (end - pin[4]) * 1e-8;  // s_memrealtime: 100 MHz
  }
  std::vector<uint32_t> kept;
  if (want_walks && kept_slots) {
    kept.resize(kept_slots);
    PM_HIP_CHECK(hipMemcpy(kept.data(), kept_dev, kept_slots * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  const uint32_t P = c.nranks <= 1 ? 1 : c.nranks;
  static const bool phase_times = std::getenv("PM_PHASE_TIMES") != nullptr;
  if (phase_times) {
    unsigned long long ks[2] = {0, 0};
    PM_HIP_CHECK(hipMemcpy(ks, c.d_gbar + kGbarWords + 8, sizeof(ks), hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[pm] lines launch: active list %.1f us, to line start %.1f us\n", (ks[1] - ks[0]) * 0.01,
                 (hs[0].tstamp[0] - ks[1]) * 0.01);
  }
  if (phase_times)
    for (unsigned j = 0; j + pl0 < done; ++j) {
      const LineStats& st = hs[j];
      std::fprintf(stderr,
                   "[pm] line %zu: P1 %.1f us, rest %.1f us, end barrier %.1f us (%s, %llu sources, census %llu "
                   "sources / %llu tokens%s)\n",
                   pl0 + j, (st.tstamp[1] - st.tstamp[0]) * 0.01, (st.tstamp[2] - st.tstamp[1]) * 0.01,
                   (st.tstamp[3] - st.tstamp[2]) * 0.01, st.single ? "block 0" : "grid", st.nsrc, st.census,
                   st.census_tok, st.split ? ", split" : "");
      std::string pos = "[pm]   positions (walks in, us, long-row pieces):";
      unsigned long long prev = st.tstamp[1];
      for (int k = 1; k < 20 && st.ptime[k]; ++k) {
        char b[192];
        std::snprintf(b, sizeof(b), " %d:(%llu, %.1f, %llu)", k, st.wn[k], (st.ptime[k] - prev) * 0.01, st.lp[k]);
        if (st.pmid[k][1] > prev)  // TDS: [state of the first walks in, expansion done] after the position start
          std::snprintf(b + std::strlen(b), sizeof(b) - std::strlen(b), "[%.1f %.1f %llu]",
                        st.pmid[k][0] > prev ? (st.pmid[k][0] - prev) * 0.01 : 0.0, (st.pmid[k][1] - prev) * 0.01,
                        st.pmid[k][2]);
        pos += b;
        prev = st.ptime[k];
      }
      std::fprintf(stderr, "%s\n", pos.c_str());
    }
  if (c.comm && c.nshards > 1) {
    // Sharded replica: the shards act on one agreed first overflowed line.  Every shard overflows the same
    // replicated line as long as table sizes and insert outcomes are identical on all of them (regrow_hash);
    // should one shard overflow alone, regrow_hash's agreement would meet collectives the others never make.
    // So the first overflowed replicated line is gathered from every shard (one collective per launch): equal
    // everywhere -> every shard regrows and reruns it; different -> every shard fails with the same message
    // (the shards that went on have applied later lines' effects, so no rerun could restore one state).
    uint64_t first = ~0ull;
    for (unsigned j = 0; j + pl0 < done; ++j) {
      if (hs[j].split) break;  // (a split line is the launch's last; split_line_finish agrees on it)
      if (c.overflow_shard == static_cast<int64_t>(c.shard) && pl0 + j < 4) hs[j].overflow = 1;
      if (hs[j].overflow) {
        first = j;
        break;
      }
    }
    const std::vector<uint64_t> all = shard_gather_u64(c, first);
    if (*std::min_element(all.begin(), all.end()) != *std::max_element(all.begin(), all.end())) {
      std::string who;
      for (size_t g = 0; g < all.size(); ++g)
        who += (who.empty() ? "" : ", ") + ("shard " + std::to_string(g) + ": " +
                                            (all[g] == ~0ull ? std::string("none") : std::to_string(pl0 + all[g])));
      throw std::runtime_error("NLC line overflowed its table on some shards only (first overflowed line: " + who +
                               ")");
    }
  }
  size_t completed = 0;
  for (unsigned j = 0; j + pl0 < done; ++j) {
    const LineStats& st = hs[j];
    const size_t pl = pl0 + j;
    c.nsources = st.nsrc;
    if (st.split) {  // (the launch's last line) effects, stats and walks combined over the shards
      FusedLineOut out;
      out.stride = static_cast<uint32_t>(c.pattern.lines[pl].cycle_length + 2);
      if (!split_line_finish(c, pl, st, kept_dev, want_walks, out)) {  // some shard overflowed (all agree)
        overflow = true;
        if (pl < 4) regrow_hash(c);
        break;
      }
      c.last_acked = out.tr.acked;
      outs.push_back(std::move(out));
      ++completed;
      break;
    }
    if (st.overflow) {
      overflow = true;
      if (pl < 4) regrow_hash(c);
      break;
    }
    FusedLineOut out;
    out.tr.sources = st.nsrc;
    out.tr.acked = st.acked;
    out.tr.edges = st.trav;
    out.tr.tokens = st.tokens;
    out.tr.walks = st.walks;
    out.deleted = st.deleted ? 1u : 0u;
    c.last_acked = st.acked;
    out.rm_v.assign(c.nranks, 0);
    out.rm_e.assign(c.nranks, 0);
    for (uint32_t r = 0; r < c.nranks; ++r) {
      out.rm_v[r] = st.removed[r];
      out.rm_e[r] = st.removed[P + r];
    }
    out.stride = static_cast<uint32_t>(c.pattern.lines[pl].cycle_length + 2);
    if (pl >= 4 && want_walks && st.walks) {
      const uint64_t b = st.wbase[0];
      if (b + st.walks * out.stride > kept.size())
        throw std::runtime_error("internal: kept TDS walks out of range of the launch's buffer");
      out.walks.assign(kept.begin() + b, kept.begin() + b + st.walks * out.stride);
    }
    outs.push_back(std::move(out));
    ++completed;
  }
  c.probe("lines parsed");
  return completed;
}

}  // namespace pm
