// Internal declarations shared by the HIP kernels (pm_kernels.hip) and the
// host driver / C-ABI (pm_api.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "host/pattern.hpp"

namespace pm {

#define PM_HIP_CHECK(expr)                                                                         \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess)                                                                          \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

// Pattern constants passed by value to kernels.
struct PatArgs {
  uint16_t adj[16];     // adj[t]: template-neighbour mask of template vertex t
  uint64_t plabel[16];  // template labels
  int32_t K;            // number of template labels (pattern_vertex_data lines)
};

// Per-rank counter attribution (owner rule of delegate_partitioned_graph).
// Device state is indexed by label-major position; perm maps back to ids.
struct OwnerArgs {
  const uint64_t* hubs;  // sorted hub ids (device), may be null
  const uint32_t* perm;  // position -> vertex id
  uint32_t nhubs;
  uint32_t nranks;
};

// Position runs of the pattern's distinct labels in the label-major order:
// a vertex at position p carries template bits tu[l] iff lo[l] <= p < hi[l].
struct LabelRuns {
  uint32_t lo[16], len[16];
  uint32_t cd[16];  // code index of position p in run l: p + cd[l] (the runs packed one after the other)
  uint16_t tu[16];
  int32_t n;
  uint32_t ncode;   // positions in the runs (code indices 0 .. ncode-1)
};

// NLC line constants for the token-passing kernels.
struct LineArgs {
  uint16_t I[16];       // template index per walk position
  uint16_t E[16];       // enumeration index per position (TDS)
  uint8_t lok[16];      // L[k] == plabel[I[k]] (label test folded)
  int32_t C;            // cycle length: walk positions 0..C+1
  int32_t VC;           // valid cycle (expect target vertex)
  uint16_t ilast;       // pattern_indices.back()
  uint16_t sv;          // pattern_selected_vertices (nem_1.hpp:155-170, 409-436, 697-719)
};

// Collectives between the shards of one sharded search.  All
// buffers are device memory; the calls are stream ordered on `s` and every
// shard makes the same calls in the same order.  RcclComm (one process per
// GPU, RCCL over xGMI) and ThreadComm (several shards driven by threads of
// one process on one device, parity tests) implement it (pm_shard.hip).
struct Comm {
  virtual ~Comm() {}
  // collectives issued and bytes this shard contributed (send side), for the per-shard statistics
  uint64_t calls = 0, bytes = 0;
  double wall = 0.0;  // host seconds spent inside the collectives (the stream idles meanwhile)
  void count(uint64_t b) {
    ++calls;
    bytes += b;
  }
  struct Timer {  // adds the scope's host time to wall
    explicit Timer(Comm* c) : c_(c), t0_(std::chrono::steady_clock::now()) {}
    ~Timer() { c_->wall += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count(); }
    Comm* c_;
    std::chrono::steady_clock::time_point t0_;
  };
  // recv receives nshards consecutive `bytes` blocks, block g = shard g's send
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  virtual void allreduce_sum_u64(uint64_t* buf, size_t count, hipStream_t s) = 0;
  virtual void allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t s) = 0;
  // all-to-all of variable blocks: block g of send (sbytes[g] bytes, blocks
  // consecutive) goes to shard g; recv holds the blocks from shards 0..G-1
  // consecutively (rbytes[g] from shard g).  Host byte counts, device buffers.
  virtual void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes,
                         hipStream_t s) = 0;
  virtual int ranks() const = 0;      // ranks of the communicator as its transport reports them
  virtual int transport() const = 0;  // PM_TRANSPORT_* (pm_abi.h)
};

// Device scratch arena (bump allocator, reset per NLC line).  A request past its end throws ArenaFull (the exact
// path-line enumeration catches it and retries in smaller source batches).
struct ArenaFull : std::runtime_error {
  ArenaFull() : std::runtime_error("device scratch arena exhausted") {}
};
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  void* get(size_t bytes) {
    size_t a = (used + 255) & ~size_t(255);
    if (a + bytes > cap) throw ArenaFull();
    used = a + bytes;
    return base + a;
  }
  void reset() { used = 0; }
};

// Superstep-0 tiling of the padded label-major CSR (DESIGN.md "Data
// layout"): one entry per (pattern label, degree class) run of rows.  kind
// 0..kHeavyKind-1: rows of one light degree class, stored in G = kind_slots
// padded slots, so the run is a dense rows x G array and a tile is rpt =
// (kTileEntries - 4) / G whole rows (rpt * G consecutive slots); kind
// kHeavyKind: rows above kHeavyDeg (stored unpadded), one kHeavyDeg-entry
// segment per tile (HSeg list).
struct KRange {
  uint64_t qbase;       // first slot of the run
  uint32_t tile0;       // first tile of the run
  uint32_t start, end;  // row positions [start, end)
  uint32_t aux;         // heavy kind: first HSeg index
  uint16_t tu, nm;      // template bits of the label and their neighbour mask
  uint32_t kind;         // light degree class (kind_slots) or kHeavyKind
  uint32_t g, rpt;       // light: slots per row, whole rows per tile (rpt * g <= kTileEntries)
  uint32_t rdiv;         // light: slot / g == (slot * rdiv) >> 19 for slot < kTileEntries
  // light: row-start lanes of the 8 load groups (load k, component c: tile
  // slot 256 k + 4 lane + c - s) for each alignment shift s of the tile base
  uint64_t rs[4][8];
  // label runs whose template bits meet nm (the only neighbours that can
  // contribute), first four inline (len 0 = unused); nrel > 4 adds a scan of
  // all LabelRuns
  uint32_t rlo[4], rlen[4];
  uint16_t rtu[4];
  uint32_t nrel;
  // the same runs merged where they touch (membership only: superstep 0's
  // first pass), up to four (len 0 = unused), nadm > 4: use the runs above
  uint32_t alo[4], alen[4];
  uint32_t nadm;
  // verify (keep_bits) of the label's template bits: bit kbit[i] survives iff
  // kneed[i] is a subset of TN (kneed = adj[t], or 1 << 16 when adj[t] = 0);
  // nkeep > 4 falls back to the LDS loop
  uint16_t kbit[4];
  uint32_t kneed[4];
  uint32_t nkeep;
  uint32_t cdelta;  // code index of a row of the range: position + cdelta (LabelRuns::cd of its label)
};
static_assert(sizeof(KRange) == 416, "KRange: cdelta fills the tail padding (scalar-load layout unchanged)");
struct HSeg {
  uint32_t row;    // row position
  uint32_t seg;    // segment index inside the row
  uint32_t h;      // heavy-row ordinal (scratch slot)
  uint32_t nseg;   // segments of the row
  uint32_t range;  // KRange index
  uint32_t tile;   // tile index (survivor mask slot)
  uint32_t split;  // a delegate's share of a sharded search: TN / count stay partial (shard_hub_combine)
};
// A delegate (hub, degree >= -d) of a sharded search: its row is split over the
// shards by target owner (delegate_partitioned_graph.ipp:1402-1648), its state
// lives on the controller, hub ordinal % nshards (ipp:346-355).
struct HubInfo {
  uint32_t pos;   // position
  uint32_t hidx;  // heavy scratch slot of this shard's share (kNoHub: no share here)
  uint64_t moff;  // controller: first entry of its M row in the hub area of mcol
};
static constexpr uint32_t kNoHub = 0xFFFFFFFFu;
static constexpr int kSub = 8;                      // 64-slot sub-tiles per tile
static constexpr uint32_t kTileEntries = 64 * kSub; // 512
static constexpr uint32_t kHeavyDeg = kTileEntries; // heavy rows: segments of this many entries
// Rows per light tile at most (LDS per-row staging of k_lcc_first; G = 1 tiles hold 256 rows)
static constexpr uint32_t kTileRows = 256;
// Superstep-0 tile descriptor (d_ttab, one u64 per tile): bits [0, 36) first slot of the tile, [36, 45)
// slots of its rows (rows * g; 0: heavy tile, loads nothing), [45, 57) KRange index
static constexpr int kTtabRemShift = 36, kTtabRangeShift = 45;
// Consecutive tiles a superstep-0 wave takes at a time (tile t goes to wave (t / kTileBlock) % W): the
// tiles of a block share their range, whose fields then hit in the scalar cache
#ifndef PM_TILE_BLOCK
#define PM_TILE_BLOCK 4
#endif
static constexpr uint32_t kTileBlock = PM_TILE_BLOCK;
// Light rows fit in one tile with room for the 16-B alignment shift of its
// loads (a light tile holds at most kTileEntries - 4 slots).
static constexpr uint32_t kLightMax = 480;
static constexpr int kHeavyKind = 47;              // light kinds 0..46 (light_kind), heavy above
static constexpr int kMaxRanges = 16 * (kHeavyKind + 1) + 1;
// Active-edge map entries: neighbour position | kAlive | kFlag (cycle mark,
// nem_1.hpp:764-770).  Positions use 30 bits (V < 2^30).
static constexpr uint32_t kAlive = 1u << 31;
static constexpr uint32_t kFlag = 1u << 30;
static constexpr uint32_t kPosMask = kFlag - 1;

// Light degree classes (degree 1..kLightMax): the padded row length G of a
// class is the degree itself up to 16, then rounded up to a multiple of 4 (to
// 64), of 8 (to 128) and of 32 (to 480): at most a few percent of padding on
// R-MAT degree mixes (power-of-two classes padded ~24 %).
__host__ __device__ inline uint32_t light_kind(uint64_t d) {  // 1 <= d <= kLightMax
  if (d <= 16) return static_cast<uint32_t>(d - 1);
  if (d <= 64) return 16 + static_cast<uint32_t>(d - 17) / 4;
  if (d <= 128) return 28 + static_cast<uint32_t>(d - 65) / 8;
  return 36 + static_cast<uint32_t>(d - 129) / 32;
}
__host__ __device__ inline uint32_t kind_slots(uint32_t k) {
  if (k < 16) return k + 1;
  if (k < 28) return 20 + 4 * (k - 16);
  if (k < 36) return 72 + 8 * (k - 28);
  return 160 + 32 * (k - 36);
}

// 2-bit code of a vertex's T_pub for the gathers of the next superstep: the
// label's template bits t0 < t1 (bit 0: T has t0, bit 1: T has t1); a label
// with more than two template vertices codes any non-empty T as 3 (gather
// T_pub).  0 <=> T_pub = 0.
__host__ __device__ inline uint32_t tpub_code(uint32_t T, uint32_t tu) {
  const uint32_t rest = tu & (tu - 1);
  if (rest & (rest - 1)) return T ? 3u : 0u;
  return ((T & tu & (0u - tu)) ? 1u : 0u) | ((T & rest) ? 2u : 0u);
}

// A label on more than two template vertices: its code 3 means "read T_pub" (the position-indexed T_pub is
// written); with one or two template vertices code 3 is just both bits, and T_pub lives in the code.
__host__ __device__ inline bool tpub_wide(uint32_t tu) {
  const uint32_t rest = tu & (tu - 1);
  return (rest & (rest - 1)) != 0;
}

// The 2-bit T_pub codes are indexed by position inside the pattern's label runs (the runs packed one after
// the other): only such positions are ever coded (members of S) or gathered (M entries), and at S=28 the
// array is 22 MB instead of 64 MB for the first later superstep's 31 M random gathers.
__host__ __device__ inline uint32_t code_index(uint32_t p, const LabelRuns& lr) {
  uint32_t c = 0xFFFFFFFFu;
  for (int l = 0; l < lr.n; ++l)
    if (p - lr.lo[l] < lr.len[l]) c = p + lr.cd[l];
  return c;
}
__host__ __device__ inline uint64_t tcode_words(const LabelRuns& lr) { return (uint64_t(lr.ncode) + 15) / 16 + 1; }

// Padded row length: the class length up to kLightMax, the degree above.
__host__ __device__ inline uint64_t padded_degree(uint64_t d) {
  if (d == 0 || d > kLightMax) return d;
  return kind_slots(light_kind(d));
}

// Outputs of one fused NLC-line kernel (pm_lines.hip), device resident.
struct LineStats {
  unsigned long long nsrc, trav, tokens, acked, deleted, walks, ftotal;
  unsigned long long wn[20];    // TDS walks per position (1..C+1)
  unsigned long long wbase[20]; // TDS: slot offset of each position's walks
  unsigned int overflow, single;  // single: finished by block 0 alone
  unsigned int split, pad_;       // split: run over this shard's own sources only, post-processing deferred
  // a line started on block 0 alone whose frontier outgrew the block: the grid continues from position esc_k
  // (its walks / frontier from esc_base on)
  unsigned int esc_k, pad2_;
  unsigned long long esc_base;
  unsigned long long lp[20];  // long-row pieces appended at each position (pm_lines.hip, kLineLong)
  unsigned long long tstamp[4];  // s_memrealtime (100 MHz) at line start, after P1, after post, line end
  unsigned long long removed[2 * 64];  // vertices | edges per rank leaving S in post-processing
  unsigned long long census;  // sources the line would select on the state at the launch's start (k_lines)
  unsigned long long census_tok;  // their first-position tokens (sum of |M[s]|): the line's work estimate
  unsigned long long ptime[20];  // s_memrealtime at the end of each position's phase (diagnostics, PM_PHASE_TIMES)
  unsigned long long pmid[20][3];  // TDS position, thread 0: its first walks' state loaded, its expansion done, its wave's entries
};

// One NLC line as seen by the fused line kernel (pm_lines.hip).
struct LineDesc {
  LineArgs la;
  int32_t tds;  // pl >= 4: tds_batch_1 (beta.cpp:762-767)
  int32_t i0;   // pattern_indices[0] (post-processing bit)
  int32_t il;   // interleave_lp
  int32_t pad;
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t rstream = nullptr;    // read-backs that overlap the next kernels of `stream` (created on first use)
  hipEvent_t ev_rb = nullptr;       // ... ordered after this event of `stream`
  // one context: the 2-bit codes are cleared on rstream right after the first later superstep read them (beside the
  // rest of the search) instead of in the next search's fills; the next superstep-0 launch waits for ev_tz
  hipEvent_t ev_tz0 = nullptr, ev_tz = nullptr;
  bool tcode_zeroed = false;   // the codes are clear (or being cleared) for the current layout
  bool tcode_zpending = false; // ... by a clear on rstream that superstep 0 has not yet waited for
  uint64_t n = 0, nnz = 0;
  bool symmetric = true;
  uint32_t nranks = 1;
  uint64_t hub_threshold = 1048576;
  std::vector<uint64_t> hubs_host;
  Pattern pattern;
  PatArgs pa{};

  // graph (device), renumbered label-major whenever the labels change:
  // vertex positions ordered by (label, degree, id); every device array below
  // is indexed by position and the adjacency holds neighbour positions (each
  // row keeps the id order of the input, so duplicates stay adjacent).
  // Degrees by vertex id live on the host; the layout uploads what it needs to scratch (the device keeps no
  // id-major array but pos: 8 B per vertex less than resident offsets, per context -- in-process shards of
  // one S=28 search on one device need the room).
  std::vector<uint32_t> deg_host; // global (out-)degree by vertex id: labels, hubs, ss0 senders' entries
  std::vector<uint32_t> rdeg_host;// directed graphs: in-degree (length of the row superstep 0 scans)
  std::vector<uint32_t> ldeg_host;// sharded: length of this shard's row of each id (owned rows, delegate shares)
  uint32_t row_degree(uint64_t v) const { return rdeg_host.empty() ? deg_host[v] : rdeg_host[v]; }
  // the layout's sort key (row_degree: global degree, or in-degree of a directed graph) and the length of the
  // row this context holds
  const std::vector<uint32_t>& key_degrees() const { return rdeg_host.empty() ? deg_host : rdeg_host; }
  const std::vector<uint32_t>& held_degrees() const { return ldeg_host.empty() ? key_degrees() : ldeg_host; }
  uint64_t nq = 0;                // padded slots (label independent)
  uint64_t* d_offp = nullptr;     // label-major padded row starts, V+1
  uint64_t* d_offr = nullptr;     // label-major unpadded offsets (degree sums), V+1
  uint32_t* d_colp = nullptr;     // padded adjacency (neighbour positions, kNone pad), nq
  uint32_t* d_perm = nullptr;     // position -> vertex id
  uint32_t* d_pos = nullptr;      // vertex id -> position
  uint64_t* d_labs = nullptr;     // labels in position order (kept only when a line has selected vertices)
  std::vector<uint32_t> perm_host;
  LabelRuns lr{};
  uint64_t* d_hubs = nullptr;
  std::vector<uint64_t> labels_host;  // labels by vertex id (layout input, result files)

  // superstep-0 tiling for the current labels and pattern
  std::vector<KRange> ktab;
  KRange* d_ktab = nullptr;
  uint64_t* d_ttab = nullptr;     // superstep-0 tile descriptors (kTtab*Shift)
  uint32_t ntiles = 0;
  bool k1_wide = false;           // some range has more than four relevant label runs
  HSeg* d_hseg = nullptr;
  uint32_t nheavy = 0;            // heavy rows (scratch slots)
  uint32_t nhseg = 0;             // heavy segments (one superstep-0 tile each)
  uint32_t* d_hscr = nullptr;     // 3 x nheavy: TN, distinct count, segments done
  uint64_t ss0_trav = 0;          // adjacency entries of label-matching rows
  uint64_t ss0_rows = 0;          // label-matching rows with degree > 0
  uint64_t ss0_trav_all = 0;      // ss0_trav summed over the shards

  // sharding: shard `shard` of `nshards` owns the rows of
  // ids v % nshards == shard (delegate rows: the entries whose target it owns)
  // and runs superstep 0 and the first later superstep of the first LCC call
  // over them; in between, the survivors' 2-bit T_pub codes are all-gathered
  // (shard_codes_after_first).  After that superstep the state of S (T_pub,
  // T_state, M rows) is all-gathered into a replica held by every shard
  // (shard_replicate): the rest of the search -- later supersteps, NLC lines,
  // later LCC calls -- runs on the replica exactly as on one GPU.
  uint32_t nshards = 1, shard = 0;
  uint64_t held_rows = 0;         // nonempty rows this context holds (a shard: owned rows + delegate shares)
  uint64_t held_hub_entries = 0;  // entries of the delegate shares it holds
  hipEvent_t ev_handoff = nullptr;  // sharded: recorded when the state became the replica (sharded_ms)
  float sharded_ms = 0.f;         // device time of the last search's sharded part (search start -> replica)
  double comm_wall0 = 0.0, comm_wall_handoff = 0.0;  // Comm::wall at the search start / at the hand-off
  uint64_t replica_rows = 0, replica_entries = 0;
  Comm* comm = nullptr;
  Comm* comm_owned = nullptr;     // deleted with the context
  uint64_t mcap = 0;              // capacity (entries) of d_colp and d_mcol (nq; + kTileEntries tail padding)
  bool replicated = false;        // the search state is the replica (sharded, after shard_replicate)
  // the later superstep of the first LCC call after which the state is replicated (sharded; PM_HANDOFF, default
  // 2: at S=28 the second superstep still has 0.8 M rows, the third 26 k); capped at diameter - 1
  uint32_t handoff_ss = 2;
  // delegates of a sharded search (hubs_host order; the shares are rows of this shard's layout)
  bool split_hubs = false;        // nshards > 1 and some vertex has degree >= hub_threshold
  uint64_t hub_area = 0;          // entries behind the dense region: M rows of the hubs this shard controls
  HubInfo* d_hubinfo = nullptr;
  std::vector<HubInfo> hubinfo;
  uint64_t* d_moff = nullptr;     // M row starts before the replica: offp with the controlled hubs in the hub area
  uint64_t* d_hubpart = nullptr;  // (count << 32 | TN) of this shard's shares, then G x H gathered
  uint64_t* d_rmoff = nullptr;    // replica: M row start per position (V)
  uint32_t* d_rmcol = nullptr;    // replica: M rows, packed
  uint64_t rmcap = 0;             // entries of d_rmcol
  bool xcode_wide = false;        // some label has more than two template vertices: the exchange carries T_pub
  bool xcode_in_tpub = false;     // ... and it landed in T_pub (no superstep-0 records): cleared after superstep 1
  void* d_xsend = nullptr;        // exchange buffers (grown on demand)
  void* d_xrecv = nullptr;
  void* d_xent_send = nullptr;
  void* d_xent_recv = nullptr;
  size_t xsend_cap = 0, xrecv_cap = 0, xent_send_cap = 0, xent_recv_cap = 0;
  uint64_t* d_xcnt = nullptr;     // per-shard counts of the exchanges (device, 4 x 64 words)
  std::vector<uint64_t> xcode_n;  // records per shard of the last code exchange (u64-mode clear after superstep 1)
  uint64_t xcode_max = 0;
  uint64_t* d_xred = nullptr;     // host-vector all-reduce staging
  size_t xred_cap = 0;

  // host side of the driver loop
  uint64_t* h_pin = nullptr;      // pinned staging for counter read-backs
  size_t h_pin_words = 0;
  uint64_t* h_pin_lines = nullptr;  // pinned staging for the fused lines' read-back
  size_t h_pin_lines_words = 0;
  bool prelaunch_lines = false;   // lcc_call enqueues the lines before it waits (run_beta, iteration 0)
  bool lines_prelaunched = false;
  size_t pre_pl0 = 0, pre_nl = 0; // the prelaunched batch
  uint32_t* pre_kept = nullptr;
  bool fine_timing = false;       // per-superstep events (result files / PM_PHASE_TIMES)
  bool tpub_clean = false;        // T_pub is zero outside the last search's slist entries
  // PM_PHASE_TIMES: host timestamps of the driver loop (diagnostics)
  bool probing = false;
  std::vector<std::pair<const char*, double>> probes;
  void probe(const char* what) {
    if (probing)
      probes.emplace_back(what, std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count());
  }

  // vertex state (device, by position)
  uint16_t* d_tpub[2] = {nullptr, nullptr};  // template_vertices (T_pub), 0 = not in S
  int cur = 0;
  uint16_t* d_tst = nullptr;      // vertex_state.template_vertices (T_state)
  uint32_t* d_mcol = nullptr;     // active-edge rows (neighbour positions) at the vertex's row start, nq
  uint32_t* d_mlen = nullptr;     // entries written in the row (alive or dead)
  uint32_t* d_malive = nullptr;   // |M[v]|
  uint32_t* d_slist = nullptr;    // S members after superstep 0 (superset of S later), positions
  uint32_t* d_nS = nullptr;       // device count of d_slist
  // slist compaction (one shard): the live entries of a superstep's mask move
  // to d_slist2 / d_nS2, then the pointers swap; per-chunk counts and bases
  uint32_t* d_slist2 = nullptr;
  uint32_t* d_nS2 = nullptr;
  uint32_t* d_ccnt = nullptr;
  uint32_t* d_cbase = nullptr;
  void* d_ctmp = nullptr;
  size_t ctmp_bytes = 0;
  uint64_t ccap = 0;              // chunk capacity of d_ccnt / d_cbase
  // list compaction (k_compact_scan): tile status words, their capacity, the launch epoch, the co-resident grid
  void* d_clstat = nullptr;
  uint64_t clstat_cap = 0, cl_epoch = 0;
  unsigned cl_grid = 0;
  bool slist_compacted = false;   // d_slist holds S only (shorter than the host bound nS_host)
  // live mask of slist per 64 entries, written by every later superstep
  // (members of S plus vertices removed in that superstep): later passes
  // skip dead chunks without touching them
  uint64_t* d_smask[2] = {nullptr, nullptr};
  uint64_t* d_kmask = nullptr;  // survivors per 64-entry chunk of the last pull superstep (the compaction's keep)
  int smask_cur = 0;
  bool smask_valid = false;       // false right after superstep 0 (all entries live)
  uint32_t* d_flags = nullptr;    // [0] not_finished, [1] asymmetric edge state, [2] deleted
  uint32_t* d_tn = nullptr;       // TN per position for the push-form supersteps (allocated on first use)
  unsigned long long* d_push = nullptr;  // push form: [send pieces, verify's first piece, pieces...]
  uint64_t push_cap = 0;
  uint64_t* d_counts = nullptr;   // per-slot per-rank counts (vertices, edges) + traversed
  uint64_t* d_part = nullptr;     // per-block counter partials (kPartGridMax x slot_words)
  uint64_t* d_tmask = nullptr;    // superstep-0 survivor masks, kSub words per tile
  uint64_t* d_tbase = nullptr;    // exclusive scan of the per-tile survivor counts
  uint32_t* d_tcode = nullptr;   // superstep-0 T_pub in 2 bits per position (k_lcc_first -> first later superstep)
  // dense superstep-0 output (symmetric graph, diameter >= 2): light tiles append
  // their contributors to their wave's slice of the region [dbase, dbase + dcap)
  // of d_mcol, and their survivors' 16-B records {position, T_pub | |M| << 16,
  // first entry (kNone: M in the padded row, state in its arrays), 0} to the
  // wave's slice of d_rarea (bounded by the rows of the wave's tiles, d_rbase);
  // heavy rows to d_hrec.  The slist and the slist-aligned records d_srec are
  // built from them; the first later superstep reads d_srec and M densely and
  // writes the rows of its survivors into their padded rows.  Nothing is stored
  // by position except the 2-bit codes (and T_pub of labels of more than two
  // template vertices).
  uint64_t dbase = 0, dcap = 0;
  uint4* d_rarea = nullptr;       // record slices of the superstep-0 waves
  uint64_t* d_rbase = nullptr;    // first record of each wave's slice (k1_grid * kWpb + 1)
  uint32_t* d_rcnt = nullptr;     // records each wave wrote
  uint64_t* d_rofs = nullptr;     // exclusive scan of d_rcnt
  uint4* d_hrec = nullptr;        // heavy rows' records (w = 1: survivor)
  uint4* d_srec = nullptr;        // records in slist order (the first later superstep)
  uint4* d_cdesc = nullptr;       // one context: where each 64-record chunk lies (records read in place, k_chunk_slices)
  bool records_in_place = false;
  bool removed_cleared = false;   // the last pull superstep cleared its removed rows' T_pub (records mode)  // the first later superstep reads the records from the superstep-0 slices
  uint64_t rarea_cap = 0, srec_cap = 0;
  uint32_t rwaves = 0;            // waves of the superstep-0 grid the slices were sized for
  void* d_rscan_tmp = nullptr;
  size_t rscan_tmp_bytes = 0;
  bool k1_records = false;        // the last superstep-0 launch wrote records (and no tile masks)
  bool k1_dense = false;         // the last superstep-0 launch wrote dense M
  uint32_t diag_step = 0;        // diagnostics only (PM_DIAG_STEP): k_lcc_step timing variants
  // the last first LCC call's mean |M| of each superstep's survivors (k_lcc_step's entries in flight for the
  // next superstep's rows), and the superstep being launched
  std::vector<double> m_per_row;
  uint64_t cur_ss = 0;
  // pull-form rows above kPullLong entries, worked in pieces by a second launch (k_lcc_step_pieces): the list,
  // and per superstep of the first call whether the previous search deferred any there (empty: not known --
  // every pull superstep gets the pieces launch; a superstep with none skips it from then on)
  void* d_lrows = nullptr;
  uint32_t lrows_cap = 0;
  void* d_lscr = nullptr;          // the last pull superstep's packing scratch (k_long_pack): pieces + counts
  uint64_t lscr_pieces = 0;
  std::vector<uint8_t> long_seen;
  bool long_seen_off = false;  // PM_PULL_PIECES=0 (diagnostics): long rows walked by one wave, as before
  uint32_t pull_long = 0;      // PM_PULL_LONG (tests): list rows above this many entries (0: kPullLong)
  uint32_t* d_tcnt = nullptr;     // superstep-0 survivors per tile
  uint32_t* d_tstart = nullptr;   // position of a tile's row 0 (heavy tile: its row)
  void* d_scan_tmp = nullptr;     // rocPRIM scan workspace for the slist build
  size_t scan_tmp_bytes = 0;
  uint64_t tmask_words = 0;
  uint64_t last_acked = 0;
  unsigned k1_grid = 0;
  uint8_t* d_tsm = nullptr;       // token source map: 0 none, 1 unacked source, 2 acked
  size_t counts_slots = 0;

  Arena arena;
  // zero fills and the T_pub clear of a search's start, batched into one launch (flush_zero)
  struct ZeroRange {
    void* p;
    uint64_t bytes;
  };
  ZeroRange zq[8];
  int nzq = 0;
  bool clear_pending = false;      // T_pub at the slist entries, then d_nS (flush_zero)
  uint32_t clear_cap = 0;          // host bound of the slist the pending clear walks (saved at reset: nS_host is
                                   // zeroed before the deferred flush)
  bool k1_fills_queued = false;    // queue_lcc_first_fills ran for the next superstep-0 launch
  uint32_t* d_zticket = nullptr;   // last-block ticket of k_zero_batch (zero between launches)
  std::vector<hipEvent_t> events;  // LCC call timing, created once
  uint32_t nS_host = 0;     // size of d_slist (host copy, valid after superstep 0)
  bool lcc_started = false; // superstep 0 of the first call done

  // fused NLC lines (pm_lines.hip)
  LineStats* d_lstats = nullptr;  // per line
  LineDesc* d_ldesc = nullptr;
  size_t d_lstats_n = 0;
  unsigned long long* d_hkey = nullptr;  // (source, vertex) hash table, persistent
  unsigned long long* d_hval = nullptr;
  uint64_t hcap = 0;
  bool hash_regrown = false;      // the last fused launch overflowed the table and grew it (rerun the line fused)
  uint64_t hash_slots = 0;        // PM_HASH_SLOTS (diagnostics): size of the context's first table (0: from |S|)
  int64_t nogrow_shard = -1;      // PM_DEBUG_NOGROW_SHARD (diagnostics): that shard reports no room to grow it
  // local split lines (one context): the part the next line launch runs (parts > 1), the parts' sources and the
  // post-processing's cleared-source list
  uint32_t lsplit_parts = 0, lsplit_part = 0;
  uint32_t* d_lsrc = nullptr;
  unsigned long long* d_ldels = nullptr;
  uint64_t lsrc_cap = 0, ldels_cap = 0;
  uint32_t local_split_parts = 0;  // parts of the last local split line (diagnostics)
  int64_t overflow_shard = -1;    // PM_DEBUG_OVERFLOW_SHARD (diagnostics): that shard alone reports its first
                                  // replicated path line of a search as overflowed (the agreement's test)
  bool no_row_compaction = false; // PM_ROW_COMPACTION=0 (diagnostics): rows keep their dead entries
  uint32_t lcc_calls = 0;  // stamp of the LCC calls (the compaction's long-row word)
  bool push_long = true;   // some row of S may be longer than a push-form piece (unknown: true)
  uint32_t* d_front = nullptr;    // slots inserted by a fused path line (cleared by it)
  unsigned* d_gbar = nullptr;     // grid barrier state of the fused line kernels
  bool lines_ctl_clean = false;   // the line launches' control words are zero (the search's fills cleared them)
  unsigned line_grid = 0;         // blocks of a full-chip line launch (one per CU)
  uint64_t live_hint = ~0ull;     // S members on this context after the last LCC call (line grid size)
  bool fused_lines = true;        // PM_FUSED_LINES=0 forces the exact-count path
  bool any_sv = false;            // some line has selected_vertices (token-source sets span lines)
  bool coop = false;              // grid-barrier kernels by cooperative launch (several contexts on the device)
  // sharded search on the replica: an NLC line whose work census (first-position tokens of its sources on the
  // replica, sum of |M[s]|) reaches split_min runs split by owner -- every shard passes the tokens of the
  // sources it owns (hub ordinal % nshards, else id % nshards) -- and the shards then exchange the line's
  // effects (pm_shard.hip split_line_finish); smaller lines run replicated (every shard all sources, no
  // exchange: a split costs a launch and 2-4 all-gathers).  0: never split.  PM_SPLIT_LINES.
  uint64_t split_min = 32768;
  unsigned long long* d_xsplit = nullptr;  // a split line's flagged M entries (replica entry indices), then
  uint64_t xsplit_cap = 0;                 // the shard's cleared sources (positions) of its post-processing
  bool force_pull = false;        // PM_FORCE_PULL=1 (diagnostics): pull-form LCC in every call

  // token-source sets (vertex_token_source_set, nem_1.hpp:131-139, 270-285) of
  // the last path line as sorted (source << 32 | vertex) keys: a
  // selected-vertices line starts from the entries of active vertices with its
  // last label (beta.cpp:823-850); every other line starts empty
  unsigned long long* d_pseen = nullptr;
  uint64_t npseen = 0, pseen_cap = 0;

  // last token-passing call (selected-vertices lines: the vertices verified)
  uint32_t* d_sources = nullptr;
  uint64_t nsources = 0;
  std::vector<std::vector<std::string>> walk_lines;  // per rank, last TDS line
  uint64_t last_walks = 0;
  uint64_t last_tds_chunks = 0;   // chunk launches of the last exact-path TDS line (unbatched: one per level)

  // timing of the fused superstep-0 kernel (for the roofline report)
  float lcc_first_ms = 0.f;
  uint64_t lcc_first_bytes = 0;
  double device_seconds = 0.0;
  double lines_seconds = 0.0;     // NLC lines of the current search (pm_run_stats::nlcc_seconds)
  double layout_seconds = 0.0;    // last label-major layout + tiling build (one-time setup)

  std::string err;
};

// The M rows of the search state: the padded rows of the context's own layout,
// or the replica's packed rows (sharded, after shard_replicate).
inline const uint64_t* m_off(const Ctx& c) { return c.replicated ? c.d_rmoff : c.d_moff ? c.d_moff : c.d_offp; }
inline uint32_t* m_col(const Ctx& c) { return c.replicated ? c.d_rmcol : c.d_mcol; }
inline uint64_t m_cap(const Ctx& c) { return c.replicated ? c.rmcap : c.mcap; }

// Kernel launchers (pm_kernels.hip).
// Label-major layout: sorts the vertices by (label, degree, id) and writes the
// renumbered adjacency into dst (E entries).  src_col holds the id-major input
// (each held row at the prefix sum of held_degrees()), or, when relabelling, is
// the current d_colp (neighbour positions, translated in place first).  Its
// scratch (~64 B per vertex) is allocated for the call and freed after it.
void build_label_layout(Ctx& c, uint32_t* src_col, bool src_is_layout, uint32_t* dst);
void build_tiling(Ctx& c);
// Counter slots: W = slot_words(c) u64 = [vertices per rank | edges per rank |
// traversed | matching rows | removed flag | asymmetry flag | pull-form long rows deferred | their pieces].
uint32_t slot_words(const Ctx& c);
// ev0/ev1 (may be null) bracket the kernel launch alone (roofline timing)
void launch_lcc_first(Ctx& c, uint64_t* d_slot, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
void lcc_first_prepare(Ctx& c);  // zeroes the heavy-row scratch before a launch
void lcc_first_set_dense(Ctx& c);  // dense superstep-0 M for this launch (sets k1_dense)
void launch_lcc_first_kernel(Ctx& c, int variant, unsigned grid, uint64_t* d_slot);  // variant != 0: diagnostics
unsigned lcc_first_grid(const Ctx& c);
// first_after_ss0: the superstep right after superstep 0 of the first call
// (T_pub is still superstep 0's output: neighbours' T_pub from the 2-bit codes)
// pub_state: the first LCC call (T_state == T_pub for every member of S; its alive count is counted, not loaded)
void launch_lcc_step(Ctx& c, uint64_t* d_slot, bool first_after_ss0 = false, bool last_of_call = false,
                     bool pub_state = false);
void ensure_slist2(Ctx& c);
// Push form of a later superstep (send + verify launches): directed inputs and
// LCC calls after the first (M may be asymmetric there).
void launch_lcc_push(Ctx& c, uint64_t* d_slot);
void launch_compact_rows(Ctx& c, uint32_t stamp);
void launch_count_state(Ctx& c, uint64_t* d_slot);
void launch_compact_slist(Ctx& c);  // keeps the live entries of the last superstep's mask
// Zero T_pub (both buffers) at the slist entries of the last search (every
// nonzero T_pub entry is one of them, plus the other shards' when sharded).
void launch_clear_tpub(Ctx& c);
// Deferred zero fill of `bytes` (a multiple of 4, 4-aligned) at p: the queued fills, and a pending T_pub clear
// (clear_pending: T_pub at the slist entries, then d_nS = 0), go out as ONE launch in flush_zero -- each
// hipMemsetAsync is a dispatch of its own, several microseconds apart on the stream.
void zero_later(Ctx& c, void* p, uint64_t bytes);
void queue_lcc_first_fills(Ctx& c);
void flush_zero(Ctx& c);
// Waits for the stream by polling it (hipStreamQuery): the driver loop's read-back waits, so the host follows
// the device at once instead of sleeping until the runtime wakes it (PM_SPIN=0: hipStreamSynchronize).
void stream_wait(hipStream_t s);
size_t slist_scan_tmp_bytes(uint64_t words);
static constexpr unsigned kPartGridMax = 2048;

struct TpResult {
  uint64_t sources = 0, acked = 0, edges = 0, tokens = 0, walks = 0;
  uint64_t batches = 0, batch_retries = 0;  // exact path lines: initiator batches run, and those that did not fit
};
TpResult run_path_line(Ctx& c, const NlcLine& line);
// Output of one line of the fused kernel (token passing + post-processing).
// rm_v / rm_e are the vertices / edges per rank that left S in
// post-processing (the active counts after the line are the counts before it
// minus these: token passing itself changes neither T_pub nor |M|).  A line
// that overflowed a capacity had no terminal or post effect (c.nsources names
// its marked sources) and is rerun through run_path_line / run_tds_line,
// launch_post_tp and count_state.
struct FusedLineOut {
  TpResult tr;
  uint32_t deleted = 0;
  bool split = false;           // ran split over the shards (stats, effects and walks combined over them)
  std::vector<uint64_t> rm_v, rm_e;
  std::vector<uint32_t> walks;  // kept TDS walks (positions), when requested
  uint32_t stride = 0;
};
// Lines pl0.. in one launch; returns how many completed (their outputs in
// outs).  It stops after a line that deleted with interleave_lp set, or before
// a line that overflowed (overflow = true: rerun that line on the exact-count
// path).
// max_lines bounds the lines of one launch.  One shard only (sharded searches
// run the per-position path with token exchange).
size_t run_lines_fused(Ctx& c, size_t pl0, bool want_walks, std::vector<FusedLineOut>& outs, bool& overflow,
                       size_t max_lines = SIZE_MAX);
// Enqueues the fused launch of lines [0, all) behind the work already on the stream
// (the first LCC call of a search, whose lines always run: beta.cpp:686-688); the
// next run_lines_fused(c, 0, ...) then only waits for it and reads its results.
void prelaunch_lines_fused(Ctx& c);
void queue_lines_ctl_clear(Ctx& c);
void side_clear_codes(Ctx& c);
void free_line_buffers(Ctx& c);
TpResult run_tds_line(Ctx& c, const NlcLine& line, std::vector<uint32_t>& walks_out, uint32_t& stride);
// The same with the kept walks handed to `sink` chunk by chunk (positions, stride C+2 each) instead of
// collected: the exact path's enumeration is depth-first over chunks of at most tds_walk_cap walks.
using TdsSink = std::function<void(const uint32_t* walks, uint64_t n)>;
TpResult run_tds_line(Ctx& c, const NlcLine& line, uint32_t& stride, const TdsSink& sink);
uint64_t tds_walk_cap(const Ctx& c, int stride);  // walks per level chunk (arena room; PM_TDS_CAP caps it)
uint32_t launch_post_tp(Ctx& c, const NlcLine& line);

LineArgs make_line_args(const Ctx& c, const NlcLine& line);

uint64_t* pinned(Ctx& c, size_t words);  // pinned host staging (pm_api.hip)
// PM_DEBUG_SYNC=1 (diagnostics): the stream is synchronised at each named point and a device fault is reported
// with the point's name and the shard (=2: every point passed is also printed); no-op otherwise.
void debug_point(Ctx& c, const char* where);

// Shard exchanges (pm_shard.hip); no-ops without a communicator.
// After a split NLC line (its tokens passed for this shard's own sources, terminal effects local): agrees on
// overflow over the shards (false: every shard reruns the line on the exact, replicated path), else runs this
// shard's post-processing, exchanges the cleared sources and the flagged M entries (every replica applies
// all of them), sums the stats, and gathers the kept walks (want_walks).  kept: this shard's kept walk slots.
bool split_line_finish(Ctx& c, size_t pl, const LineStats& st, const uint32_t* kept_dev, bool want_walks,
                       FusedLineOut& out);
// One context, a line whose (source, vertex) pairs outgrew the largest table: the fused kernel over the line's
// sources in parts (the owner rule with `parts` parts), the post-processing once after every part.  false: some
// part still overflowed at the finest split tried (the caller takes the exact path).
bool local_split_line(Ctx& c, size_t pl, bool want_walks, FusedLineOut& out);
// One part of such a line (pm_lines.hip): its statistics; on overflow the table is cleared.
LineStats run_line_part(Ctx& c, size_t pl, uint32_t parts, uint32_t part, uint32_t*& kept_dev);
// after superstep 0 (sharded, delegates): the shares' TN / counts all-gathered and OR-ed / summed, the
// shares' M entries sent to the controller (all-to-all), the controller verifies (slot: ss0 counters)
void shard_hub_combine(Ctx& c, uint64_t* d_slot);
void shard_codes_after_first(Ctx& c);  // after superstep 0: every shard's survivors' T_pub codes
void shard_replicate(Ctx& c);          // the state of S of every shard -> the replica (collective)
// after the first later superstep when the replica is built after the second: every shard's S rows' T_pub
void shard_tpub_exchange(Ctx& c);
std::vector<uint64_t> shard_allreduce(Ctx& c, const std::vector<uint64_t>& v);  // host vector, sum
// The minimum of v over the shards (v itself without a communicator): capacities that steer the replicated
// part of a sharded search (arena, line hash table) must be the same on every shard, or an overflow -- and the
// collectives of the path it takes -- could happen on some shards only.
uint64_t shard_agree_min(Ctx& c, uint64_t v);
std::vector<uint64_t> shard_gather_u64(Ctx& c, uint64_t v);  // every shard's v (collective)
// S rows of the current state (slist entries with T_pub != 0) packed on the device: per row
// {position, T_pub | T_state << 16, |M|, first entry} (4 u32) and its alive M entries; counts[0..1] =
// rows, entries (device).  rec / ent hold nS_host rows / the caller's entry bound.
void pack_state(Ctx& c, uint32_t* rec, uint32_t* ent, uint64_t ent_cap, uint64_t* counts);
uint64_t pack_state_entry_bound(Ctx& c);  // entries of the rows pack_state may write (host sync)

}  // namespace pm
