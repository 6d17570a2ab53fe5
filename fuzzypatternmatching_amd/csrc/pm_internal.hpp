// Internal declarations shared by the HIP kernels (pm_kernels.hip) and the
// host driver / C-ABI (pm_api.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
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
struct OwnerArgs {
  const uint64_t* hubs;  // sorted hub ids (device), may be null
  uint32_t nhubs;
  uint32_t nranks;
};

// NLC line constants for the token-passing kernels.
struct LineArgs {
  uint16_t I[16];       // template index per walk position
  uint16_t E[16];       // enumeration index per position (TDS)
  uint8_t lok[16];      // L[k] == plabel[I[k]] (label test folded)
  int32_t C;            // cycle length: walk positions 0..C+1
  int32_t VC;           // valid cycle (expect target vertex)
  uint16_t ilast;       // pattern_indices.back()
  uint16_t pad;
};

// Device scratch arena (bump allocator, reset per NLC line).
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  void* get(size_t bytes) {
    size_t a = (used + 255) & ~size_t(255);
    if (a + bytes > cap) throw std::runtime_error("device scratch arena exhausted");
    used = a + bytes;
    return base + a;
  }
  void reset() { used = 0; }
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t n = 0, nnz = 0;
  bool symmetric = true;
  uint32_t nranks = 1;
  uint64_t hub_threshold = 1048576;
  std::vector<uint64_t> hubs_host;
  Pattern pattern;
  PatArgs pa{};

  // graph (device)
  uint64_t* d_off = nullptr;
  uint32_t* d_col = nullptr;
  uint64_t* d_labels = nullptr;
  uint64_t* d_hubs = nullptr;
  std::vector<uint64_t> labels_host;  // for result files

  // vertex state (device)
  uint16_t* d_tl = nullptr;       // template bits matching the vertex label
  uint64_t* d_tlbits = nullptr;   // 1 bit per vertex: tl != 0
  uint16_t* d_tpub[2] = {nullptr, nullptr};  // template_vertices (T_pub), 0 = not in S
  int cur = 0;
  uint16_t* d_tst = nullptr;      // vertex_state.template_vertices (T_state)
  uint32_t* d_mcol = nullptr;     // active-edge rows, stored at the vertex's CSR offset
  uint8_t* d_mst = nullptr;       // per entry: bit0 alive, bit1 flag (cycle mark)
  uint32_t* d_mlen = nullptr;     // entries written in the row (alive or dead)
  uint32_t* d_malive = nullptr;   // |M[v]|
  uint32_t* d_slist = nullptr;    // S members after superstep 0 (superset of S later)
  uint32_t* d_nS = nullptr;       // device count of d_slist
  uint32_t* d_flags = nullptr;    // [0] not_finished, [1] asymmetric edge state, [2] deleted
  uint64_t* d_counts = nullptr;   // per-slot per-rank counts (vertices, edges) + traversed
  uint64_t* d_part = nullptr;     // per-block counter partials (kMaxGrid x slot_words)
  uint64_t* d_cmask = nullptr;    // superstep-0 survivor mask per 64-vertex chunk
  uint64_t* d_cbase = nullptr;    // exclusive scan of the chunk popcounts
  void* d_scan_tmp = nullptr;     // hipcub scan workspace for the slist build
  size_t scan_tmp_bytes = 0;
  uint64_t last_acked = 0;
  unsigned k1_resident_blocks = 0;
  uint8_t* d_tsm = nullptr;       // token source map: 0 none, 1 unacked source, 2 acked
  size_t counts_slots = 0;

  Arena arena;
  uint32_t nS_host = 0;     // size of d_slist (host copy, valid after superstep 0)
  bool lcc_started = false; // superstep 0 of the first call done

  // last token-passing call
  uint32_t* d_sources = nullptr;
  uint64_t nsources = 0;
  std::vector<std::vector<std::string>> walk_lines;  // per rank, last TDS line
  uint64_t last_walks = 0;

  // timing of the fused superstep-0 kernel (for the roofline report)
  float lcc_first_ms = 0.f;
  uint64_t lcc_first_bytes = 0;
  double device_seconds = 0.0;

  std::string err;
};

// Kernel launchers (pm_kernels.hip).
void launch_degree_labels(Ctx& c);
void launch_label_match(Ctx& c);
// Counter slots: W = slot_words(c) u64 = [vertices per rank | edges per rank |
// traversed | matching rows | removed flag | asymmetry flag].
uint32_t slot_words(const Ctx& c);
void launch_lcc_first(Ctx& c, uint64_t* d_slot);
void launch_lcc_first_kernel(Ctx& c, int variant, unsigned grid);  // variant != 0: ablation builds
unsigned lcc_first_grid(const Ctx& c);
unsigned query_k1_resident_blocks(int device);
void launch_lcc_step(Ctx& c, uint64_t* d_slot);
void launch_count_state(Ctx& c, uint64_t* d_slot);
size_t slist_scan_tmp_bytes(uint64_t n);
static constexpr unsigned kPartGridMax = 2048;

struct TpResult {
  uint64_t sources = 0, acked = 0, edges = 0, tokens = 0, walks = 0;
};
TpResult run_path_line(Ctx& c, const NlcLine& line);
TpResult run_tds_line(Ctx& c, const NlcLine& line, std::vector<uint32_t>& walks_out, uint32_t& stride);
uint32_t launch_post_tp(Ctx& c, const NlcLine& line);

LineArgs make_line_args(const Ctx& c, const NlcLine& line);

}  // namespace pm
