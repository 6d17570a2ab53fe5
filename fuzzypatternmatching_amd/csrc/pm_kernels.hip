// HIP kernels (gfx950 / CDNA4) for the label-constrained pattern-matching path.
//
// Layout in HBM (see DESIGN.md "Data layout").  Vertices are renumbered
// label-major when the labels are loaded: position order = (label, degree,
// id), so every pattern label owns one contiguous run of positions and the
// template bits of a neighbour follow from its position alone (LabelRuns).
//   offp[V+1] u64, colp[E] u32    CSR by position; entries are neighbour
//                                 positions, each row in input (id) order so
//                                 duplicates stay adjacent
//   perm[V], pos[V] u32           position <-> vertex id (output, owner rule)
//   tpub[2][V] u16                template_vertices (T_pub), ping-pong per superstep;
//                                 0 <=> vertex not in the state map S
//   tst[V] u16                    vertex_state.template_vertices (T_state)
//   mcol[E] u32                   active-edge map M[v], stored in v's own CSR slot
//                                 [offp[v], offp[v]+mlen[v]) so no prefix scan is needed;
//                                 entry = neighbour position | kAlive | kFlag (edge flag)
//   mlen[V], malive[V] u32        written length / alive count of M[v]
//   slist[nS] u32                 positions that entered S in superstep 0 (S only shrinks)
//
// Superstep 0 (k_lcc_first) visits only the label-matching runs, tiled by
// degree class; later supersteps (k_lcc_step) are row-per-lane scheduled
// through "strips" over M.  Irregular integer work: no MFMA (north_star).

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "pm_device.hpp"
#include "pm_internal.hpp"

namespace pm {


// ---------------------------------------------------------------------------
// Label-major padded layout (built when the labels change, outside any search).
//
// Vertices are stably sorted by (label, degree); rows of degree <= kHeavyDeg
// get padded_degree() slots (kNone fill), so every (label, degree class) run
// is a dense rows x G array whose slot addresses follow from the tile index
// alone: superstep 0 needs no row-offset loads, one round trip per tile.
// (Degree labels, vertex_data_db_degree.hpp:109 label = bit_width(degree), are
// computed on the host: the device holds no id-major degree array.)
__global__ void k_layout_keys(const uint32_t* __restrict__ deg, uint64_t n, uint32_t* __restrict__ dkey,
                              uint32_t* __restrict__ ids) {
  for (uint64_t v = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; v < n; v += uint64_t(gridDim.x) * blockDim.x) {
    dkey[v] = deg[v];
    ids[v] = static_cast<uint32_t>(v);
  }
}

__global__ void k_gather_labels(const uint64_t* __restrict__ labels, const uint32_t* __restrict__ ids, uint64_t n,
                                uint64_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = labels[ids[i]];
}

// Degrees in position order: padded (pad) and real (real).
__global__ void k_perm_degrees(const uint32_t* __restrict__ deg, const uint32_t* __restrict__ perm, uint64_t n,
                               uint64_t* __restrict__ pad, uint64_t* __restrict__ real) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = perm[i];
    const uint64_t d = deg[u];
    pad[i] = padded_degree(d);
    real[i] = d;
  }
}

__global__ void k_inverse_perm(const uint32_t* __restrict__ perm, uint64_t n, uint32_t* __restrict__ pos) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    pos[perm[i]] = static_cast<uint32_t>(i);
}

// Relabel, step 1: row starts by vertex id of the current layout, and the
// adjacency translated back to ids in place (padding stays kNone).
__global__ void k_row_starts_by_id(const uint64_t* __restrict__ offp, const uint32_t* __restrict__ perm, uint64_t n,
                                   uint64_t* __restrict__ start) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    start[perm[i]] = offp[i];
}

__global__ void k_to_ids(uint32_t* __restrict__ col, uint64_t nq, const uint32_t* __restrict__ perm) {
  for (uint64_t e = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; e < nq; e += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t x = col[e];
    if (x != kNone) col[e] = perm[x];
  }
}

// One wave per destination row: slot j < degree gets pos[src[src_start[id] + j]],
// the padding kNone.
__global__ __launch_bounds__(kBlock) void k_copy_rows(const uint32_t* __restrict__ src,
                                                      const uint64_t* __restrict__ src_start,
                                                      const uint32_t* __restrict__ deg,
                                                      const uint64_t* __restrict__ offp,
                                                      const uint32_t* __restrict__ perm,
                                                      const uint32_t* __restrict__ pos, uint64_t n,
                                                      uint32_t* __restrict__ dst) {
  const int lane = lane_id();
  const uint64_t nw = uint64_t(gridDim.x) * kWpb;
  for (uint64_t i = blockIdx.x * uint64_t(kWpb) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave); i < n; i += nw) {
    const uint64_t d0 = offp[i], slots = offp[i + 1] - d0;
    const uint32_t u = perm[i];
    const uint64_t du = deg[u];
    const uint64_t s0 = src_start[u];
    for (uint64_t j = lane; j < slots; j += kWave) dst[d0 + j] = j < du ? pos[src[s0 + j]] : kNone;
  }
}

// ---------------------------------------------------------------------------
// K1: superstep 0 of the first LCC call fused with its global verify.
//
// Pull form of nonunique_ee.hpp:519-569 (senders), :368-406 + :647-816
// (receivers) and :841-866 + :886-977 (verify): for every vertex u whose label
// matches a template (Tl(u) != 0), scan its row (on a symmetric CSR the
// in-row equals the out-row with multiplicity); an entry v contributes iff
// Tl(v) != 0 and (Tl(v) & NbrMask(Tl(u))) != 0 (valid parent).  Then
//   TN(u) = OR of contributing Tl(v); u in S iff TN(u) != 0;
//   M[u]  = distinct contributing v (first occurrence in the sorted row);
//   T_state = keep_bits(Tl(u), TN); empty -> removed (sets not_finished).
// Survivors get T_pub = T_state, |M[u]| and a bit in the tile survivor mask.
//
// Only the label-matching runs of the padded label-major CSR are visited
// (KRange table, staged in LDS); Tl(v) follows from v's position (LabelRuns).
// A tile is kTileEntries consecutive slots: every lane issues kSub adjacency
// loads before any use (one memory round trip per tile).  G <= 64: a sub-tile
// holds 64/G rows, G lanes each; per-row OR and count come from wave ballots,
// M positions from a masked popcount.  G = 128..1024: sub-tiles are the
// consecutive 64-slot slices of G/64-slot rows, reduced in order.  Rows above
// kHeavyDeg are cut into kHeavyDeg segments (one per tile) whose M stays
// uncompacted (dead entries keep bit0 = 0); the last segment to finish
// (ticket counter) runs the verify.  Only neighbour-mask bits of TN are
// reduced: bits outside NbrMask(Tu) never affect keep_bits.
__device__ __forceinline__ uint16_t wave_or_bits(uint32_t x, uint16_t nm, int shift, uint64_t gmask) {
  uint16_t r = 0, b = nm;
  while (b) {
    const int t = __ffs(static_cast<int>(b)) - 1;
    b &= static_cast<uint16_t>(b - 1);
    const uint64_t bb = __ballot((x >> t) & 1u);
    if ((bb >> shift) & gmask) r |= static_cast<uint16_t>(1u << t);
  }
  return r;
}

struct K1Out {
  uint16_t* tst;
  uint16_t* tpub;
  uint32_t* mcol;
  uint32_t* mlen;
  uint32_t* malive;
  uint32_t* tcnt;    // per tile: survivors
  uint32_t* tstart;  // per tile: position of row 0 (light) or the heavy row
  uint32_t* tcode;   // T_pub in 2 bits per position (tpub_code), OR-ed in
  // dense M: survivor records {position, T_pub | |M| << 16, first entry in mcol[dbase..] (kNone: M in the
  // padded row, T_state / |M| / alive count in their arrays), 0}, appended to the wave's slice of rarea
  // (rbase[w] .. + its rows bound; count to rcnt[w]); heavy rows to hrec[h] (w = 1: survivor).  Null: no
  // dense M (tile masks, position-indexed state)
  uint4* rarea;
  const uint64_t* rbase;
  uint32_t* rcnt;
  uint4* hrec;
  uint64_t dbase;    // dense M: first entry of the region in mcol
  uint64_t dslice;   // dense M: entries of the region owned by each wave of the grid
};


// Template bits of neighbour position p that can meet the range's nm: four
// runs held in registers (wave-uniform), the rest (rare) scanned from LDS.
struct RelRuns {
  uint32_t lo[4], len[4], tu[4];
  uint32_t nrel;
  uint32_t alo[4], alen[4];  // merged runs (admission test)
  uint32_t nadm;
};

// The range table is read through the constant address space: every index
// into it is wave-uniform, so the fields arrive by scalar loads (SGPRs, no LDS
// copy, no readfirstlane).
typedef __attribute__((address_space(4))) const KRange* KTab;

__device__ __forceinline__ RelRuns load_rel(KTab R) {
  RelRuns x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x.lo[i] = __builtin_amdgcn_readfirstlane(R->rlo[i]);
    x.len[i] = __builtin_amdgcn_readfirstlane(R->rlen[i]);
    x.tu[i] = __builtin_amdgcn_readfirstlane(R->rtu[i]);
  }
  x.nrel = __builtin_amdgcn_readfirstlane(R->nrel);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x.alo[i] = __builtin_amdgcn_readfirstlane(R->alo[i]);
    x.alen[i] = __builtin_amdgcn_readfirstlane(R->alen[i]);
  }
  x.nadm = __builtin_amdgcn_readfirstlane(R->nadm);
  return x;
}

template <bool WIDE>
__device__ __forceinline__ uint16_t tbits_rel(uint32_t p, const RelRuns& x, const uint32_t* s_runs, int nruns) {
  uint32_t t = 0;
  if (WIDE) {  // more than four relevant runs somewhere: scan all runs (LDS)
    for (int l = 0; l < nruns; ++l)
      if (p - s_runs[3 * l] < s_runs[3 * l + 1]) t |= s_runs[3 * l + 2];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (p - x.lo[i] < x.len[i]) t |= x.tu[i];
  }
  return static_cast<uint16_t>(t);
}

// keep_bits(tu, TN) of a range from its precomputed needs (wave-uniform).
struct KeepArgs {
  uint32_t bit[4], need[4];
  uint32_t n;
};

__device__ __forceinline__ KeepArgs load_keep(KTab R) {
  KeepArgs k;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    k.bit[i] = __builtin_amdgcn_readfirstlane(R->kbit[i]);
    k.need[i] = __builtin_amdgcn_readfirstlane(R->kneed[i]);
  }
  k.n = __builtin_amdgcn_readfirstlane(R->nkeep);
  return k;
}

__device__ __forceinline__ uint16_t keep_fast(uint16_t tu, uint16_t TN, const KeepArgs& k, const uint16_t* adj) {
  if (k.n > 4) return keep_bits(tu, TN, adj);
  // unused entries hold bit 0 (the KRange is zero-initialised): no test of n
  uint32_t out = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if ((TN & k.need[i]) == k.need[i]) out |= k.bit[i];
  return static_cast<uint16_t>(out);
}

// Verify of the row at position u by the calling lane; returns survivor.
__device__ __forceinline__ bool k1_finish_row(uint32_t u, uint32_t cdelta, uint16_t tu, uint16_t TN, uint32_t len,
                                              uint32_t cnt, const uint16_t* adj, const KeepArgs& ka,
                                              const OwnerArgs& oa, const K1Out& o, BlockAcc& acc,
                                              unsigned long long* s_hist) {
  if (!TN) return false;
  const uint16_t T = keep_fast(tu, TN, ka, adj);
  if (!T) {
    acc.removed = 1;
    return false;
  }
  // 32-bit byte offsets (positions < 2^30): scalar base + vector offset stores
  const uint32_t b2 = u * 2u, b4 = u * 4u;
  *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tst) + b2) = T;
  *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.mlen) + b4) = len;
  *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.malive) + b4) = cnt;
  const uint32_t ci = u + cdelta;
  atomicOr(&o.tcode[ci >> 4], tpub_code(T, tu) << ((ci & 15u) << 1));
  // dense mode: T_pub in the record (a heavy row's M stays in its padded row: no first entry); a
  // label of more than two template vertices also keeps its position-indexed T_pub (code 3 gathers).  (Not
  // code 3 of a two-vertex label: both bits -- the removed rows of the next superstep rely on both T_pub
  // buffers being clean.)
  if (!o.rarea || tpub_wide(tu)) *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tpub) + b2) = T;
  if (oa.nranks <= 1) {
    acc.vs += 1;
    acc.es += cnt;
  } else {
    acc_owner(s_hist, oa, u, cnt);
  }
  return true;
}

// DPP lane moves (gfx9 encodings): wave_shr:1 gives lane i the value of lane
// i-1; row_shl:s gives lane i the value of lane i+s inside its 16-lane row.
__device__ __forceinline__ uint32_t dpp_wave_shr1(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(v), 0x138, 0xF, 0xF, false));
}
// wave_shr:1 with lane 0 reading 0 (no copy of an "old" value first)
__device__ __forceinline__ uint32_t dpp_wave_shr1_z(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x138, 0xF, 0xF, true));
}
template <int S>
__device__ __forceinline__ uint32_t dpp_row_shl(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x100 + S, 0xF, 0xF, true));
}

// One 64-slot slice of a row scanned by the whole wave (G >= 64 and heavy
// segments).  j = slot index of this lane inside the row; carry = the row's
// previous slot (kNone at the row start).  COMPACT: M position = running
// distinct count, else the slot itself.
template <bool COMPACT, int MODE>
__device__ __forceinline__ void k1_slice(uint32_t v, uint16_t tv, uint32_t j, uint64_t rowbase, uint16_t nm,
                                         const K1Out& o, uint32_t& cnt, uint32_t& tnacc, uint32_t& carry) {
  const int lane = lane_id();
  uint32_t pv = dpp_wave_shr1(v);
  if (lane == 0) pv = carry;
  carry = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), kWave - 1));
  const bool ok = v != kNone;
  const bool first = ok && (j == 0 || pv != v);
  const bool cm = ok && (tv & nm) != 0;
  const bool contrib = cm && first;
  const uint64_t bal = __ballot(contrib);
  if (MODE & 9) {
  } else if (COMPACT) {
    if (contrib) {
      const uint64_t dst = rowbase + cnt + __builtin_popcountll(bal & ((1ull << lane) - 1));
      o.mcol[dst] = v | kAlive;
    }
  } else if (ok) {
    o.mcol[rowbase + j] = contrib ? (v | kAlive) : v;
  }
  cnt += static_cast<uint32_t>(__builtin_popcountll(bal));
  if (cm) tnacc |= tv;
}

// A wave-uniform 64-bit value held in scalar registers.  readfirstlane returns
// int: each half goes through uint32_t, or the low half would sign-extend.
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32)));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x)));
  return (uint64_t(hi) << 32) | lo;
}

// A superstep-0 tile from its descriptor word (d_ttab): first slot, slots of its rows (0: a heavy tile),
// KRange index.  The table is read through the constant address space (scalar loads).
typedef __attribute__((address_space(4))) const uint64_t* TTab;
__device__ __forceinline__ uint64_t ttab_slot(uint64_t w) { return w & ((1ull << kTtabRemShift) - 1); }
__device__ __forceinline__ uint32_t ttab_rem(uint64_t w) {
  return static_cast<uint32_t>(w >> kTtabRemShift) & ((1u << (kTtabRangeShift - kTtabRemShift)) - 1);
}
__device__ __forceinline__ uint32_t ttab_range(uint64_t w) { return static_cast<uint32_t>(w >> kTtabRangeShift); }

// The tile after t of a wave that takes kTileBlock consecutive tiles out of every W * kTileBlock.
__device__ __forceinline__ uint32_t k1_next(uint32_t t, uint32_t W) {
  const uint32_t n = t + 1;
  return __builtin_amdgcn_readfirstlane((n % kTileBlock) ? n : n + (W - 1) * kTileBlock);
}

// The slots of a light tile in two 16-B loads per lane: load k, component c
// of lane l holds the slot at 256 k + 4 l + c of the 16-B aligned window that
// starts s = base & 3 slots before the tile (rpt * g <= kTileEntries - 4, so
// the window covers the tile).  Buffer loads through a descriptor that ends at
// the tile (lanes past it read 0, a heavy tile or a tile past the end reads
// nothing): the lane offsets are loop-invariant and no slot is masked here.
// Window slots outside the tile (the s slots before it, the tail after it) are
// phase A contributors like any other; their tile-relative slot falls outside
// [0, rows * g) and phase B drops them.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t k1_load(uint32_t (&v)[kSub], uint64_t w, const uint32_t* __restrict__ colp,
                                            uint32_t voff) {
  const uint32_t rem = ttab_rem(w);
  const uint64_t b = rem ? ttab_slot(w) : 0;
  const uint32_t s = static_cast<uint32_t>(b) & 3u;
  const uint64_t wbase = uniform64(reinterpret_cast<uint64_t>(colp + (b - s)));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(wbase), 0, static_cast<int>(__builtin_amdgcn_readfirstlane(rem ? (rem + s) * 4u : 0u)),
      0x00020000);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    // aux 2: nontemporal (the adjacency is read once per superstep 0)
    const u32x4 x = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(voff) + k * 1024, 0, 2));
#pragma unroll
    for (int c = 0; c < 4; ++c) v[4 * k + c] = x[c];
  }
  return s;
}

// Per-wave LDS staging of a light tile: the tile's contributing entries in
// slot order (neighbour position, slot relative to the tile start: outside
// [0, rows * g) for the window slots around the tile), which become M rows
// once the verify has decided which rows survive, and per-row accumulators:
// TN (two rows per word, zero between tiles) and the row's first / last + 1
// list index (valid while its TN is non-zero).
struct K1Stage {
  uint32_t lx[kTileEntries];
  uint16_t lrel[kTileEntries];
  uint16_t hd[kTileRows], tl[kTileRows];
  uint32_t tn[kTileRows / 2];
  unsigned long long sm[kTileRows / kWave];  // survivor bits of the tile's rows
};
// 4.6 KB per wave: eight 4-wave blocks (8 waves per SIMD) fit the CU's 160 KB of LDS with the block's
// other shared arrays
static_assert(sizeof(K1Stage) * kWpb + 2 * kMaxRanks * 8 + kWpb * 6 * 8 + 32 + 3 * 16 * 4 <= 160 * 1024 / 8,
              "k_lcc_first LDS exceeds 8 blocks per CU");

// Phase A of a light tile: appends the tile window's contributing slots
// (neighbour position in an admitted run, first occurrence in its row) to the
// wave's staging list in slot order and returns their number (wave-uniform).
// NR merged-run compares (unused runs have length 0); NR = 0: the full label
// test (more than four runs).  Per 16-B load: the compares of its four
// components land in 64-bit lane masks; a component's left neighbour is the
// previous component of the same lane (component 0: lane - 1's component 3),
// the row starts come from the range's masks for the tile's shift s, and a
// lane's contributors are written in component order after those of the lower
// lanes (prefix = sum of four masked popcounts), which keeps slot order.  The
// lane masks drive exec directly (inverse ballot); rel = window slot - s.
template <int NR, bool WIDE>
__device__ __forceinline__ uint32_t k1_phase_a(const uint32_t (&v)[kSub], KTab R, uint32_t s,
                                               const RelRuns& rel_runs, const uint32_t* s_runs, int nruns,
                                               uint16_t nm, K1Stage& st) {
  const int lane = lane_id();
  uint32_t nlist = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    uint64_t C[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t x = v[4 * k + c];
      uint64_t in_m = 0;  // one ballot per compare: each folds into its compare's mask
      if (NR == 0) {
        in_m = __builtin_amdgcn_ballot_w64((tbits_rel<WIDE>(x, rel_runs, s_runs, nruns) & nm) != 0);
      } else {
#pragma unroll
        for (int i = 0; i < NR; ++i) in_m |= __builtin_amdgcn_ballot_w64(x - rel_runs.alo[i] < rel_runs.alen[i]);
      }
      uint64_t ne_m;
      if (c > 0) {
        ne_m = __builtin_amdgcn_ballot_w64(v[4 * k + c - 1] != x);
      } else {
        ne_m = __builtin_amdgcn_ballot_w64(dpp_wave_shr1_z(v[4 * k + 3]) != x);
        if (k > 0) {  // lane 0 continues from lane 63's last component of the previous load
          const uint32_t p = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v[3]), kWave - 1));
          const uint32_t x0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 0));
          // (p != x0) as integer carry arithmetic: a bool here would be widened on the VALU
          ne_m = (ne_m & ~1ull) | ((uint64_t(p ^ x0) + 0xFFFFFFFFull) >> 32);
        }
        // k = 0: lane 0's component 0 is either before the tile or its first slot (a row start)
      }
      C[c] = in_m & (R->rs[s][4 * k + c] | ne_m);
    }
    const uint64_t any = C[0] | C[1] | C[2] | C[3];
    if (any) {
      if (__builtin_amdgcn_inverse_ballot_w64(any)) {
        uint32_t idx = nlist;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          idx += __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(C[c] >> 32),
                                           __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(C[c]), 0));
        // window slot relative to the tile start (wraps below 0: outside the tile)
        const uint32_t rel0 = static_cast<uint32_t>(k * 256 + 4 * lane) - s;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (__builtin_amdgcn_inverse_ballot_w64(C[c])) {
            st.lx[idx] = v[4 * k + c];
            st.lrel[idx] = static_cast<uint16_t>(rel0 + c);
            ++idx;
          }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) nlist += static_cast<uint32_t>(__builtin_popcountll(C[c]));
    }
  }
  return nlist;
}

// Row of a staged entry of a tile (kNoRow: a window slot outside the tile's rows).
static constexpr uint32_t kNoRow = 0xFFFFu;
__device__ __forceinline__ uint32_t k1_row(uint32_t rel, uint32_t rem, uint32_t rdiv) {
  return rel < rem ? (__umul24(rel, rdiv) >> 19) : kNoRow;
}

// Inclusive prefix sum over the wave's 64 lanes (DPP: four row shifts, then
// the row-15 and row-31 broadcasts).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xF, 0xF, true));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xF, 0xF, true));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xF, 0xF, true));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xF, 0xF, true));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xA, 0xF, false));
  x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xC, 0xF, false));
  return x;
}

// A dense superstep-0 record: {position, T_pub | |M| << 16 | (row start >> 32) << 25, first dense M entry,
// row start (low 32 bits)} -- |M| <= 480 (light rows) fits 9 bits; the padded row start (the slot of the row,
// where the first later superstep moves a survivor's M) rides along so that superstep needs no offp load.  A
// start at or above 127 * 2^32 codes 127: load offp.
__device__ __forceinline__ uint4 k1_record(uint32_t u, uint32_t T, uint32_t cnt, uint32_t first, uint64_t start) {
  const uint32_t hi = static_cast<uint32_t>(min<uint64_t>(start >> 32, 127));
  return make_uint4(u, T | (cnt << 16) | (hi << 25), first, static_cast<uint32_t>(start));
}

// Light tile: rem = rows * g slots from slot qb of rows of g slots (R->rpt = min((kTileEntries - 4) / g,
// kTileRows) rows per tile), the first at position ustart.
// Phase A, per 16-B load, all in wave masks: a lane's neighbour can contribute
// iff its position lies in one of the range's relevant label runs (one
// compare per run, the masks OR-ed on the scalar unit) and it is the first
// occurrence in its row (row start, or differs from its left neighbour);
// only the contributing lanes (a few percent of the slots) are appended to
// the LDS staging list.  Phase B1: row TN / first and last list index from
// the list (entries outside the tile's rows dropped).  Phase B2, one lane per
// row of the groups that hold listed rows: verify, and the survivors' state
// goes out at once.  Dense M (o.rarea): one 16-B record per survivor in the
// wave's record slice {position, T_pub | |M| << 16, first M entry, 0}
// (T_state = T_pub and the alive count = |M| are implied until the first later
// superstep rewrites them) and the survivors' M entries compacted into the
// wave's slice of the dense region (the records' first entries are the
// exclusive prefix sums of |M| over the tile's survivors); otherwise
// position-indexed state, survivor mask words, the tile's count, and M at the
// start of each survivor's padded row; the 2-bit T_pub code OR-ed into tcode.
// The stores are issued
// in place: held back to the next iteration they cost more (the pending
// state's registers) than the wait for them at its top.
template <int MODE, bool WIDE>
__device__ __forceinline__ void k1_light_tile(const uint32_t (&v)[kSub], uint32_t s, uint64_t qb, uint32_t rem,
                                              uint32_t ustart, uint32_t rows, uint32_t g, uint32_t rpt,
                                              uint32_t rdiv, KTab R, uint16_t tu, uint16_t nm,
                                              const RelRuns& rel_runs, const uint32_t* s_runs, int nruns,
                                              const KeepArgs& keep, const uint16_t* s_adj, const OwnerArgs& oa,
                                              BlockAcc& acc, unsigned long long* s_hist, unsigned long long* tm,
                                              uint32_t tile, K1Stage& st, const K1Out& o, uint64_t& dcur,
                                              uint64_t dend, uint64_t& rcur, uint32_t cstart) {
  const int lane = lane_id();
  // admission compares specialised on the number of merged runs (wave-uniform)
  uint32_t nlist;
  if (WIDE || rel_runs.nadm > 4)
    nlist = k1_phase_a<0, WIDE>(v, R, s, rel_runs, s_runs, nruns, nm, st);
  else if (rel_runs.nadm <= 1)
    nlist = k1_phase_a<1, false>(v, R, s, rel_runs, s_runs, nruns, nm, st);
  else if (rel_runs.nadm == 2)
    nlist = k1_phase_a<2, false>(v, R, s, rel_runs, s_runs, nruns, nm, st);
  else
    nlist = k1_phase_a<4, false>(v, R, s, rel_runs, s_runs, nruns, nm, st);
  nlist = __builtin_amdgcn_readfirstlane(nlist);
  if (MODE & 16) return;  // diagnostic: phase A only
  // position-indexed mode: the slist build reads every tile's count
  const bool counts = !o.rarea && !(MODE & 128);
  if (nlist == 0) {
    if (counts && lane == 0) {
      o.tcnt[tile] = 0u;
      o.tstart[tile] = ustart;
    }
    return;
  }
  __builtin_amdgcn_wave_barrier();
  // Dense mode with at most 64 contributors (the common case: ~20 per tile at S=28): phases B1, B2 and the
  // M stores in registers, one contributor per lane in list order.  A row's contributors are consecutive
  // lanes; its head lane (first lane of the row) verifies it with the row's TN (OR-ed in the row's LDS half
  // word) and |M| = its run of lanes; the kept lanes (rows that survive) store their entries compacted.
  // (diagnostic builds: MODE 1024 / 2048 / 4096 drop the register path's code atomics / M stores / records)
  if ((MODE & ~(1024 | 2048 | 4096)) == 0 && o.rarea && nlist <= static_cast<uint32_t>(kWave) &&
      dcur + nlist <= dend) {
    const bool valid = static_cast<uint32_t>(lane) < nlist;
    uint32_t x = 0, row = kNoRow;
    if (valid) {
      x = st.lx[lane];
      row = k1_row(st.lrel[lane], rem, rdiv);
    }
    const bool inrow = row != kNoRow;
    const uint32_t r1 = inrow ? row + 1u : 0u;  // (0: no row; lane 0 reads 0 from the shift)
    const bool head = inrow && dpp_wave_shr1_z(r1) != r1;
    const uint64_t im = __builtin_amdgcn_ballot_w64(inrow);
    if (!im) return;  // only window slots outside the tile's rows
    const uint64_t hm = __builtin_amdgcn_ballot_w64(head);
    if (inrow)
      atomicOr(&st.tn[row >> 1], static_cast<uint32_t>(tbits_rel<WIDE>(x, rel_runs, s_runs, nruns) & nm)
                                     << ((row & 1u) << 4));
    __builtin_amdgcn_wave_barrier();
    uint16_t* tn16 = reinterpret_cast<uint16_t*>(st.tn);
    uint16_t T = 0;
    uint32_t cnt = 0;
    if (head) {
      const uint16_t TN = tn16[row];
      // the row's lanes run up to the next head or the first lane past the tile's rows
      const uint64_t ends = (hm | ~im) & ~((2ull << lane) - 1ull);  // (lane 63: shift of 64 wraps to 0)
      const uint32_t nxt = lane == kWave - 1 || !ends ? static_cast<uint32_t>(kWave)
                                                      : static_cast<uint32_t>(__builtin_ctzll(ends));
      cnt = nxt - static_cast<uint32_t>(lane);
      if (TN) {  // (an admitted contributor always meets nm: TN != 0)
        T = keep_fast(tu, TN, keep, s_adj);
        if (!T) {
          acc.removed = 1;
        } else if (oa.nranks <= 1) {
          acc.vs += 1;
          acc.es += cnt;
        } else {
          acc_owner(s_hist, oa, ustart + row, cnt);
        }
        tn16[row] = 0;  // (TN words are zero between tiles)
      }
    }
    const uint64_t sb = __builtin_amdgcn_ballot_w64(T != 0);
    if (!sb) return;
    // a lane is kept iff the head of its row (the highest head lane at or below it) survives
    const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t hb = hm & upto;
    const bool kept = inrow && hb && ((sb >> (63 - __builtin_clzll(hb))) & 1ull);
    const uint64_t kb = __builtin_amdgcn_ballot_w64(kept);
    const uint32_t kidx = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(kb >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(kb), 0));
    if (kept && !(MODE & 2048)) o.mcol[o.dbase + dcur + kidx] = x | kAlive;
    if (T) {
      const uint32_t u = ustart + row;
      const uint32_t code = tpub_code(T, tu);
      // (one atomic per survivor: merging a tile's codes per word first -- a wave scan or a scalar walk over the
      // survivor lanes -- measured 1.94 / 1.89 ms per launch instead of 1.47 although it cut WRITE to 0.38 GB)
      const uint32_t ci = cstart + row;
      if (!(MODE & 1024)) atomicOr(&o.tcode[ci >> 4], code << ((ci & 15u) << 1));
      if (tpub_wide(tu)) *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tpub) + u * 2u) = T;
      const uint64_t rslot = rcur + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(sb >> 32),
                                                              __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(sb), 0));
      // the head's kidx: the kept entries before its row (consecutive lanes) = its first dense entry
      if (!(MODE & 4096))
        o.rarea[rslot] = k1_record(u, T, cnt, static_cast<uint32_t>(dcur + kidx), qb + uint64_t(row) * g);
    }
    rcur = uniform64(rcur + __builtin_popcountll(sb));
    dcur = uniform64(dcur + __builtin_popcountll(kb));
    return;
  }
  // phase B1 over the list: a row's entries are consecutive (slot order), so
  // its first entry records the row's first list index and its last entry the
  // end; TN is OR-ed into the row's half word.  The lowest and highest listed
  // rows bound the groups B2 visits.
  uint32_t rlo = kNoRow, rhi = 0;
#pragma unroll 1
  for (uint32_t i0 = 0; i0 < nlist; i0 += kWave) {
    const uint32_t i = i0 + lane;
    uint32_t row = kNoRow;
    if (i < nlist) {
      const uint32_t x = st.lx[i];
      row = k1_row(st.lrel[i], rem, rdiv);
      if (row != kNoRow) {
        const uint32_t prow = i ? k1_row(st.lrel[i - 1], rem, rdiv) : kNoRow;
        const uint32_t nrow = i + 1 < nlist ? k1_row(st.lrel[i + 1], rem, rdiv) : kNoRow;
        if (row != prow) st.hd[row] = static_cast<uint16_t>(i);
        if (row != nrow) st.tl[row] = static_cast<uint16_t>(i + 1);
        atomicOr(&st.tn[row >> 1], static_cast<uint32_t>(tbits_rel<WIDE>(x, rel_runs, s_runs, nruns) & nm)
                                       << ((row & 1u) << 4));
      }
    }
    // listed rows are increasing along the list: the chunk's first / last valid lanes hold its extremes
    const uint64_t vm = __builtin_amdgcn_ballot_w64(row != kNoRow);
    if (vm) {
      const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(row), __builtin_ctzll(vm)));
      const uint32_t z = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(row), 63 - __builtin_clzll(vm)));
      rlo = min(rlo, a);
      rhi = max(rhi, z);
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (rlo == kNoRow) {  // only window slots outside the tile's rows
    if (counts && lane == 0) {
      o.tcnt[tile] = 0u;
      o.tstart[tile] = ustart;
    }
    return;
  }
  if (MODE & 32) {  // diagnostic: phase A + B1 only
    for (uint32_t r = lane; r < rpt; r += 2 * kWave) st.tn[r >> 1] = 0;
    return;
  }
  // phase B2 over the groups [g0, g1) that hold listed rows
  uint16_t* tn16 = reinterpret_cast<uint16_t*>(st.tn);
  const uint32_t g0 = rlo / kWave, g1 = rhi / kWave + 1;
  // dense M when the tile's list fits the rest of the wave's slice (the survivors' entries are a part of it)
  const bool dense = o.rarea && dcur + nlist <= dend;
  const uint64_t dpos = dcur;
  uint32_t mrun = 0;  // survivors' M entries of the groups before this one
  uint32_t any = 0;
#pragma unroll 1
  for (uint32_t gi = g0; gi < g1; ++gi) {
    const uint32_t row = gi * kWave + lane;
    uint16_t T = 0;
    uint32_t cnt = 0;
    if (row <= rhi) {
      const uint16_t TN = tn16[row];
      if (TN) {
        cnt = static_cast<uint32_t>(st.tl[row]) - st.hd[row];
        T = keep_fast(tu, TN, keep, s_adj);
        if (!T) {
          acc.removed = 1;
        } else if (oa.nranks <= 1) {
          acc.vs += 1;
          acc.es += cnt;
        } else {
          acc_owner(s_hist, oa, ustart + row, cnt);
        }
        tn16[row] = 0;  // (TN words are zero between tiles)
      }
    }
    const bool surv = T != 0;
    const uint64_t b = __builtin_amdgcn_ballot_w64(surv);
    if (lane == 0) st.sm[gi] = b;
    if (!b) continue;
    any += static_cast<uint32_t>(__builtin_popcountll(b));
    // the survivors' first M entries in the tile's compacted M: exclusive prefix of |M| over them
    const uint32_t c = surv ? cnt : 0u;
    const uint32_t incl = wave_incl_sum(c);
    if (surv) {
      const uint32_t code = tpub_code(T, tu);
      if (!(MODE & 128)) {
        // 32-bit byte offsets (positions < 2^30): scalar base + vector offset stores
        const uint32_t u = ustart + row, b2 = u * 2u, b4 = u * 4u;
        if (!(MODE & 512)) {
          const uint32_t ci = cstart + row;  // code index of row 0 + row (wave-uniform base)
          atomicOr(&o.tcode[ci >> 4], code << ((ci & 15u) << 1));
        }
        if (o.rarea) {
          if (!dense) {
            *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tst) + b2) = T;
            *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.mlen) + b4) = cnt;
            *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.malive) + b4) = cnt;
          }
          // a label of more than two template vertices keeps its position-indexed T_pub (the next
          // superstep's code-3 gathers)
          if (tpub_wide(tu)) *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tpub) + b2) = T;
          const uint64_t rslot = rcur + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(b >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(b), 0));
          o.rarea[rslot] = k1_record(u, T, cnt, dense ? static_cast<uint32_t>(dpos + mrun + incl - c) : kNone,
                                     qb + uint64_t(row) * g);
        } else {
          *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tst) + b2) = T;
          *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(o.tpub) + b2) = T;
          *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.mlen) + b4) = cnt;
          *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(o.malive) + b4) = cnt;
        }
      }
      if (!dense) st.hd[row] = static_cast<uint16_t>(mrun + incl - c);  // (the padded M copy below)
    }
    if (o.rarea) rcur = uniform64(rcur + __builtin_popcountll(b));
    mrun += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), kWave - 1));
  }
  if (counts) {  // survivor mask words (bit r = row r) up to the last group with listed rows; the count
    if (static_cast<uint32_t>(lane) < g1) tm[lane] = static_cast<uint32_t>(lane) >= g0 ? st.sm[lane] : 0ull;
    if (lane == 0) {
      o.tcnt[tile] = any;
      o.tstart[tile] = ustart;
    }
  }
  if (!any) return;
  if (MODE & 129) return;  // diagnostics: without the M stores
  // the survivors' entries in list order: entry i is the kidx-th kept one, and the kidx - hd[r]-th of its
  // row r (hd: the row's first entry in the compacted M)
  uint32_t* const dm = o.mcol + o.dbase + dpos;
  char* const mtile = reinterpret_cast<char*>(o.mcol + qb);  // 32-bit in-tile offsets
  uint32_t base = 0;
#pragma unroll 1
  for (uint32_t i0 = 0; i0 < nlist; i0 += kWave) {
    const uint32_t i = i0 + lane;
    bool kept = false;
    uint32_t row = kNoRow;
    if (i < nlist) {
      row = k1_row(st.lrel[i], rem, rdiv);
      kept = row != kNoRow && ((st.sm[row / kWave] >> (row % kWave)) & 1ull);  // (listed rows lie in [g0, g1))
    }
    const uint64_t kb = __builtin_amdgcn_ballot_w64(kept);
    if (kept) {
      const uint32_t kidx = base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(kb >> 32),
                                                             __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(kb), 0));
      const uint32_t x = st.lx[i] | kAlive;
      if (dense) dm[kidx] = x;
      else *reinterpret_cast<uint32_t*>(mtile + ((row * g + (kidx - st.hd[row])) << 2)) = x;
    }
    base += static_cast<uint32_t>(__builtin_popcountll(kb));
  }
  if (dense) dcur = uniform64(dcur + mrun);
}

// Heavy rows (above kHeavyDeg): one kHeavyDeg segment per tile, uncompacted M;
// the segments' TN / counts meet in the hscr scratch and the last segment to
// finish (ticket) runs the verify.  Rare: kept out of line.
template <int MODE, bool WIDE>
__device__ __forceinline__ BlockAcc k1_heavy_tile(KTab kt, uint32_t hi,
                                                            const HSeg* __restrict__ hseg,
                                                            const uint64_t* __restrict__ offp,
                                                            const uint32_t* __restrict__ colp, const uint32_t* s_runs,
                                                            int nruns, const uint16_t* s_adj, OwnerArgs oa, K1Out o,
                                                            uint32_t* __restrict__ hscr, uint32_t nheavy,
                                                            unsigned long long* s_hist, unsigned long long* tm) {
  BlockAcc acc;
  const int lane = lane_id();
  const HSeg hs = hseg[hi];
  const KTab R = kt + __builtin_amdgcn_readfirstlane(hs.range);
  const uint16_t tu = R->tu;
  const uint16_t nm = R->nm;
  const RelRuns rel_runs = load_rel(R);
  const KeepArgs keep = load_keep(R);
  const uint64_t b0 = offp[hs.row];
  const uint32_t deg = static_cast<uint32_t>(offp[hs.row + 1] - b0);
  const uint32_t j_beg = hs.seg * kHeavyDeg;
  const uint32_t j_end = min(deg, j_beg + kHeavyDeg);
  uint32_t cnt = 0, tnacc = 0;
  uint32_t carry = j_beg ? colp[b0 + j_beg - 1] : kNone;
  for (uint32_t j0 = j_beg; j0 < j_end; j0 += kSub * kWave) {
    uint32_t v[kSub];
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
      const uint32_t j = j0 + q * kWave + lane;
      v[q] = j < j_end ? colp[b0 + j] : kNone;
    }
#pragma unroll
    for (int q = 0; q < kSub; ++q)
      k1_slice<false, MODE>(v[q], tbits_rel<WIDE>(v[q], rel_runs, s_runs, nruns), j0 + q * kWave + lane, b0, nm, o,
                            cnt, tnacc, carry);
  }
  const uint16_t TN = wave_or_bits(tnacc, nm, 0, ~0ull);
  bool surv = false;
  if (lane == 0 && !(MODE & 8)) {
    uint32_t* h_tn = hscr;
    uint32_t* h_cnt = hscr + nheavy;
    uint32_t* h_done = hscr + 2 * nheavy;
    if (TN) atomicOr(&h_tn[hs.h], static_cast<uint32_t>(TN));
    if (cnt) atomicAdd(&h_cnt[hs.h], cnt);
    __threadfence();
    // (a delegate's share: its TN / count stay in the scratch for shard_hub_combine)
    if (atomicAdd(&h_done[hs.h], 1u) == hs.nseg - 1 && !hs.split) {
      __threadfence();
      const uint16_t TNall = static_cast<uint16_t>(atomicOr(&h_tn[hs.h], 0u));
      const uint32_t call = atomicAdd(&h_cnt[hs.h], 0u);
      surv = k1_finish_row(hs.row, R->cdelta, tu, TNall, deg, call, s_adj, keep, oa, o, acc, s_hist);
      // dense mode: the heavy row's record (its M in the padded row); hrec was zeroed before the launch
      if (surv && o.hrec) o.hrec[hs.h] = make_uint4(hs.row, 0u, kNone, 1u);
    }
  }
  if (!o.rarea) {
    if (lane == 0 && surv && !(MODE & 8)) tm[0] = 1ull;  // (read only when the tile count is 1)
    if (lane == 0 && !(MODE & 8)) {
      o.tcnt[hs.tile] = surv ? 1u : 0u;
      o.tstart[hs.tile] = hs.row;
    }
  }
  return acc;
}

// MODE (diagnostic builds only, 0 in the product): bit0 drops the M stores, bit9 the T_pub code atomics,
// bit1 skips light tiles, bit2 skips heavy tiles, bit3 keeps only the loads
// and the label test (checksum), bit4 stops light tiles after phase A, bit5
// after phase B1.  WIDE: some range has more than four
// relevant label runs (tbits_rel scans them all).
// NT > 1: NT tiles per wait -- the slots of the next NT tiles in flight while the current NT are processed (NT
// times the bytes in flight per wave, 1/NT of the waits; more registers, fewer waves).
template <int MODE, bool WIDE = false, int WMIN = 8, int NT = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WMIN, 8))) void k_lcc_first(
    const KRange* __restrict__ ktab, const uint64_t* __restrict__ ttab, uint32_t ntiles, const HSeg* __restrict__ hseg,
    const uint64_t* __restrict__ offp, const uint32_t* __restrict__ colp, LabelRuns lr, PatArgs pa, OwnerArgs oa,
    K1Out o, uint32_t* __restrict__ hscr, uint32_t nheavy, uint32_t nhseg, unsigned long long* __restrict__ tmask,
    Partials pp) {
  const KTab kt = (KTab)ktab;  // nr + 1 entries, read by scalar loads
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  __shared__ uint16_t s_adj[16];
  __shared__ uint32_t s_runs[3 * 16];
  __shared__ K1Stage s_stage[kWpb];
  load_adj(s_adj, pa);
  if (threadIdx.x < 16) {
    const int l = threadIdx.x;
    s_runs[3 * l] = lr.lo[l];
    s_runs[3 * l + 1] = l < lr.n ? lr.len[l] : 0u;
    s_runs[3 * l + 2] = lr.tu[l];
  }
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform
  K1Stage& st = s_stage[wid];
  for (int i = threadIdx.x % kWave; i < static_cast<int>(kTileRows / 2); i += kWave) st.tn[i] = 0;
  __syncthreads();
  BlockAcc acc;
  // (wave-uniform: left to the compiler the grid stride lands in a VGPR, the next-tile test becomes a
  // divergent branch and every loop-carried tile field a VGPR copied and re-read each iteration)
  const uint32_t W = __builtin_amdgcn_readfirstlane(gridDim.x * kWpb);
  const int nruns = lr.n;
  const TTab tt = (TTab)ttab;
  const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWpb + wid);
  // one light tile (w: its descriptor, v: its slots, s: their alignment shift); a heavy tile or a tile past the
  // end (w = 0) does nothing here
  auto light2 = [&](uint32_t t, uint64_t wcur, const uint32_t (&vc)[kSub], uint32_t sc, uint64_t& dcur,
                    uint64_t dend, uint64_t& rcur) {
    const uint32_t rem = ttab_rem(wcur);
    if (rem) {  // a light tile (heavy tiles: the loop below)
      const KTab R = kt + ttab_range(wcur);
      const uint16_t tu = R->tu;
      const uint16_t nm = R->nm;
      const RelRuns rel_runs = load_rel(R);
      if (MODE & 8) {
#pragma unroll
        for (int q = 0; q < kSub; ++q) acc.vs += vc[q] ^ tbits_rel<WIDE>(vc[q], rel_runs, s_runs, nruns);
      } else if (!(MODE & 2)) {
        const KeepArgs keep = load_keep(R);
        const uint32_t rpt = R->rpt;
        const uint32_t ustart = R->start + (t - R->tile0) * rpt;
        const uint32_t rows = min(rpt, R->end - ustart);
        k1_light_tile<MODE, WIDE>(vc, sc, ttab_slot(wcur), rem, ustart, rows, R->g, rpt, R->rdiv, R, tu, nm,
                                  rel_runs, s_runs, nruns, keep, s_adj, oa, acc, s_hist, tmask + uint64_t(t) * kSub, t,
                                  st, o, dcur, dend, rcur, ustart + R->cdelta);
      }
    }
  };
  if constexpr (NT > 1) {
    // NT tiles per wait: the slots of the next NT tiles in flight while the current NT are processed
    uint32_t tc[NT], tx[NT], sc[NT], sx[NT];
    uint64_t wc[NT], wx[NT];
    uint32_t vc[NT][kSub], vx[NT][kSub];
    const uint32_t voff = 16u * static_cast<uint32_t>(lane_id());
    tc[0] = gw * kTileBlock;
#pragma unroll
    for (int i = 1; i < NT; ++i) tc[i] = k1_next(tc[i - 1], W);
    tx[0] = k1_next(tc[NT - 1], W);
#pragma unroll
    for (int i = 1; i < NT; ++i) tx[i] = k1_next(tx[i - 1], W);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      wc[i] = tc[i] < ntiles ? tt[tc[i]] : 0ull;
      wx[i] = tx[i] < ntiles ? tt[tx[i]] : 0ull;
      sc[i] = k1_load(vc[i], wc[i], colp, voff);
    }
    uint64_t dcur = uniform64(uint64_t(gw) * o.dslice);
    const uint64_t dend = uniform64(dcur + o.dslice);
    uint64_t rcur = o.rarea ? uniform64(o.rbase[gw]) : 0;
    while (tc[0] < ntiles) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        tc[i] = __builtin_amdgcn_readfirstlane(tc[i]);
        tx[i] = __builtin_amdgcn_readfirstlane(tx[i]);
        wc[i] = uniform64(wc[i]);
        wx[i] = uniform64(wx[i]);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the current tiles' slots (and the last group's stores)
      dcur = uniform64(dcur);
      rcur = uniform64(rcur);
      uint32_t ty[NT];
      uint64_t wy[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) sx[i] = k1_load(vx[i], wx[i], colp, voff);
      ty[0] = k1_next(tx[NT - 1], W);
#pragma unroll
      for (int i = 1; i < NT; ++i) ty[i] = k1_next(ty[i - 1], W);
#pragma unroll
      for (int i = 0; i < NT; ++i) wy[i] = ty[i] < ntiles ? tt[ty[i]] : 0ull;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        sc[i] = __builtin_amdgcn_readfirstlane(sc[i]);
        light2(tc[i], wc[i], vc[i], sc[i], dcur, dend, rcur);
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        tc[i] = tx[i];
        tx[i] = ty[i];
        wc[i] = wx[i];
        wx[i] = wy[i];
        sc[i] = sx[i];
#pragma unroll
        for (int q = 0; q < kSub; ++q) vc[i][q] = vx[i][q];
      }
    }
    rcur = uniform64(rcur);
    if (o.rarea && lane_id() == 0) o.rcnt[gw] = static_cast<uint32_t>(rcur - o.rbase[gw]);
  } else {
    // tiles t = (j W + gw) kTileBlock + i; descriptors read one tile ahead of the loads they address, the
    // slots of the next tile in flight while the current one is processed
    uint32_t t = gw * kTileBlock;
    uint32_t tn = k1_next(t, W);
    uint64_t wcur = t < ntiles ? tt[t] : 0ull, wnx = tn < ntiles ? tt[tn] : 0ull;
    uint32_t vc[kSub], vn[kSub];
    const uint32_t voff = 16u * static_cast<uint32_t>(lane_id());  // byte offset of the lane's 16 B in a load
    uint32_t sc = k1_load(vc, wcur, colp, voff);
    // dense M: this wave's slice of the region
    uint64_t dcur = uniform64(uint64_t(gw) * o.dslice);
    const uint64_t dend = uniform64(dcur + o.dslice);
    // dense mode: this wave's record slice
    uint64_t rcur = o.rarea ? uniform64(o.rbase[gw]) : 0;
    while (t < ntiles) {
      t = __builtin_amdgcn_readfirstlane(t);
      tn = __builtin_amdgcn_readfirstlane(tn);
      wcur = uniform64(wcur);
      wnx = uniform64(wnx);
      // this tile's slots (requested a whole tile ago) and the previous tile's stores are complete here,
      // ahead of the next tile's loads: the vector memory counter retires in issue order, so a wait at
      // the first use would also wait for the stores this tile issues
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      dcur = uniform64(dcur);
      rcur = uniform64(rcur);
      const uint32_t sn = k1_load(vn, wnx, colp, voff);
      const uint32_t tnn = k1_next(tn, W);
      const uint64_t wnn = tnn < ntiles ? tt[tnn] : 0ull;
      sc = __builtin_amdgcn_readfirstlane(sc);
      // (the body of light2, written out: the lambda costs this loop ~6 % through its register allocation)
      const uint32_t rem = ttab_rem(wcur);
      if (rem) {  // a light tile (heavy tiles: the loop below)
        const KTab R = kt + ttab_range(wcur);
        const uint16_t tu = R->tu;
        const uint16_t nm = R->nm;
        const RelRuns rel_runs = load_rel(R);
        if (MODE & 8) {
#pragma unroll
          for (int q = 0; q < kSub; ++q) acc.vs += vc[q] ^ tbits_rel<WIDE>(vc[q], rel_runs, s_runs, nruns);
        } else if (!(MODE & 2)) {
          const KeepArgs keep = load_keep(R);
          const uint32_t rpt = R->rpt;
          const uint32_t ustart = R->start + (t - R->tile0) * rpt;
          const uint32_t rows = min(rpt, R->end - ustart);
          k1_light_tile<MODE, WIDE>(vc, sc, ttab_slot(wcur), rem, ustart, rows, R->g, rpt, R->rdiv, R, tu, nm,
                                    rel_runs, s_runs, nruns, keep, s_adj, oa, acc, s_hist, tmask + uint64_t(t) * kSub,
                                    t, st, o, dcur, dend, rcur, ustart + R->cdelta);
        }
      }
      t = tn;
      tn = tnn;
      wcur = wnx;
      wnx = wnn;
      sc = sn;
#pragma unroll
      for (int q = 0; q < kSub; ++q) vc[q] = vn[q];
    }
    rcur = uniform64(rcur);
    if (o.rarea && lane_id() == 0) o.rcnt[gw] = static_cast<uint32_t>(rcur - o.rbase[gw]);
  }
  // heavy rows, one segment per wave at a time (a separate loop: no slot
  // buffers live, so the light loop's register budget is its own)
  if (!(MODE & 4))
    for (uint32_t hi = blockIdx.x * kWpb + wid; hi < nhseg; hi += W) {
      const BlockAcc h = k1_heavy_tile<MODE, WIDE>(kt, hi, hseg, offp, colp, s_runs, nruns, s_adj, oa, o, hscr,
                                                   nheavy, s_hist, tmask + uint64_t(hseg[hi].tile) * kSub);
      acc.vs += h.vs;
      acc.es += h.es;
      acc.removed |= h.removed;
    }
  flush_block(acc, oa, s_hist, s_red, pp);
}
// slist from the superstep-0 survivor masks: an exclusive scan of the
// per-tile survivor counts (rocPRIM) gives each tile's base; a tile's mask bit
// r is row r of the tile, at position tstart + r (a heavy tile: bit 0, its row).
__global__ void k_slist_write(const uint32_t* __restrict__ tcnt, const uint32_t* __restrict__ tstart,
                              const unsigned long long* __restrict__ tmask, const uint64_t* __restrict__ base,
                              uint32_t ntiles, uint32_t* __restrict__ slist, uint32_t* __restrict__ nS) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x) {
    uint32_t c = tcnt[t];
    uint64_t o = base[t];
    if (t == ntiles - 1) *nS = static_cast<uint32_t>(o + c);
    if (!c) continue;
    const uint32_t p0 = tstart[t];
    const unsigned long long* w = tmask + uint64_t(t) * kSub;
    for (uint32_t q = 0; c && q < kSub; ++q) {
      unsigned long long m = w[q];
      c -= static_cast<uint32_t>(__builtin_popcountll(m));
      while (m) {
        const int b = __ffsll(static_cast<long long>(m)) - 1;
        m &= m - 1;
        slist[o++] = p0 + q * kWave + static_cast<uint32_t>(b);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K2: one later LCC superstep fused with its verify (pull form over M).
//
// Senders (nonunique_ee.hpp:571-633): v in S with T_pub(v) != 0 sends T_pub(v)
// to every u in M[v].  Receivers (:412-443, :647-816): u in S, T_pub(u) != 0,
// valid parent -> TN(u) |= T_pub(v), flag M[u][v].  On the symmetric active-edge
// map ("M symmetry") u in M[v] <=> v in M[u], so each row u pulls
// from its own entries.  Verify (:886-977): keep_bits(T_state, TN); empty ->
// removed; else T_pub = T_state, erase flag-0 entries, clear flags.  An entry
// whose flag was preset by a cycle terminal (nem_1.hpp:764-770) survives one
// verify without a message; if its neighbour is still in S that breaks the
// symmetry, which is reported through the asymmetry counter (the host then
// refuses to go on).
//
// After superstep 0 the rows are short (a few entries): one lane per row of
// slist walks its row four entries at a time (four independent loads, then
// four T_pub gathers); rows above kLprMax entries are walked by the whole
// wave, one after the other.  Dead 64-entry chunks of slist are skipped
// through the live mask of the previous superstep.
static constexpr uint32_t kLprMax = 32;

// Rows above kPullLong entries (R-MAT hubs that survived superstep 0 with their superstep-0 length: up to millions
// of entries at C5 S=27, of which a few thousand stay alive) are not walked by one wave, which made the pull
// supersteps of C5's first call 15 / 6 / 5 ms long: the step kernel defers such a row to a list and every wave of a
// second launch (k_lcc_step_pieces) takes kPullPiece-entry pieces of the listed rows; the last piece of a row to
// finish verifies it.  In the call's last pull superstep the pieces also pack the row's alive entries (a scratch
// slice per piece) and k_long_pack moves them to the row start: the row compaction at the end of the call
// (k_compact_rows: one wave per row, 12 ms at C5) finds these rows compacted.
static constexpr uint32_t kPullLong = 4096;
static constexpr uint32_t kPullPiece = 2048;
struct LongRow {
  uint32_t u;        // position
  uint32_t i;        // slist index (chunk i / 64, bit i % 64 of the live / keep masks)
  uint64_t beg;      // first M entry
  uint32_t len;      // M entries
  uint16_t Ts, nm;   // T_state, neighbour mask of T_pub
  uint64_t pbase;    // number of its first piece (pieces are numbered over the whole list, in list order)
  uint32_t tn, cnt;  // the pieces' OR / count
  uint32_t done;     // pieces finished (ticket)
  uint32_t T;        // T_pub after the verify (0: removed)
};
struct LongList {
  LongRow* rows;            // null: every row is walked in the step kernel
  unsigned long long* cnt;  // listed rows << 32 | their pieces (counter slot word 2P + 4): one atomic reserves both,
                            // so the rows' first pieces increase with their list index
  uint32_t cap;
  uint32_t min_len;         // rows above this many entries are listed (kPullLong; PM_PULL_LONG in tests)
  uint32_t* scr;            // last pull superstep: piece k's alive entries at scr + k * kPullPiece (null: no packing)
  uint32_t* pcnt;           // ... and their number
  uint64_t scr_pieces;      // pieces the scratch holds (a row with a piece beyond it is left to k_compact_rows)
};

// (store = false: timing variant PM_DIAG_STEP & 4)
__device__ __forceinline__ void k2_entry(uint32_t* __restrict__ mcol, uint64_t e, uint32_t m, uint16_t tv,
                                         uint16_t nm, uint32_t& tn, uint32_t& cnt, bool& asym, bool store = true) {
  const bool ok = (tv & nm) != 0;
  const bool fl = (m & kFlag) != 0;
  const bool flag = ok || fl;
  const uint32_t m2 = (m & kPosMask) | (flag ? kAlive : 0u);  // flags cleared by verify
  if (store && m2 != m) mcol[e] = m2;
  if (fl && !ok && tv) asym = true;
  if (ok) tn |= tv;
  cnt += flag ? 1u : 0u;
}

__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) x |= __shfl_xor(x, d, kWave);
  return x;
}

__device__ __forceinline__ uint32_t wave_max32(uint32_t x) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) x = max(x, static_cast<uint32_t>(__shfl_xor(x, d, kWave)));
  return x;
}

// The superstep-0 records in place (one context): the concatenation of the waves' slices is indexed through the
// slice of each 64-record chunk (cdesc) and the slices' output offsets (rofs, rofs[W] = the light records); the
// heavy survivors' records follow in srec.  The first later superstep writes slist (the positions) as it reads.
struct RecSrc {
  const uint4* rarea;
  const uint64_t* rbase;
  const uint64_t* rofs;
  const uint4* cdesc;  // per chunk {rarea index of its first record (lo, hi), its records in that slice, next slice}
  uint32_t W;
};
// U: entries in flight per lane in the flattened rows.  3 when the superstep's rows are short (S=28's first
// later superstep: 3.2 entries per row, a chunk of 64 rows fits one round of 192; 4 spills 16 VGPRs at 6 waves
// per SIMD, and the spill reloads are memory operations in the same in-order counter: 564 -> 519 us), 4
// otherwise (C5: longer rows, 4 in flight was 10-40 % faster on every pull superstep).
#ifndef PM_STEP_WAVES
#define PM_STEP_WAVES 6  // waves per SIMD the register budget of k_lcc_step is sized for
#endif
// FIRST: the first later superstep with superstep-0 records and codes (srec, tcode non-null, every entry live):
// the generic paths folded away, so the instantiation holds only the registers that superstep needs.
template <int U, bool FIRST = false, int WAVES = PM_STEP_WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void k_lcc_step(
    const uint64_t* __restrict__ offp, const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp,
    const unsigned long long* __restrict__ mask_in, unsigned long long* __restrict__ mask_out,
    uint16_t* __restrict__ tcur, uint16_t* __restrict__ tnxt, uint16_t* __restrict__ tst, PatArgs pa,
    OwnerArgs oa, uint32_t* __restrict__ mcol, uint32_t* __restrict__ mlen,
    uint32_t* __restrict__ malive, Partials pp, const uint32_t* __restrict__ tcode, LabelRuns lr, uint32_t diag,
    const uint4* __restrict__ srec, uint64_t dbase, unsigned long long* __restrict__ keep_out, RecSrc rs,
    uint32_t* __restrict__ slist_out, LongList ll, int pub_state, int dead_state) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  __shared__ uint16_t s_adj[16];
  __shared__ uint64_t s_beg[kWpb][kWave];  // flattened short rows (per wave)
  __shared__ uint32_t s_end[kWpb][kWave], s_tn[kWpb][kWave], s_cnt[kWpb][kWave];
  __shared__ uint16_t s_nm[kWpb][kWave];
  __shared__ uint64_t s_dst[kWpb][kWave];  // dense survivors' padded row starts (flattened copy)
  // FIRST: the flattened dense rows' entries are not updated in place -- their alive bits after the walk (bit t of the
  // walk) go to LDS and the survivors' row moves apply them; a removed row's dense entries are never read again
  constexpr int kAlvWords = kWave * kLprMax / 64 + 4;
  __shared__ unsigned long long s_alv[FIRST ? kWpb : 1][FIRST ? kAlvWords : 1];
  __shared__ uint32_t s_wofs[FIRST ? kWpb : 1][FIRST ? kWave : 1];  // the row's first walk entry (~0: stored in place)
  __shared__ uint32_t s_rlo[16], s_rlen[16], s_rtu[16], s_rcd[16];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  load_adj(s_adj, pa);
  if (threadIdx.x < 16) {
    const int l = threadIdx.x;
    s_rlo[l] = lr.lo[l];
    s_rlen[l] = l < lr.n ? lr.len[l] : 0u;
    s_rtu[l] = lr.tu[l];
    s_rcd[l] = lr.cd[l];
  }
  __syncthreads();
  const int nruns = lr.n;
  // T_pub of neighbour position p: from the 2-bit codes when present (the
  // label's template bits from its run), the T_pub array otherwise
  auto tpub_of = [&](uint32_t p) -> uint16_t {
    if (!FIRST && !tcode) return tcur[p];
    // the label's template bits and the code index from its run (an M entry lies in a template label's run)
    uint32_t tu = 0, ci = 0;
    for (int l = 0; l < nruns; ++l)
      if (p - s_rlo[l] < s_rlen[l]) {
        tu = s_rtu[l];
        ci = p + s_rcd[l];
      }
    const uint32_t code = (tcode[ci >> 4] >> ((ci & 15u) << 1)) & 3u;
    if (!code) return 0;
    const uint32_t rest = tu & (tu - 1);
    if (rest & (rest - 1)) return tcur[p];
    return static_cast<uint16_t>(((code & 1u) ? (tu & (0u - tu)) : 0u) | ((code & 2u) ? rest : 0u));
  };
  BlockAcc acc;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t nS = *nSp;
  const uint64_t nchunks = (uint64_t(nS) + kWave - 1) / kWave;
  // the first LCC call (pub_state): a member's T_state equals its T_pub -- every superstep writes both, only the
  // NLC post-processing after the call clears T_pub bits alone -- and its alive count is the number of its alive
  // entries, which the walk counts: two of the five scattered state loads per row (T_state, |M| alive) are not
  // made (the second later superstep at S=28 is bound by random line fetches, ~5 per row)
  const bool derive = pub_state && !FIRST && !srec;
  // one chunk of 64 slist entries (live: the chunk's live mask, non-zero)
  auto chunk_body = [&](uint64_t chunk, uint64_t live) {
    const uint64_t i = chunk * kWave + lane;
    uint32_t u = kNone;
    uint16_t Tu = 0, nm = 0, Ts = 0;
    uint64_t beg = 0, pb = 0, pstart = ~0ull;  // pstart: a dense record's padded row start (k1_record)
    uint32_t len = 0, alive0 = 0;
    bool drow = false;  // M read from the dense superstep-0 region
    if (i < nS && ((live >> lane) & 1ull)) {
      // the row's state is loaded with T_pub in one round trip (a removed
      // row, T_pub = 0, ignores it)
      uint32_t l, dm = kNone;
      if (FIRST || srec) {  // dense superstep-0 output: the records, in slist order (coalesced)
        uint4 r;
        if (rs.rarea) {  // in place: the chunk's first slice, a later one for lanes past its end (rare)
          // (descriptors exist for the light records' chunks only: the heavy records after them are in srec)
          const uint64_t nl = rs.rofs[rs.W];
          if (i < nl) {
            const uint4 d = rs.cdesc[chunk];
            if (static_cast<uint32_t>(lane) < d.z) {
              r = rs.rarea[((uint64_t(d.y) << 32) | d.x) + lane];
            } else {
              uint32_t sl = d.w;
              while (i >= rs.rofs[sl + 1]) ++sl;
              r = rs.rarea[rs.rbase[sl] + (i - rs.rofs[sl])];
            }
          } else {
            r = srec[i];
          }
          slist_out[i] = r.x;  // (the list the compaction and the next supersteps read)
        } else {
          r = srec[i];
        }
        u = r.x;
        Tu = static_cast<uint16_t>(r.y);
        dm = r.z;
        l = dm != kNone ? (r.y >> 16) & 0x1FFu : mlen[u];
        if (dm != kNone && (r.y >> 25) < 127u) pstart = (uint64_t(r.y >> 25) << 32) | r.w;
      } else {
        u = slist[i];
        Tu = tcur[u];
        l = mlen[u];
      }
      // a dense superstep-0 row: T_state = T_pub, |M| = its length, and its padded row start is
      // needed only if it survives (one scattered load instead of six per row)
      uint64_t b = 0;
      uint32_t a0 = l;
      if (dm == kNone) {
        b = offp[u];
        // (timing variant diag 16: the same two loads dropped without the count: results wrong)
        a0 = derive ? 0u : (diag & 16) ? l : malive[u];
        Ts = derive || (diag & 16) ? Tu : tst[u];
      } else {
        Ts = Tu;
      }
      if (Tu) {
        drow = dm != kNone;
        pb = b;
        beg = drow ? dbase + dm : b;
        len = l;
        alive0 = a0;
        nm = nbr_mask(Tu, s_adj);
      } else {
        tnxt[u] = 0;
      }
    }
    // a row above kPullLong entries goes to the long-row list (its pieces: k_lcc_step_pieces, which also verifies
    // it and sets its live / keep bits); a full list leaves it to this wave.  (A dense superstep-0 row -- at most
    // 480 entries, moved to its padded row if it survives -- stays here whatever the threshold.)
    bool deferred = false;
    if (ll.rows && len > ll.min_len && !drow) {
      const uint32_t np = (len + kPullPiece - 1) / kPullPiece;
      const unsigned long long old = atomicAdd(ll.cnt, (1ull << 32) | np);
      const unsigned long long r = old >> 32, pb = old & 0xFFFFFFFFull;
      if (r < ll.cap) {
        LongRow lrow{};
        lrow.u = u;
        lrow.i = static_cast<uint32_t>(i);
        lrow.beg = beg;
        lrow.len = len;
        lrow.Ts = Ts;
        lrow.nm = nm;
        lrow.pbase = pb;
        ll.rows[r] = lrow;
        deferred = true;
        len = 0;
      }
    }
    uint32_t tn = 0, cnt = 0;
    uint32_t talive = 0;  // (derive) alive entries this lane walked: the superstep's traversed count
    bool asym = false;
    // short rows: flattened over the wave -- the chunk's rows are concatenated
    // and every lane takes every 64th entry (four in flight), so a chunk costs
    // ceil(entries / 256) rounds of two dependent loads instead of one round per
    // four entries of its longest row; per-row OR / count through LDS atomics
    const bool lng = len > kLprMax;
    const uint32_t ls = lng ? 0u : len;
    const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(ls));
    const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
    uint64_t dmask = 0;  // (FIRST) flattened dense rows: updates deferred to the row moves
    if constexpr (FIRST) {
      const bool dfr = drow && ls > 0 && !(diag & 4);
      dmask = __ballot(dfr);
      s_wofs[w][lane] = dfr ? incl - ls : ~0u;
    }
    if (total) {
      s_end[w][lane] = incl;
      s_beg[w][lane] = beg;
      s_nm[w][lane] = nm;
      s_tn[w][lane] = 0;
      s_cnt[w][lane] = 0;
      __builtin_amdgcn_wave_barrier();
      for (uint32_t t0 = 0; t0 < total; t0 += U * kWave) {
        uint32_t m[U];
        uint16_t tv[U];
        int rr[U];
        uint64_t e[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
          const uint32_t t = t0 + q * kWave + lane;
          m[q] = 0u;
          rr[q] = 0;
          e[q] = 0;
          if (t < total) {
            int lo = 0, hi = kWave - 1;  // row of entry t
            while (lo < hi) {
              const int mid = (lo + hi) >> 1;
              if (s_end[w][mid] > t) hi = mid; else lo = mid + 1;
            }
            rr[q] = lo;
            e[q] = s_beg[w][lo] + (t - (lo ? s_end[w][lo - 1] : 0u));
            m[q] = mcol[e[q]];
          }
        }
#pragma unroll
        for (int q = 0; q < U; ++q)
          tv[q] = (m[q] & kAlive) ? ((diag & 1) ? uint16_t(m[q] & 0x7Fu) : tpub_of(m[q] & kPosMask)) : uint16_t(0);
#pragma unroll
        for (int q = 0; q < U; ++q) {
          const bool dr = FIRST && ((dmask >> rr[q]) & 1ull) && t0 + q * kWave + lane < total;
          uint32_t cq = 0;
          if (m[q] & kAlive) {
            uint32_t tq = 0;
            ++talive;
            k2_entry(mcol, e[q], m[q], tv[q], s_nm[w][rr[q]], tq, cq, asym, !(diag & 4) && !dr);
            if (tq) atomicOr(&s_tn[w][rr[q]], tq);
            if (cq) atomicAdd(&s_cnt[w][rr[q]], cq);
          }
          if constexpr (FIRST) {  // (walk entries t0 + 64 q .. + 63: one word)
            const uint64_t av = __ballot(dr && cq != 0);
            if (dmask && lane == 0 && (t0 >> 6) + q < static_cast<uint32_t>(kAlvWords)) s_alv[w][(t0 >> 6) + q] = av;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      tn = s_tn[w][lane];
      cnt = s_cnt[w][lane];
      __builtin_amdgcn_wave_barrier();
    }
    // long rows: the whole wave walks each
    uint64_t lb = __ballot(lng);
    while (lb) {
      const int r = __ffsll(static_cast<long long>(lb)) - 1;
      lb &= lb - 1;
      const uint64_t br = (uint64_t(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(beg >> 32), r))) << 32) |
                          static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(beg), r));
      const uint32_t lr = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(len), r));
      const uint16_t nmr = static_cast<uint16_t>(__builtin_amdgcn_readlane(static_cast<int>(nm), r));
      uint32_t tnr = 0, cntr = 0;
      for (uint32_t j0 = 0; j0 < lr; j0 += 4 * kWave) {
        uint32_t m[4];
        uint16_t tv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t j = j0 + q * kWave + lane;
          m[q] = j < lr ? mcol[br + j] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) tv[q] = (m[q] & kAlive) ? tpub_of(m[q] & kPosMask) : uint16_t(0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (m[q] & kAlive) {
            ++talive;
            k2_entry(mcol, br + j0 + q * kWave + lane, m[q], tv[q], nmr, tnr, cntr, asym, !(diag & 4));
          }
      }
      tnr = wave_or32(tnr);
      cntr = static_cast<uint32_t>(wave_sum(cntr));
      if (lane == r) {
        tn = tnr;
        cnt = cntr;
      }
    }
    bool survivor = false, removed = false, cleared = false;
    uint32_t mv = 0;  // entries of this lane's dense survivor row to move to its padded row
    if (Tu && !deferred) {
      const uint16_t T = keep_bits(Ts, static_cast<uint16_t>(tn), s_adj);
      if (T) {
        survivor = true;
        // dead_state: a later superstep of this call rewrites T_state and |M| alive of its survivors and derives
        // them from T_pub and the walk until then (derive), so these stores are dead
        if (!dead_state) {
          tst[u] = T;
          malive[u] = cnt;
        }
        tnxt[u] = T;
        // dense M: the survivor's (updated) row moves to its padded row (below, flattened over the wave)
        if (drow) {
          pb = pstart != ~0ull ? pstart : offp[u];
          mv = len;
          mlen[u] = len;
        }
      } else {
        removed = true;
        cnt = 0;
        // dense superstep-0 records: both T_pub buffers of u are still clean (superstep 0 wrote u's
        // T_pub only into its record) and its state arrays were never written, so a removed row writes
        // nothing -- M[v] cleared (nonunique_ee.hpp:941-964) is its absence from every later list
        if (!(FIRST || srec) || !drow) {
          tnxt[u] = 0;
          malive[u] = 0;
        }
        // first later superstep: neighbours read u's T_pub through the 2-bit codes unless u's label has
        // more than two template vertices, so the buffer read now can be cleared at once and u leaves
        // the live list (otherwise it stays live one more superstep, which clears the other buffer)
        if (FIRST || tcode) {
          uint32_t tu = 0;
          for (int l = 0; l < nruns; ++l)
            if (u - s_rlo[l] < s_rlen[l]) tu = s_rtu[l];
          const uint32_t rest = tu & (tu - 1);
          if (!(rest & (rest - 1))) {
            if (!srec) tcur[u] = 0;  // (with records it was never written)
            cleared = true;
          }
        }
      }
    }
    // the dense survivors' rows, concatenated over the wave: every lane moves every 64th entry, four in flight
    // (a row per lane would wait out one load per entry)
    {
      if (diag & 2) mv = 0;  // (timing variant: no row moves)
      const uint32_t incl2 = static_cast<uint32_t>(wave_incl_scan(mv));
      const uint32_t total2 = static_cast<uint32_t>(__shfl(incl2, kWave - 1, kWave));
      if (total2) {
        __threadfence_block();  // the entry updates of other lanes before the copies read them
        s_end[w][lane] = incl2;
        s_beg[w][lane] = beg;
        s_dst[w][lane] = pb;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t t0 = 0; t0 < total2; t0 += 4 * kWave) {
          uint32_t x[4];
          uint64_t d[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t t = t0 + q * kWave + lane;
            d[q] = ~0ull;
            if (t < total2) {
              int lo = 0, hi = kWave - 1;
              while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_end[w][mid] > t) hi = mid; else lo = mid + 1;
              }
              const uint32_t j = t - (lo ? s_end[w][lo - 1] : 0u);
              x[q] = mcol[s_beg[w][lo] + j];
              d[q] = s_dst[w][lo] + j;
              if constexpr (FIRST) {  // a deferred row: its alive bits from the walk
                const uint32_t wo = s_wofs[w][lo];
                if (wo != ~0u) {
                  const uint32_t tw = wo + j;
                  x[q] = (x[q] & kPosMask) | (((s_alv[w][tw >> 6] >> (tw & 63u)) & 1ull) ? kAlive : 0u);
                }
              }
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (d[q] != ~0ull) mcol[d[q]] = x[q];
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    // live mask of the next superstep (S only shrinks); a vertex removed now
    // stays live one more superstep so that its 0 also reaches the other
    // T_pub buffer (it is dropped once it arrives with T_pub = 0)
    const uint64_t lm = __ballot(survivor || (removed && !cleared));
    if (lane == 0) mask_out[chunk] = lm;
    // keep_out: the survivors (T_pub just written != 0), the list compaction's keep mask
    const uint64_t km = __ballot(survivor);
    if (keep_out && lane == 0) keep_out[chunk] = km;
    acc.trav += derive ? talive : alive0;
    acc.removed |= removed;
    acc.asym |= asym;
    if (survivor) {
      if (oa.nranks <= 1) {
        acc.vs += 1;
        acc.es += cnt;
      } else {
        acc_owner(s_hist, oa, u, cnt);
      }
    }
  };
  if (FIRST || !mask_in) {
    // first later superstep (every entry live): one chunk per wave at a time
    for (uint64_t chunk = uint64_t(blockIdx.x) * kWpb + w; chunk < nchunks; chunk += uint64_t(gridDim.x) * kWpb)
      chunk_body(chunk, ~0ull);
  } else {
    // later: the wave's chunks stay strided over the grid (clustered live
    // chunks spread over waves), but each lane loads the live mask of one of
    // the wave's next 64 chunks, dead ones get their zero output mask in the
    // same pass, and the wave then works through the live ones
    const uint64_t W = uint64_t(gridDim.x) * kWpb;
    for (uint64_t k0 = uint64_t(blockIdx.x) * kWpb + w; k0 < nchunks; k0 += W * kWave) {
      const uint64_t ch = k0 + uint64_t(lane) * W;
      const uint64_t lm = ch < nchunks ? mask_in[ch] : 0ull;
      if (ch < nchunks && !lm) {
        mask_out[ch] = 0;
        if (keep_out) keep_out[ch] = 0;
      }
      uint64_t bal = __ballot(lm != 0);
      while (bal) {
        const int j = __ffsll(static_cast<long long>(bal)) - 1;
        bal &= bal - 1;
        const uint64_t live =
            (uint64_t(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(lm >> 32), j))) << 32) |
            static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(lm), j));
        chunk_body(k0 + uint64_t(j) * W, live);
      }
    }
  }
  flush_block(acc, oa, s_hist, s_red, pp);
}

// The deferred long rows of a pull superstep (k_lcc_step: rows above kPullLong entries), in kPullPiece-entry pieces:
// piece k of the list (rows in list order, row r's pieces numbered from its pbase) goes to wave k % W of the grid
// (its row found by a binary search over the rows' first pieces), four entries in flight per lane.  A piece updates
// its entries as the step kernel does (k2_entry), ORs its TN and adds its count into the row's words; the last
// piece of the row to finish (ticket) verifies it: T_state, T_pub, |M| alive and its live / keep bits (OR-ed into
// the masks the step kernel wrote without it), or its removal.  Packing (ll.scr): the piece's alive entries go to
// its scratch slice in order, their number to pcnt.
__global__ __launch_bounds__(kBlock) void k_lcc_step_pieces(LongList ll, uint16_t* tcur, uint16_t* __restrict__ tnxt,
                                                            uint16_t* __restrict__ tst, PatArgs pa, OwnerArgs oa,
                                                            uint32_t* __restrict__ mcol, uint32_t* __restrict__ malive,
                                                            Partials pp, const uint32_t* __restrict__ tcode,
                                                            LabelRuns lr, int has_srec,
                                                            unsigned long long* __restrict__ mask_out,
                                                            unsigned long long* __restrict__ keep_out,
                                                            int count_trav) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  __shared__ uint16_t s_adj[16];
  __shared__ uint32_t s_rlo[16], s_rlen[16], s_rtu[16], s_rcd[16];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  load_adj(s_adj, pa);
  if (threadIdx.x < 16) {
    const int l = threadIdx.x;
    s_rlo[l] = lr.lo[l];
    s_rlen[l] = l < lr.n ? lr.len[l] : 0u;
    s_rtu[l] = lr.tu[l];
    s_rcd[l] = lr.cd[l];
  }
  __syncthreads();
  const int nruns = lr.n;
  // neighbour T_pub as the step kernel reads it (2-bit codes right after superstep 0, else the T_pub array)
  auto tpub_of = [&](uint32_t p) -> uint16_t {
    if (!tcode) return tcur[p];
    uint32_t tu = 0, ci = 0;
    for (int l = 0; l < nruns; ++l)
      if (p - s_rlo[l] < s_rlen[l]) {
        tu = s_rtu[l];
        ci = p + s_rcd[l];
      }
    const uint32_t code = (tcode[ci >> 4] >> ((ci & 15u) << 1)) & 3u;
    if (!code) return 0;
    const uint32_t rest = tu & (tu - 1);
    if (rest & (rest - 1)) return tcur[p];
    return static_cast<uint16_t>(((code & 1u) ? (tu & (0u - tu)) : 0u) | ((code & 2u) ? rest : 0u));
  };
  BlockAcc acc;
  bool asym = false;
  const int lane = lane_id();
  const uint64_t W = uint64_t(gridDim.x) * kWpb;
  const uint64_t gw = uint64_t(blockIdx.x) * kWpb + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t nrows = static_cast<uint32_t>(min<unsigned long long>(*ll.cnt >> 32, ll.cap));
  const LongRow* rows = ll.rows;
  const uint64_t pend = nrows ? rows[nrows - 1].pbase + (rows[nrows - 1].len + kPullPiece - 1) / kPullPiece : 0;
  for (uint64_t k = gw; k < pend; k += W) {
    uint32_t lo = 0, hi = nrows - 1;  // the last row whose first piece is at or below k
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (rows[mid].pbase <= k) lo = mid; else hi = mid - 1;
    }
    LongRow* R = ll.rows + __builtin_amdgcn_readfirstlane(lo);
    const uint64_t beg = R->beg;
    const uint32_t len = R->len, np = (len + kPullPiece - 1) / kPullPiece;
    const uint32_t q = static_cast<uint32_t>(k - R->pbase);
    const uint16_t nm = R->nm;
    const uint32_t j0 = q * kPullPiece, j1 = min(len, j0 + kPullPiece);
    const bool pack = ll.scr && k < ll.scr_pieces;
    uint32_t* const out = pack ? ll.scr + k * kPullPiece : nullptr;
    uint32_t tn = 0, cnt = 0, kept = 0;
    for (uint32_t jb = j0; jb < j1; jb += 4 * kWave) {
      uint32_t m[4];
      uint16_t tv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t j = jb + t * kWave + lane;
        m[t] = j < j1 ? mcol[beg + j] : 0u;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) tv[t] = (m[t] & kAlive) ? tpub_of(m[t] & kPosMask) : uint16_t(0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint32_t c1 = 0;
        if (m[t] & kAlive) {
          if (count_trav) ++acc.trav;  // (the step kernel did not load the row's alive count)
          k2_entry(mcol, beg + jb + t * kWave + lane, m[t], tv[t], nm, tn, c1, asym);
        }
        cnt += c1;
        if (pack) {  // (entries stay in row order: component t covers jb + 64 t .. jb + 64 t + 63)
          const uint64_t b = __ballot(c1 != 0);
          if (c1) out[kept + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(b >> 32),
                                                       __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(b), 0u))] =
              (m[t] & kPosMask) | kAlive;
          kept += static_cast<uint32_t>(__builtin_popcountll(b));
        }
      }
    }
    tn = wave_or32(tn);
    cnt = static_cast<uint32_t>(wave_sum(cnt));
    if (lane == 0) {
      if (pack) ll.pcnt[k] = kept;
      if (tn) atomicOr(&R->tn, tn);
      if (cnt) atomicAdd(&R->cnt, cnt);
      __threadfence();
      if (atomicAdd(&R->done, 1u) == np - 1) {  // the row's last piece: verify it
        __threadfence();
        const uint16_t TN = static_cast<uint16_t>(atomicOr(&R->tn, 0u));
        const uint32_t CNT = atomicAdd(&R->cnt, 0u);
        const uint32_t u = R->u, i = R->i;
        const unsigned long long bit = 1ull << (i % kWave);
        const uint16_t T = keep_bits(R->Ts, TN, s_adj);
        R->T = T;
        if (T) {
          tst[u] = T;
          tnxt[u] = T;
          malive[u] = CNT;
          atomicOr(&mask_out[i / kWave], bit);
          if (keep_out) atomicOr(&keep_out[i / kWave], bit);
          if (oa.nranks <= 1) {
            acc.vs += 1;
            acc.es += CNT;
          } else {
            acc_owner(s_hist, oa, u, CNT);
          }
        } else {
          acc.removed = 1;
          tnxt[u] = 0;
          malive[u] = 0;
          // (as the step kernel: right after superstep 0 a label of at most two template vertices is read
          // through its codes, so the T_pub buffer read now is cleared at once and the row leaves the list)
          bool cleared = false;
          if (tcode) {
            uint32_t tu = 0;
            for (int l = 0; l < nruns; ++l)
              if (u - s_rlo[l] < s_rlen[l]) tu = s_rtu[l];
            const uint32_t rest = tu & (tu - 1);
            if (!(rest & (rest - 1))) {
              if (!has_srec) tcur[u] = 0;
              cleared = true;
            }
          }
          if (!cleared) atomicOr(&mask_out[i / kWave], bit);
        }
      }
    }
  }
  acc.asym |= asym;
  flush_block(acc, oa, s_hist, s_red, pp);
}

// Packing of the listed rows that survived the call's last pull superstep (their pieces all in the scratch): one
// block per row scans its pieces' counts and copies their alive entries to the row start, in order; mlen = |M|.
__global__ __launch_bounds__(kBlock) void k_long_pack(LongList ll, uint32_t* __restrict__ mcol,
                                                      uint32_t* __restrict__ mlen) {
  __shared__ uint32_t s_w[kWpb];
  __shared__ uint32_t s_carry;
  const uint32_t nrows = static_cast<uint32_t>(min<unsigned long long>(*ll.cnt >> 32, ll.cap));
  const int lane = lane_id(), w = threadIdx.x / kWave;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const LongRow& R = ll.rows[r];
    const uint32_t np = (R.len + kPullPiece - 1) / kPullPiece;
    if (!R.T || R.pbase + np > ll.scr_pieces) continue;  // (block-uniform) removed, or not all in the scratch
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t q0 = 0; q0 < np; q0 += blockDim.x) {
      const uint32_t q = q0 + threadIdx.x;
      const uint32_t c = q < np ? ll.pcnt[R.pbase + q] : 0u;
      const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(c));
      if (lane == kWave - 1) s_w[w] = incl;
      __syncthreads();
      uint32_t wpre = 0, tot = 0;
      for (int j = 0; j < kWpb; ++j) {
        wpre += j < w ? s_w[j] : 0u;
        tot += s_w[j];
      }
      const uint32_t base = s_carry;
      __syncthreads();
      if (threadIdx.x == 0) s_carry = base + tot;
      // this thread's piece: c entries from its scratch slice to the row at base + wpre + incl - c
      const uint32_t* src = ll.scr + (R.pbase + q) * uint64_t(kPullPiece);
      uint32_t* dst = mcol + R.beg + base + wpre + incl - c;
      for (uint32_t j = 0; j < c; ++j) dst[j] = src[j];
      __syncthreads();
    }
    if (threadIdx.x == 0) mlen[R.u] = s_carry;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// K2', push form of a later LCC superstep (directed inputs, and every LCC call
// after the first, where a cycle terminal's edge flag may have broken the
// symmetry of M; nonunique_ee.hpp:571-633 senders, :412-443 + :647-816
// receivers, :886-977 verify).  Two launches per superstep:
//   send:   every v of S (T_pub(v) != 0) delivers T_pub(v) to each alive u of
//           M[v]; a receiver u in S with a valid parent gets TN(u) |= T_pub(v)
//           (atomic OR, before the edge check, hazard 5) and, when v is in
//           M[u] (rows are in neighbour-id order: binary search), that entry's
//           flag is set;
//   verify: keep_bits(T_state, TN); survivors keep their flagged entries,
//           flags cleared; an emptied vertex leaves S.
// Rows are walked by one lane each (M rows are short after superstep 0).
__device__ __forceinline__ int64_t m_find(const uint32_t* __restrict__ mcol, uint64_t b, uint32_t len,
                                          const uint32_t* __restrict__ perm, uint32_t vid) {
  uint64_t lo = b, hi = b + len;
  while (lo < hi) {  // first entry whose neighbour id >= vid
    const uint64_t mid = (lo + hi) >> 1;
    if (perm[mcol[mid] & kPosMask] < vid) lo = mid + 1; else hi = mid;
  }
  return lo < b + len ? static_cast<int64_t>(lo) : -1;
}

// Entry-parallel: each wave takes 64 slist entries (rows); rows of at most kPushLong entries are walked
// flattened over the wave (every lane takes every 64th entry of their concatenation, four in flight), longer
// rows (R-MAT hubs: a lane walking a row of 10^5..10^6 entries, each with a binary search, took seconds) are
// cut into kPushLong-entry pieces appended to a list that every wave of a second launch works through.
static constexpr uint32_t kPushLong = 256;

struct PushArgs {
  const uint64_t* offp;
  const uint32_t* slist;
  const uint32_t* nS;
  const uint16_t* tcur;
  uint16_t* tnxt;
  uint16_t* tst;
  const uint32_t* perm;
  uint32_t* mcol;
  const uint32_t* mlen;
  uint32_t* malive;
  uint32_t* tn;
  unsigned long long* pieces;   // (slist index << 32 | piece) of the long rows
  unsigned long long* npieces;  // zeroed before the launches (the send and the verify have lists of their own)
  uint64_t piece_cap;
};

// Sender entry: v (id vid, T_pub Tv) delivers to the neighbour in entry m.
__device__ __forceinline__ void push_send_entry(const PushArgs& a, const uint16_t* s_adj, uint32_t v, uint32_t vid,
                                                uint16_t Tv, uint32_t m) {
  if (!(m & kAlive)) return;
  const uint32_t u = m & kPosMask;
  const uint16_t Tu = a.tcur[u];
  if (!Tu || !(Tv & nbr_mask(Tu, s_adj))) return;  // u not in S, or not a valid parent
  // (bits already present are not sent again: a hub's TN word takes one atomic per new bit instead of one per
  // neighbour, which serialised on the word)
  if ((a.tn[u] & Tv) != Tv) atomicOr(&a.tn[u], static_cast<uint32_t>(Tv));
  const int64_t e = m_find(a.mcol, a.offp[u], a.mlen[u], a.perm, vid);
  if (e >= 0) {
    const uint32_t x = a.mcol[e];
    if ((x & kPosMask) == v && (x & kAlive)) atomicOr(&a.mcol[e], kFlag);
  }
}

// Receiver-side verify of one entry of a surviving row: keep flagged entries (flags cleared); returns kept.
__device__ __forceinline__ uint32_t push_verify_entry(uint32_t* mcol, uint64_t e) {
  const uint32_t m = mcol[e];
  if (!(m & kAlive)) return 0u;
  const bool keep = (m & kFlag) != 0;
  mcol[e] = (m & kPosMask) | (keep ? kAlive : 0u);
  return keep ? 1u : 0u;
}

// Appends the pieces of a long row (slist index i, len entries); false when the list is full.
__device__ __forceinline__ bool push_pieces(const PushArgs& a, uint64_t i, uint32_t len) {
  const uint32_t np = (len + kPushLong - 1) / kPushLong;
  const unsigned long long b = atomicAdd(a.npieces, static_cast<unsigned long long>(np));
  if (b + np > a.piece_cap) {  // full: the reserved slots below the cap are marked empty
    for (uint64_t q = b; q < a.piece_cap && q < b + np; ++q) a.pieces[q] = ~0ull;
    return false;
  }
  for (uint32_t q = 0; q < np; ++q) a.pieces[b + q] = (static_cast<unsigned long long>(i) << 32) | q;
  return true;
}

// VERIFY = 0: the senders; 1: the receivers' verify (T from TN, survivors' entries compacted in place).
template <int VERIFY>
__global__ __launch_bounds__(kBlock) void k_lcc_push_rows(PushArgs a, PatArgs pa, OwnerArgs oa, Partials pp,
                                                         unsigned long long* __restrict__ trav_out) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  __shared__ uint16_t s_adj[16];
  __shared__ uint64_t s_beg[kWpb][kWave];
  __shared__ uint32_t s_end[kWpb][kWave], s_v[kWpb][kWave], s_vid[kWpb][kWave], s_cnt[kWpb][kWave];
  __shared__ uint16_t s_T[kWpb][kWave];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  load_adj(s_adj, pa);
  __syncthreads();
  BlockAcc acc;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t nS = *a.nS;
  const uint64_t nch = (nS + kWave - 1) / kWave;
  for (uint64_t ch = uint64_t(blockIdx.x) * kWpb + w; ch < nch; ch += uint64_t(gridDim.x) * kWpb) {
    const uint64_t i = ch * kWave + lane;
    uint32_t v = 0, vid = 0, len = 0;
    uint64_t beg = 0;
    uint16_t T = 0;
    bool lng = false;
    if (i < nS) {
      v = a.slist[i];
      const uint16_t Tv = a.tcur[v];
      if (!VERIFY) {
        if (Tv) {
          T = Tv;
          vid = a.perm[v];
          beg = a.offp[v];
          len = a.mlen[v];
          acc.trav += a.malive[v];
        }
      } else if (!Tv) {
        a.tnxt[v] = 0;
      } else {
        T = keep_bits(a.tst[v], static_cast<uint16_t>(a.tn[v]), s_adj);
        a.tn[v] = 0;
        if (!T) {
          a.tnxt[v] = 0;
          a.malive[v] = 0;
          acc.removed = 1;
        } else {
          a.tst[v] = T;
          a.tnxt[v] = T;
          beg = a.offp[v];
          len = a.mlen[v];
          if (oa.nranks <= 1) acc.vs += 1;
          else acc_owner(s_hist, oa, v, 0);  // (its edges are added where its entries are counted)
        }
      }
      if (len > kPushLong) {
        lng = push_pieces(a, i, len);
        if (lng) {
          if (VERIFY) a.malive[v] = 0;  // (the pieces add their kept entries)
          len = 0;
        }
      }
    }
    (void)lng;
    // the short rows flattened over the wave (a long row whose pieces did not fit stays here)
    const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(len));
    const uint32_t total = static_cast<uint32_t>(__shfl(incl, kWave - 1, kWave));
    if (!total) continue;
    s_end[w][lane] = incl;
    s_beg[w][lane] = beg;
    s_v[w][lane] = v;
    s_vid[w][lane] = vid;
    s_T[w][lane] = T;
    s_cnt[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t t0 = 0; t0 < total; t0 += 4 * kWave) {
      uint32_t m[4];
      int rr[4];
      uint64_t e[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t t = t0 + q * kWave + lane;
        rr[q] = -1;
        m[q] = 0;
        e[q] = 0;
        if (t < total) {
          int lo = 0, hi = kWave - 1;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_end[w][mid] > t) hi = mid; else lo = mid + 1;
          }
          rr[q] = lo;
          e[q] = s_beg[w][lo] + (t - (lo ? s_end[w][lo - 1] : 0u));
          m[q] = a.mcol[e[q]];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (rr[q] < 0) continue;
        if (!VERIFY) {
          push_send_entry(a, s_adj, s_v[w][rr[q]], s_vid[w][rr[q]], s_T[w][rr[q]], m[q]);
        } else if (m[q] & kAlive) {
          const bool keep = (m[q] & kFlag) != 0;
          a.mcol[e[q]] = (m[q] & kPosMask) | (keep ? kAlive : 0u);
          if (keep) atomicAdd(&s_cnt[w][rr[q]], 1u);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (VERIFY && len) {  // this lane's short row: its kept count
      const uint32_t cnt = s_cnt[w][lane];
      a.malive[v] = cnt;
      if (oa.nranks <= 1) acc.es += cnt;
      else atomicAdd(&s_hist[oa.nranks + owner_of(v, oa)], static_cast<unsigned long long>(cnt));
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!VERIFY) {
    block_atomic_add(trav_out, acc.trav);  // the superstep's traversed-entries word
  } else {
    flush_block(acc, oa, s_hist, s_red, pp);
  }
}

// The long rows' pieces (pieces [p0, *npieces) of the list): one wave per piece, four entries per lane.
template <int VERIFY>
__global__ __launch_bounds__(kBlock) void k_lcc_push_pieces(PushArgs a, PatArgs pa, OwnerArgs oa, Partials pp,
                                                           uint64_t p0) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  __shared__ uint16_t s_adj[16];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  load_adj(s_adj, pa);
  __syncthreads();
  BlockAcc acc;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t np = min<uint64_t>(*a.npieces, a.piece_cap);
  for (uint64_t k = p0 + uint64_t(blockIdx.x) * kWpb + w; k < np; k += uint64_t(gridDim.x) * kWpb) {
    const unsigned long long pc = a.pieces[k];
    if (pc == ~0ull) continue;  // (a slot of a row that did not fit)
    const uint32_t v = a.slist[pc >> 32];
    const uint32_t q = static_cast<uint32_t>(pc);
    const uint64_t b = a.offp[v] + uint64_t(q) * kPushLong;
    const uint32_t len = min(kPushLong, a.mlen[v] - q * kPushLong);
    uint32_t cnt = 0;
    const uint16_t Tv = VERIFY ? 0 : a.tcur[v];
    const uint32_t vid = VERIFY ? 0 : a.perm[v];
#pragma unroll
    for (int r = 0; r < static_cast<int>(kPushLong / kWave); ++r) {
      const uint32_t j = r * kWave + lane;
      if (j >= len) continue;
      if (!VERIFY) push_send_entry(a, s_adj, v, vid, Tv, a.mcol[b + j]);
      else cnt += push_verify_entry(a.mcol, b + j);
    }
    if (VERIFY) {
      cnt = static_cast<uint32_t>(wave_sum(cnt));
      if (lane == 0 && cnt) {
        atomicAdd(&a.malive[v], cnt);
        if (oa.nranks <= 1) acc.es += cnt;
        else atomicAdd(&s_hist[oa.nranks + owner_of(v, oa)], static_cast<unsigned long long>(cnt));
      }
    }
  }
  if (VERIFY) flush_block(acc, oa, s_hist, s_red, pp);
}

// Counts of the current state (after token-passing post-processing).
__global__ __launch_bounds__(kBlock) void k_count_state(const uint32_t* __restrict__ slist,
                                                        const uint32_t* __restrict__ nSp,
                                                        const uint16_t* __restrict__ tpub,
                                                        const uint32_t* __restrict__ malive, OwnerArgs oa,
                                                        Partials pp) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  BlockAcc acc;
  const uint32_t nS = *nSp;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nS + 0ull;
       i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = slist[i];
    if (!tpub[u]) continue;
    if (oa.nranks <= 1) {
      acc.vs += 1;
      acc.es += malive[u];
    } else {
      acc_owner(s_hist, oa, u, malive[u]);
    }
  }
  flush_block(acc, oa, s_hist, s_red, pp);
}

// ---------------------------------------------------------------------------
// launchers
static unsigned grid_for(uint64_t items, unsigned per_block, unsigned cap = 65535u) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

static OwnerArgs owner_args(const Ctx& c) {
  OwnerArgs oa;
  oa.hubs = c.d_hubs;
  oa.perm = c.d_perm;
  oa.nhubs = static_cast<uint32_t>(c.hubs_host.size());
  oa.nranks = c.nranks;
  return oa;
}

uint32_t slot_words(const Ctx& c) { return 2 * (c.nranks <= 1 ? 1 : c.nranks) + 6; }

static Partials partials(Ctx& c, uint64_t* d_slot) {
  return Partials{reinterpret_cast<unsigned long long*>(c.d_part), reinterpret_cast<unsigned long long*>(d_slot)};
}

// Counters are added into the (zeroed) slot by the kernels themselves.
static void reduce_into(Ctx&, unsigned, uint64_t*) {}

// Sorts the vertices by (label, degree, id) (two stable LSD radix passes:
// degree, then label) and writes the renumbered adjacency into dst.  Sharded
// (nshards > 1): by (label, degree class, owner, degree, id) -- two more
// passes (owner, class) between them -- so every (label, class) run of the
// tiling splits into one contiguous sub-run per shard while the label runs
// stay whole.  Keys use the global degrees (key_degrees); slots and copied rows
// the shard's own rows (held_degrees: other shards' rows are empty here).
__global__ void k_owner_keys(const uint32_t* __restrict__ ids, uint64_t n, uint32_t nshards,
                             uint32_t* __restrict__ key) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    key[i] = ids[i] % nshards;
}

// degree class: 0 for degree 0, 1 + light_kind for degree <= kLightMax,
// kHeavyKind + 1 above (monotone in the degree)
__host__ __device__ inline uint32_t degree_class(uint64_t d) {
  if (d == 0) return 0;
  if (d > kLightMax) return kHeavyKind + 1;
  return 1 + light_kind(d);
}

// hub_thr (sharded searches with delegates): a delegate's share is a heavy row on every shard
// whatever its length there, so every delegate sorts into the heavy class
__global__ void k_class_keys(const uint32_t* __restrict__ deg, const uint32_t* __restrict__ ids, uint64_t n,
                             uint64_t hub_thr, uint32_t* __restrict__ key) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = ids[i];
    const uint64_t d = deg[u];
    key[i] = d >= hub_thr ? kHeavyKind + 1 : degree_class(d);
  }
}

__global__ void k_gather_pos(const uint32_t* __restrict__ pos, const uint64_t* __restrict__ ids, uint64_t n,
                             uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = pos[ids[i]];
}

__global__ void k_patch_moff(const HubInfo* __restrict__ info, uint32_t nh, uint64_t* __restrict__ moff) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nh; j += gridDim.x * blockDim.x)
    if (info[j].moff != ~0ull) moff[info[j].pos] = info[j].moff;
}

// Scratch of one call: device allocations freed with the object.
namespace {
struct Scratch {
  std::vector<void*> ps;
  ~Scratch() {
    for (void* p : ps) (void)hipFree(p);
  }
  template <typename T>
  T* get(uint64_t n) {
    void* p = nullptr;
    PM_HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(n, 1) * sizeof(T)));
    ps.push_back(p);
    return static_cast<T*>(p);
  }
};
}  // namespace

void build_label_layout(Ctx& c, uint32_t* src_col, bool src_is_layout, uint32_t* dst) {
  const uint64_t n = c.n;
  if (n) {
    Scratch sc;
    const unsigned g = grid_for(n, kBlock, 8192);
    // the layout's inputs by vertex id, from the host: sort-key degrees, held-row lengths, labels
    const std::vector<uint32_t>& kd = c.key_degrees();
    const std::vector<uint32_t>& hd = c.held_degrees();
    auto* kdeg = sc.get<uint32_t>(n);
    PM_HIP_CHECK(hipMemcpyAsync(kdeg, kd.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
    uint32_t* hdeg = kdeg;
    if (&hd != &kd) {
      hdeg = sc.get<uint32_t>(n);
      PM_HIP_CHECK(hipMemcpyAsync(hdeg, hd.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
    }
    auto* labels = sc.get<uint64_t>(n);
    PM_HIP_CHECK(hipMemcpyAsync(labels, c.labels_host.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
    auto* src_start = sc.get<uint64_t>(n);
    rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> hw(hdeg, Widen());
    if (src_is_layout) {
      hipLaunchKernelGGL(k_row_starts_by_id, dim3(g), dim3(kBlock), 0, c.stream, c.d_offp, c.d_perm, n, src_start);
      hipLaunchKernelGGL(k_to_ids, dim3(grid_for(c.nq, kBlock, 65535)), dim3(kBlock), 0, c.stream, src_col, c.nq,
                         c.d_perm);
    }
    auto* dkey = sc.get<uint32_t>(n);
    auto* dkey2 = sc.get<uint32_t>(n);
    auto* ids = sc.get<uint32_t>(n);
    auto* ids2 = sc.get<uint32_t>(n);
    auto* lkey = sc.get<uint64_t>(n);
    // labels in position order: kept for selected-vertices lines only (their destination filter)
    if (c.any_sv && !c.d_labs) PM_HIP_CHECK(hipMalloc(&c.d_labs, n * sizeof(uint64_t)));
    uint64_t* labs = c.any_sv ? c.d_labs : sc.get<uint64_t>(n);
    hipLaunchKernelGGL(k_layout_keys, dim3(g), dim3(kBlock), 0, c.stream, kdeg, n, dkey, ids);
    size_t tmp = 0, tmp2 = 0, tmp3 = 0, tmp4 = 0;
    PM_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, dkey, dkey2, ids, ids2, size_t(n), 0, 32,
                                                    c.stream));
    PM_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp2, lkey, labs, ids2, c.d_perm, size_t(n),
                                                    0, 64, c.stream));
    PM_HIP_CHECK(rocprim::inclusive_scan(nullptr, tmp3, lkey, c.d_offp + 1, size_t(n), rocprim::plus<uint64_t>(),
                                         c.stream));
    PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, tmp4, hw, src_start, uint64_t(0), size_t(n),
                                         rocprim::plus<uint64_t>(), c.stream));
    tmp = std::max(std::max(tmp, tmp2), std::max(tmp3, tmp4));
    void* d_tmp = sc.get<char>(tmp);
    if (!src_is_layout) {  // the id-major input: held rows one after the other
      size_t t4 = tmp;
      PM_HIP_CHECK(rocprim::exclusive_scan(d_tmp, t4, hw, src_start, uint64_t(0), size_t(n),
                                           rocprim::plus<uint64_t>(), c.stream));
    }
    PM_HIP_CHECK(rocprim::radix_sort_pairs(d_tmp, tmp, dkey, dkey2, ids, ids2, size_t(n), 0, 32,
                                                    c.stream));
    if (c.nshards > 1) {
      int obits = 1;
      while ((1u << obits) < c.nshards) ++obits;
      hipLaunchKernelGGL(k_owner_keys, dim3(g), dim3(kBlock), 0, c.stream, ids2, n, c.nshards, dkey);
      PM_HIP_CHECK(rocprim::radix_sort_pairs(d_tmp, tmp, dkey, dkey2, ids2, ids, size_t(n), 0,
                                                      obits, c.stream));
      hipLaunchKernelGGL(k_class_keys, dim3(g), dim3(kBlock), 0, c.stream, kdeg, ids, n,
                         c.split_hubs ? c.hub_threshold : ~0ull, dkey);
      PM_HIP_CHECK(rocprim::radix_sort_pairs(d_tmp, tmp, dkey, dkey2, ids, ids2, size_t(n), 0, 6,
                                                      c.stream));
    }
    hipLaunchKernelGGL(k_gather_labels, dim3(g), dim3(kBlock), 0, c.stream, labels, ids2, n, lkey);
    PM_HIP_CHECK(rocprim::radix_sort_pairs(d_tmp, tmp, lkey, labs, ids2, c.d_perm, size_t(n), 0,
                                                    64, c.stream));
    hipLaunchKernelGGL(k_inverse_perm, dim3(g), dim3(kBlock), 0, c.stream, c.d_perm, n, c.d_pos);
    // label-major offsets of this shard's rows: padded (slots) and real (degree sums)
    auto* pdeg = lkey;  // reuse
    auto* rdeg = sc.get<uint64_t>(n);
    hipLaunchKernelGGL(k_perm_degrees, dim3(g), dim3(kBlock), 0, c.stream, hdeg, c.d_perm, n, pdeg, rdeg);
    size_t t3 = tmp;
    PM_HIP_CHECK(rocprim::inclusive_scan(d_tmp, t3, pdeg, c.d_offp + 1, size_t(n), rocprim::plus<uint64_t>(), c.stream));
    t3 = tmp;
    PM_HIP_CHECK(rocprim::inclusive_scan(d_tmp, t3, rdeg, c.d_offr + 1, size_t(n), rocprim::plus<uint64_t>(), c.stream));
    PM_HIP_CHECK(hipMemsetAsync(c.d_offp, 0, sizeof(uint64_t), c.stream));
    PM_HIP_CHECK(hipMemsetAsync(c.d_offr, 0, sizeof(uint64_t), c.stream));
    hipLaunchKernelGGL(k_copy_rows, dim3(grid_for(n, kWpb, 65535)), dim3(kBlock), 0, c.stream, src_col, src_start,
                       hdeg, c.d_offp, c.d_perm, c.d_pos, n, dst);
    PM_HIP_CHECK(hipGetLastError());
    c.perm_host.resize(n);
    PM_HIP_CHECK(hipMemcpyAsync(c.perm_host.data(), c.d_perm, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));  // (the scratch is freed on return)
  } else {
    PM_HIP_CHECK(hipMemsetAsync(c.d_offp, 0, sizeof(uint64_t), c.stream));
    PM_HIP_CHECK(hipMemsetAsync(c.d_offr, 0, sizeof(uint64_t), c.stream));
    c.perm_host.clear();
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  }
}

// Superstep-0 tiling for the current layout and pattern (host-side table).
void build_tiling(Ctx& c) {
  // distinct pattern labels and their template bits
  std::vector<uint64_t> labs;
  std::vector<uint16_t> tus;
  for (int t = 0; t < c.pa.K; ++t) {
    auto it = std::find(labs.begin(), labs.end(), c.pa.plabel[t]);
    if (it == labs.end()) {
      labs.push_back(c.pa.plabel[t]);
      tus.push_back(static_cast<uint16_t>(1u << t));
    } else {
      tus[it - labs.begin()] |= static_cast<uint16_t>(1u << t);
    }
  }
  const int nl = static_cast<int>(labs.size());
  // Run boundaries in the label-major order (host binary searches over
  // perm_host): B[0] = first position with the label, B[1 + k] = first with
  // light kind >= k (k < kHeavyKind), B[1 + kHeavyKind] = first with
  // degree > kLightMax, B[kLB - 1] = one past the label's last position.
  static constexpr int kLB = kHeavyKind + 3;
  const uint64_t n = c.n;
  auto lab_at = [&](uint64_t i) { return c.labels_host[c.perm_host[i]]; };
  auto cls_at = [&](uint64_t i) {
    const uint64_t d = c.row_degree(c.perm_host[i]);
    return c.split_hubs && d >= c.hub_threshold ? static_cast<uint32_t>(kHeavyKind + 1) : degree_class(d);
  };
  auto first_where = [](uint64_t lo, uint64_t hi, auto&& pred) {  // first i in [lo, hi) with pred(i)
    while (lo < hi) {
      const uint64_t m = (lo + hi) >> 1;
      if (pred(m)) hi = m; else lo = m + 1;
    }
    return lo;
  };
  std::vector<uint64_t> bounds(std::max(nl, 1) * kLB, 0);
  for (int l = 0; l < nl; ++l) {
    uint64_t* B = bounds.data() + l * kLB;
    const uint64_t L = labs[l];
    B[0] = first_where(0, n, [&](uint64_t i) { return lab_at(i) >= L; });
    B[kLB - 1] = first_where(B[0], n, [&](uint64_t i) { return lab_at(i) > L; });
    for (uint32_t k = 0; k <= static_cast<uint32_t>(kHeavyKind); ++k)
      B[1 + k] = first_where(B[0], B[kLB - 1], [&](uint64_t i) { return cls_at(i) >= 1 + k; });
  }
  // this shard's sub-run of [a, b) (positions are owner-sorted inside a run); the heavy run whole when
  // delegates are split (any shard may hold a delegate's share; other rows of the run are empty here)
  auto owned = [&](uint64_t a, uint64_t b, bool heavy) {
    if (c.nshards <= 1 || (heavy && c.split_hubs)) return std::make_pair(a, b);
    const uint32_t G = c.nshards, me = c.shard;
    const uint64_t x = first_where(a, b, [&](uint64_t i) { return c.perm_host[i] % G >= me; });
    const uint64_t y = first_where(x, b, [&](uint64_t i) { return c.perm_host[i] % G > me; });
    return std::make_pair(x, y);
  };
  auto dev_at = [&](const uint64_t* arr, uint64_t i) {
    uint64_t x = 0;
    PM_HIP_CHECK(hipMemcpy(&x, arr + i, sizeof(x), hipMemcpyDeviceToHost));
    return x;
  };
  c.lr = LabelRuns{};
  c.lr.n = nl;
  uint32_t cb = 0;
  for (int l = 0; l < nl; ++l) {
    c.lr.lo[l] = static_cast<uint32_t>(bounds[l * kLB + 0]);
    c.lr.len[l] = static_cast<uint32_t>(bounds[l * kLB + kLB - 1] - bounds[l * kLB + 0]);
    c.lr.tu[l] = tus[l];
    c.lr.cd[l] = cb - c.lr.lo[l];  // (mod 2^32)
    cb += c.lr.len[l];
  }
  c.lr.ncode = cb;
  if (std::getenv("PM_CODE_BY_POSITION")) {  // diagnostics: codes indexed by position (64 MB at S=28)
    for (int l = 0; l < nl; ++l) c.lr.cd[l] = 0;
    c.lr.ncode = static_cast<uint32_t>(c.n);
  }
  std::vector<KRange> tab;
  std::vector<HSeg> hs;
  std::vector<uint64_t> ttab;  // tile descriptors (kTtabRemShift / kTtabRangeShift)
  uint32_t tiles = 0, nheavy = 0;
  c.ss0_trav = 0;
  c.ss0_rows = 0;
  // delegates of a sharded search: positions, and the hub area of the ones this shard controls
  std::unordered_map<uint64_t, uint32_t> hub_at;  // position -> hub ordinal
  c.hubinfo.clear();
  if (c.split_hubs) {
    const uint64_t H = c.hubs_host.size();
    std::vector<uint32_t> hp(H);
    uint64_t* d_ids = nullptr;
    uint32_t* d_hp = nullptr;
    PM_HIP_CHECK(hipMalloc(&d_ids, H * sizeof(uint64_t)));
    PM_HIP_CHECK(hipMalloc(&d_hp, H * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMemcpy(d_ids, c.hubs_host.data(), H * sizeof(uint64_t), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gather_pos, dim3(grid_for(H, kBlock, 1024)), dim3(kBlock), 0, c.stream, c.d_pos, d_ids, H,
                       d_hp);
    PM_HIP_CHECK(hipMemcpyAsync(hp.data(), d_hp, H * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    (void)hipFree(d_ids);
    (void)hipFree(d_hp);
    uint64_t area = c.dbase + c.dcap;  // the hub area follows the dense region in mcol
    for (uint64_t j = 0; j < H; ++j) {
      HubInfo hi{hp[j], kNoHub, ~0ull};
      if (j % c.nshards == c.shard) {
        hi.moff = area;
        area += c.deg_host[c.hubs_host[j]];
      }
      c.hubinfo.push_back(hi);
      hub_at[hp[j]] = static_cast<uint32_t>(j);
    }
    if (area > c.dbase + c.dcap + c.hub_area) throw std::runtime_error("internal: hub area overflow");
  }
  for (int l = 0; l < nl; ++l) {
    const uint64_t* B = bounds.data() + l * kLB;
    const uint16_t tu = tus[l];
    uint16_t nm = 0;
    for (int t = 0; t < 16; ++t)
      if ((tu >> t) & 1u) nm |= c.pa.adj[t];
    const uint64_t first_nz = B[1], hi = B[kLB - 1];
    // every label-matching vertex sends along its out-edges: the scanned rows'
    // entries (other shards' rows are empty in offr); directed graphs scan
    // in-rows, so the senders' out-degrees are summed instead
    if (!c.symmetric)
      for (uint64_t i = B[0]; i < hi; ++i) c.ss0_trav += c.deg_host[c.perm_host[i]];
    if (hi <= first_nz) continue;
    if (c.symmetric) c.ss0_trav += dev_at(c.d_offr, hi) - dev_at(c.d_offr, first_nz);
    // kind k = [B[1+k], B[2+k]) for k < kHeavyKind (light class k); kHeavyKind = [B[1+kHeavyKind], hi)
    for (int kind = 0; kind <= kHeavyKind; ++kind) {
      const auto ab = owned(B[1 + kind], kind == kHeavyKind ? hi : B[2 + kind], kind == kHeavyKind);
      const uint64_t a = ab.first, b = ab.second;
      if (b <= a) continue;
      if (kind < kHeavyKind) c.ss0_rows += b - a;  // heavy rows: those with entries here (below)
      if (!nm) continue;  // such rows never enter S (TN = 0): scanned by no kernel, counted above
      KRange R{};
      R.tile0 = tiles;
      R.start = static_cast<uint32_t>(a);
      R.end = static_cast<uint32_t>(b);
      R.tu = tu;
      R.nm = nm;
      R.cdelta = c.lr.cd[l];
      R.kind = static_cast<uint32_t>(kind);
      if (kind < kHeavyKind) {
        R.g = kind_slots(static_cast<uint32_t>(kind));
        R.rpt = std::min<uint32_t>((kTileEntries - 4) / R.g, kTileRows);
        R.rdiv = ((1u << 19) + R.g - 1) / R.g;
        for (uint32_t sh = 0; sh < 4; ++sh)
          for (uint32_t sl = 0; sl < R.rpt * R.g; sl += R.g) {  // tile slot sl sits at load offset sl + sh
            const uint32_t o = sl + sh, k = o / 256, ln = (o % 256) / 4, cc = o % 4;
            R.rs[sh][4 * k + cc] |= 1ull << ln;
          }
      }
      R.qbase = dev_at(c.d_offp, a);
      R.nrel = 0;
      R.nadm = 0;
      R.nkeep = 0;
      for (int t = 0; t < 16; ++t) {
        if (!((tu >> t) & 1u)) continue;
        if (R.nkeep < 4) {
          R.kbit[R.nkeep] = static_cast<uint16_t>(1u << t);
          R.kneed[R.nkeep] = c.pa.adj[t] ? c.pa.adj[t] : (1u << 16);
        }
        ++R.nkeep;
      }
      for (int m = 0; m < nl; ++m) {
        if (!(tus[m] & nm) || c.lr.len[m] == 0) continue;
        if (R.nrel < 4) {
          R.rlo[R.nrel] = c.lr.lo[m];
          R.rlen[R.nrel] = c.lr.len[m];
          R.rtu[R.nrel] = tus[m];
        }
        ++R.nrel;
        if (R.nadm > 0 && R.nadm <= 4 && R.alo[R.nadm - 1] + R.alen[R.nadm - 1] == c.lr.lo[m]) {
          R.alen[R.nadm - 1] += c.lr.len[m];  // touches the previous relevant run
        } else {
          if (R.nadm < 4) {
            R.alo[R.nadm] = c.lr.lo[m];
            R.alen[R.nadm] = c.lr.len[m];
          }
          ++R.nadm;
        }
      }
      uint64_t nt;
      if (kind < kHeavyKind) {
        nt = (b - a + R.rpt - 1) / R.rpt;
      } else {
        R.aux = static_cast<uint32_t>(hs.size());
        std::vector<uint64_t> o(b - a + 1);
        PM_HIP_CHECK(hipMemcpy(o.data(), c.d_offp + a, o.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (uint64_t i = a; i < b; ++i) {
          const uint64_t deg = o[i - a + 1] - o[i - a];
          if (!deg) continue;  // (sharded: another shard's row)
          ++c.ss0_rows;
          const uint32_t ns = static_cast<uint32_t>((deg + kHeavyDeg - 1) / kHeavyDeg);
          auto hj = hub_at.find(i);
          const uint32_t split = hj != hub_at.end() ? 1u : 0u;
          if (split) c.hubinfo[hj->second].hidx = nheavy;
          for (uint32_t sgm = 0; sgm < ns; ++sgm) {
            const uint32_t tile = tiles + static_cast<uint32_t>(hs.size() - R.aux);
            hs.push_back(
                HSeg{static_cast<uint32_t>(i), sgm, nheavy, ns, static_cast<uint32_t>(tab.size()), tile, split});
          }
          ++nheavy;
        }
        nt = hs.size() - R.aux;
      }
      if (uint64_t(tiles) + nt >= 0xFFFFFFFFull - 2ull * kPartGridMax * kWpb * kTileBlock)
        throw std::runtime_error("superstep-0 tiling exceeds 2^32 tiles");
      const uint64_t rfield = uint64_t(tab.size()) << kTtabRangeShift;
      if (tab.size() >= (1u << (64 - kTtabRangeShift - 7))) throw std::runtime_error("internal: tile range index");
      for (uint64_t k = 0; k < nt; ++k) {
        if (kind >= kHeavyKind) {  // heavy segment tile: loads nothing in the light loop
          ttab.push_back(rfield);
          continue;
        }
        const uint64_t rows = std::min<uint64_t>(R.rpt, (b - a) - k * R.rpt);
        const uint64_t qb = R.qbase + k * R.rpt * R.g;
        if (qb >> kTtabRemShift) throw std::runtime_error("superstep-0 tile slot exceeds 2^36");
        ttab.push_back(qb | ((rows * R.g) << kTtabRemShift) | rfield);
      }
      tiles += static_cast<uint32_t>(nt);
      tab.push_back(R);
    }
  }
  if (c.comm) {
    std::vector<uint64_t> t = shard_allreduce(c, {c.ss0_trav});
    c.ss0_trav_all = t[0];
  } else {
    c.ss0_trav_all = c.ss0_trav;
  }
  if (tab.size() + 1 > static_cast<size_t>(kMaxRanges)) throw std::runtime_error("internal: too many tile ranges");
  KRange sent{};
  sent.tile0 = tiles;
  tab.push_back(sent);
  c.ktab = tab;
  c.k1_wide = false;
  for (const auto& R : tab)
    if (R.nrel > 4) c.k1_wide = true;
  c.ntiles = tiles;
  c.nheavy = nheavy;
  c.nhseg = static_cast<uint32_t>(hs.size());
  if (c.d_ktab) (void)hipFree(c.d_ktab);
  if (c.d_ttab) (void)hipFree(c.d_ttab);
  c.d_ttab = nullptr;
  if (c.d_hseg) (void)hipFree(c.d_hseg);
  if (c.d_hscr) (void)hipFree(c.d_hscr);
  if (c.d_tmask) (void)hipFree(c.d_tmask);
  if (c.d_tbase) (void)hipFree(c.d_tbase);
  if (c.d_tcnt) (void)hipFree(c.d_tcnt);
  if (c.d_tstart) (void)hipFree(c.d_tstart);
  c.d_tcnt = c.d_tstart = nullptr;
  if (c.d_scan_tmp) (void)hipFree(c.d_scan_tmp);
  c.d_ktab = nullptr;
  c.d_hseg = nullptr;
  c.d_hscr = nullptr;
  c.d_tmask = c.d_tbase = nullptr;
  c.d_scan_tmp = nullptr;
  PM_HIP_CHECK(hipMalloc(&c.d_ktab, tab.size() * sizeof(KRange)));
  PM_HIP_CHECK(hipMemcpy(c.d_ktab, tab.data(), tab.size() * sizeof(KRange), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMalloc(&c.d_ttab, std::max<size_t>(1, ttab.size()) * sizeof(uint64_t)));
  if (!ttab.empty())
    PM_HIP_CHECK(hipMemcpy(c.d_ttab, ttab.data(), ttab.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMalloc(&c.d_hseg, std::max<size_t>(1, hs.size()) * sizeof(HSeg)));
  if (!hs.empty()) PM_HIP_CHECK(hipMemcpy(c.d_hseg, hs.data(), hs.size() * sizeof(HSeg), hipMemcpyHostToDevice));
  PM_HIP_CHECK(hipMalloc(&c.d_hscr, std::max<size_t>(1, 3 * size_t(nheavy)) * sizeof(uint32_t)));
  c.tmask_words = std::max<uint64_t>(1, uint64_t(tiles) * kSub);
  PM_HIP_CHECK(hipMalloc(&c.d_tmask, c.tmask_words * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMalloc(&c.d_tbase, c.tmask_words * sizeof(uint64_t)));
  PM_HIP_CHECK(hipMalloc(&c.d_tcnt, std::max<size_t>(1, tiles) * sizeof(uint32_t)));
  PM_HIP_CHECK(hipMalloc(&c.d_tstart, std::max<size_t>(1, tiles) * sizeof(uint32_t)));
  c.scan_tmp_bytes = slist_scan_tmp_bytes(std::max<uint64_t>(1, tiles));
  PM_HIP_CHECK(hipMalloc(&c.d_scan_tmp, std::max<size_t>(1, c.scan_tmp_bytes)));
  c.k1_grid = lcc_first_grid(c);
  // record slices of the superstep-0 waves (dense mode): each wave's bound is the rows of the light tiles
  // it visits (tile t goes to wave (t / kTileBlock) % W of a persistent grid of W waves)
  {
    void* ptrs[] = {c.d_rarea, c.d_rbase, c.d_rcnt, c.d_rofs, c.d_hrec, c.d_srec, c.d_rscan_tmp, c.d_cdesc};
    for (void* q : ptrs)
      if (q) (void)hipFree(q);
    c.d_rarea = c.d_hrec = c.d_srec = nullptr;
    c.d_cdesc = nullptr;
    c.d_rbase = c.d_rofs = nullptr;
    c.d_rcnt = nullptr;
    c.d_rscan_tmp = nullptr;
    c.rwaves = 0;
    if (c.dcap && c.symmetric) {
      const uint32_t W = c.k1_grid * kWpb;
      std::vector<uint64_t> rows(W + 1, 0);
      for (size_t r = 0; r + 1 < tab.size(); ++r) {
        const KRange& R = tab[r];
        if (R.kind >= static_cast<uint32_t>(kHeavyKind)) continue;
        const uint64_t nrows = R.end - R.start, nt = (nrows + R.rpt - 1) / R.rpt;
        for (uint64_t k = 0; k < nt; ++k)
          rows[((R.tile0 + k) / kTileBlock) % W] += std::min<uint64_t>(R.rpt, nrows - k * R.rpt);
      }
      uint64_t tot = 0;
      for (uint32_t w = 0; w < W; ++w) {
        const uint64_t x = rows[w];
        rows[w] = tot;
        tot += x;
      }
      rows[W] = tot;
      c.rarea_cap = std::max<uint64_t>(tot, 1);
      c.srec_cap = tot + nheavy + c.hubinfo.size() + 1;
      PM_HIP_CHECK(hipMalloc(&c.d_rarea, c.rarea_cap * sizeof(uint4)));
      PM_HIP_CHECK(hipMalloc(&c.d_srec, c.srec_cap * sizeof(uint4)));
      PM_HIP_CHECK(hipMalloc(&c.d_rbase, (W + 1) * sizeof(uint64_t)));
      PM_HIP_CHECK(hipMalloc(&c.d_rcnt, std::max<uint32_t>(W, 1) * sizeof(uint32_t)));
      PM_HIP_CHECK(hipMalloc(&c.d_rofs, (W + 1) * sizeof(uint64_t)));
      PM_HIP_CHECK(hipMalloc(&c.d_hrec, std::max<uint64_t>(nheavy, 1) * sizeof(uint4)));
      PM_HIP_CHECK(hipMemcpy(c.d_rbase, rows.data(), (W + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
      rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> it(c.d_rcnt, Widen());
      PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, c.rscan_tmp_bytes, it, c.d_rofs, uint64_t(0), size_t(W),
                                           rocprim::plus<uint64_t>(), c.stream));
      PM_HIP_CHECK(hipMalloc(&c.d_rscan_tmp, std::max<size_t>(c.rscan_tmp_bytes, 1)));
      c.rwaves = W;
    }
  }
  if (c.d_hubinfo) (void)hipFree(c.d_hubinfo);
  if (c.d_moff) (void)hipFree(c.d_moff);
  if (c.d_hubpart) (void)hipFree(c.d_hubpart);
  c.d_hubinfo = nullptr;
  c.d_moff = nullptr;
  c.d_hubpart = nullptr;
  if (c.split_hubs) {
    const uint64_t H = c.hubinfo.size();
    PM_HIP_CHECK(hipMalloc(&c.d_hubinfo, H * sizeof(HubInfo)));
    PM_HIP_CHECK(hipMemcpy(c.d_hubinfo, c.hubinfo.data(), H * sizeof(HubInfo), hipMemcpyHostToDevice));
    PM_HIP_CHECK(hipMalloc(&c.d_hubpart, (uint64_t(c.nshards) + 1) * H * sizeof(uint64_t)));
    // M row starts until the replica: the layout's, with the controlled delegates in the hub area
    PM_HIP_CHECK(hipMalloc(&c.d_moff, (c.n + 1) * sizeof(uint64_t)));
    PM_HIP_CHECK(hipMemcpyAsync(c.d_moff, c.d_offp, (c.n + 1) * sizeof(uint64_t), hipMemcpyDeviceToDevice, c.stream));
    hipLaunchKernelGGL(k_patch_moff, dim3(grid_for(H, kBlock, 1024)), dim3(kBlock), 0, c.stream, c.d_hubinfo,
                       static_cast<uint32_t>(H), c.d_moff);
    PM_HIP_CHECK(hipGetLastError());
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  }
}

static K1Out k1_out(Ctx& c, unsigned grid) {
  // records: dense M on the grid the record slices were sized for
  const bool rec = c.k1_dense && c.d_rarea && grid * kWpb == c.rwaves;
  c.k1_records = rec;
  K1Out o{};
  o.tst = c.d_tst;
  o.tpub = c.d_tpub[c.cur];
  o.mcol = c.d_mcol;
  o.mlen = c.d_mlen;
  o.malive = c.d_malive;
  o.tcnt = c.d_tcnt;
  o.tstart = c.d_tstart;
  o.tcode = c.d_tcode;
  o.rarea = rec ? c.d_rarea : nullptr;
  o.rbase = c.d_rbase;
  o.rcnt = c.d_rcnt;
  o.hrec = rec ? c.d_hrec : nullptr;
  o.dbase = c.dbase;
  o.dslice = c.k1_dense ? c.dcap / (uint64_t(std::max(grid, 1u)) * kWpb) : 0;
  return o;
}

void launch_lcc_first_kernel(Ctx& c, int variant, unsigned grid, uint64_t* d_slot) {
  if (c.ntiles == 0) return;
  if (c.tcode_zpending) {  // (the codes' clear on rstream, side_clear_codes)
    PM_HIP_CHECK(hipStreamWaitEvent(c.stream, c.ev_tz, 0));
    c.tcode_zpending = false;
  }
  c.tcode_zeroed = false;  // (this launch writes them)
#define PM_K1_ARGS                                                                                                    \
  dim3(grid), dim3(kBlock), 0, c.stream, c.d_ktab, c.d_ttab, c.ntiles, c.d_hseg,                                                  \
      c.d_offp, c.d_colp, c.lr, c.pa, owner_args(c), k1_out(c, grid), c.d_hscr, c.nheavy, c.nhseg,                         \
      reinterpret_cast<unsigned long long*>(c.d_tmask), partials(c, d_slot)
  switch (variant) {
    case 0:
      if (c.k1_wide) hipLaunchKernelGGL((k_lcc_first<0, true>), PM_K1_ARGS);
      else hipLaunchKernelGGL(k_lcc_first<0>, PM_K1_ARGS);
      break;
#ifdef PM_DIAG_VARIANTS  // ablation builds of the kernel: lib/libpm_diag.so only (make diag; tools/k1_*.py)
    case 1: hipLaunchKernelGGL(k_lcc_first<1>, PM_K1_ARGS); break;
    case 2: hipLaunchKernelGGL(k_lcc_first<2>, PM_K1_ARGS); break;
    case 4: hipLaunchKernelGGL(k_lcc_first<4>, PM_K1_ARGS); break;
    case 8: hipLaunchKernelGGL(k_lcc_first<8>, PM_K1_ARGS); break;
    case 10: hipLaunchKernelGGL(k_lcc_first<10>, PM_K1_ARGS); break;
    case 12: hipLaunchKernelGGL(k_lcc_first<12>, PM_K1_ARGS); break;
    case 16: hipLaunchKernelGGL(k_lcc_first<16>, PM_K1_ARGS); break;
    case 32: hipLaunchKernelGGL(k_lcc_first<32>, PM_K1_ARGS); break;
    case 80: hipLaunchKernelGGL(k_lcc_first<80>, PM_K1_ARGS); break;
    case 128: hipLaunchKernelGGL(k_lcc_first<128>, PM_K1_ARGS); break;
    case 512: hipLaunchKernelGGL(k_lcc_first<512>, PM_K1_ARGS); break;
    case 1024: hipLaunchKernelGGL(k_lcc_first<1024>, PM_K1_ARGS); break;
    case 2048: hipLaunchKernelGGL(k_lcc_first<2048>, PM_K1_ARGS); break;
    case 4096: hipLaunchKernelGGL(k_lcc_first<4096>, PM_K1_ARGS); break;
    case 7168: hipLaunchKernelGGL(k_lcc_first<7168>, PM_K1_ARGS); break;
    case 5: hipLaunchKernelGGL((k_lcc_first<0, false, 5>), PM_K1_ARGS); break;  // 5 waves/SIMD, no spills
    // (variant numbers keep bit 1 clear: the timing harness reads it as "no dense M")
    case 13: hipLaunchKernelGGL((k_lcc_first<0, false, 6>), PM_K1_ARGS); break;      // 6 waves/SIMD
    case 17: hipLaunchKernelGGL((k_lcc_first<0, false, 8, 2>), PM_K1_ARGS); break;   // 2 tiles per wait
    case 21: hipLaunchKernelGGL((k_lcc_first<0, false, 6, 2>), PM_K1_ARGS); break;
    case 25: hipLaunchKernelGGL((k_lcc_first<0, false, 7, 2>), PM_K1_ARGS); break;
    case 29: hipLaunchKernelGGL((k_lcc_first<0, false, 5, 3>), PM_K1_ARGS); break;   // 3 tiles per wait
    case 33: hipLaunchKernelGGL((k_lcc_first<0, false, 4, 3>), PM_K1_ARGS); break;
    case 37: hipLaunchKernelGGL((k_lcc_first<0, false, 4, 4>), PM_K1_ARGS); break;   // 4 tiles per wait
#endif
    default: throw std::runtime_error("unknown superstep-0 kernel variant (ablation variants: lib/libpm_diag.so)");
  }
#undef PM_K1_ARGS
  PM_HIP_CHECK(hipGetLastError());
}

// Persistent grid: the resident blocks of the whole chip (occupancy query),
// never more waves than tiles.
unsigned lcc_first_grid(const Ctx& c) {
  int per_cu = 0;
  PM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lcc_first<0>, kBlock,
                                                           0));
  hipDeviceProp_t prop;
  PM_HIP_CHECK(hipGetDeviceProperties(&prop, c.device));
  uint64_t cap = std::min<uint64_t>(kPartGridMax, uint64_t(std::max(per_cu, 1)) * prop.multiProcessorCount);
  // (diagnostics: PM_K1_GRID sets the persistent grid -- the record slices follow it)
  if (const char* e = std::getenv("PM_K1_GRID")) cap = std::clamp<uint64_t>(std::strtoull(e, nullptr, 10), 1, kPartGridMax);
  return grid_for(c.ntiles, kWpb, static_cast<unsigned>(cap));
}

// Dense M when the next superstep is the pull-form k_lcc_step of this call
// (first call on a symmetric graph, diameter >= 2); PM_DENSE_M=0 disables it.
void lcc_first_set_dense(Ctx& c) {
  static const bool dense_env = !std::getenv("PM_DENSE_M") || std::string(std::getenv("PM_DENSE_M")) != "0";
  c.k1_dense = dense_env && c.dcap && c.symmetric && c.pattern.graph.diameter >= 2;
}

void lcc_first_prepare(Ctx& c) {
  if (c.nheavy) PM_HIP_CHECK(hipMemsetAsync(c.d_hscr, 0, 3 * size_t(c.nheavy) * sizeof(uint32_t), c.stream));
  if (c.nheavy && c.d_hrec) PM_HIP_CHECK(hipMemsetAsync(c.d_hrec, 0, size_t(c.nheavy) * sizeof(uint4), c.stream));
}

// slist from the superstep-0 records (dense mode): the records of the waves' slices, concatenated in wave
// order, copied to srec and their positions to slist; the heavy survivors follow (k_slist_heavy).  Every wave
// copies an equal share of the output (a multiple of 64 records), its first slice found by a binary search of
// the slice offsets: one wave per slice would wait for the largest slice.
__global__ void k_slist_from_records(const uint4* __restrict__ rarea, const uint64_t* __restrict__ rbase,
                                     const uint32_t* __restrict__ rcnt, const uint64_t* __restrict__ rofs,
                                     uint32_t W, uint4* __restrict__ srec, uint32_t* __restrict__ slist,
                                     uint32_t* __restrict__ nS) {
  const int lane = lane_id();
  const uint64_t total = rofs[W - 1] + rcnt[W - 1];
  if (blockIdx.x == 0 && threadIdx.x == 0) *nS = static_cast<uint32_t>(total);
  const uint64_t nw = uint64_t(gridDim.x) * kWpb;
  const uint64_t w = blockIdx.x * uint64_t(kWpb) + threadIdx.x / kWave;
  const uint64_t per = ((total + nw - 1) / nw + kWave - 1) / kWave * kWave;
  const uint64_t o0 = w * per, o1 = min(total, o0 + per);
  if (o0 >= o1) return;
  // the slice holding output o0: the last slice starting at or before it (empty slices share offsets)
  uint32_t lo = 0, hi = W - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (rofs[mid] <= o0) lo = mid;
    else hi = mid - 1;
  }
  uint32_t sl = lo;
  uint64_t send = sl + 1 < W ? rofs[sl + 1] : total;  // end of the lane's current slice
  for (uint64_t i = o0 + lane; i < o1; i += kWave) {
    while (i >= send) {
      ++sl;
      send = sl + 1 < W ? rofs[sl + 1] : total;
    }
    const uint4 r = rarea[rbase[sl] + (i - rofs[sl])];
    srec[i] = r;
    slist[i] = r.x;
  }
}

__global__ void k_slist_heavy(const uint4* __restrict__ hrec, uint32_t nheavy, const uint16_t* __restrict__ tst,
                              uint4* __restrict__ srec, uint32_t* __restrict__ slist, uint32_t* __restrict__ nS) {
  for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nheavy; h += gridDim.x * blockDim.x) {
    const uint4 r = hrec[h];
    if (!r.w) continue;
    const uint32_t i = atomicAdd(nS, 1u);
    srec[i] = make_uint4(r.x, tst[r.x], kNone, 0u);  // T_pub = T_state after superstep 0
    slist[i] = r.x;
  }
}

// Records in place (one context): the slice holding the first record of each 64-record chunk of the slices'
// concatenation, rofs[W] = the number of light records, and the list count (the heavy survivors are appended
// after them by k_slist_heavy).
// (rofs_in and rofs are the same array -- thread 0 writes rofs[W], which no thread reads -- so neither is
// declared __restrict__)
__global__ void k_chunk_slices(const uint64_t* rofs_in, const uint32_t* __restrict__ rcnt,
                               const uint64_t* __restrict__ rbase, uint32_t W, uint64_t* rofs,
                               uint4* __restrict__ cdesc, uint32_t* __restrict__ nS) {
  const uint64_t total = rofs_in[W - 1] + rcnt[W - 1];
  const uint64_t nch = (total + kWave - 1) / kWave;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rofs[W] = total;
    *nS = static_cast<uint32_t>(total);
  }
  for (uint64_t ch = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; ch < nch; ch += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t o0 = ch * kWave;
    uint32_t lo = 0, hi = W - 1;  // the last slice starting at or before o0 (empty slices share offsets)
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (rofs_in[mid] <= o0) lo = mid;
      else hi = mid - 1;
    }
    const uint64_t end = lo + 1 < W ? rofs_in[lo + 1] : total;  // (rofs[W] is being written by thread 0)
    const uint64_t b = rbase[lo] + (o0 - rofs_in[lo]);
    cdesc[ch] = make_uint4(static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32),
                           static_cast<uint32_t>(min<uint64_t>(kWave, end - o0)), lo + 1);
  }
}

// The same in one launch with the slices' scan (round 6: it replaces the library scan's two launches): every block
// scans the W <= 8192 slice counts in LDS (32 KB, read from L2), block 0 writes rofs[0..W] and the list count, and
// the blocks share the chunk descriptors.
static constexpr uint32_t kRsMaxW = 8192;
__global__ __launch_bounds__(kBlock) void k_record_slices(const uint32_t* __restrict__ rcnt,
                                                          const uint64_t* __restrict__ rbase, uint32_t W,
                                                          uint64_t* __restrict__ rofs, uint4* __restrict__ cdesc,
                                                          uint32_t* __restrict__ nS) {
  // (counts staged coalesced, one pad word per 32 so that a thread's 32 consecutive counts sit in distinct banks;
  // the offsets then overwrite them -- the block barrier of the scan lies between)
  __shared__ uint32_t s_buf[kRsMaxW + kRsMaxW / 32];
  uint32_t* const s_pad = s_buf;
  uint32_t* const s_ofs = s_buf;
  __shared__ uint32_t s_w[kWpb];
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  constexpr uint32_t per = kRsMaxW / kBlock;  // consecutive counts per thread
#pragma unroll
  for (uint32_t q = 0; q < per; ++q) {
    const uint32_t i = q * kBlock + tid;
    s_pad[i + i / 32] = i < W ? rcnt[i] : 0u;
  }
  __syncthreads();
  uint32_t v[per];
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t q = 0; q < per; ++q) {
    const uint32_t i = tid * per + q;
    v[q] = s_pad[i + i / 32];
    sum += v[q];
  }
  const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(sum));
  if (lane == kWave - 1) s_w[w] = incl;
  __syncthreads();
  uint32_t o = incl - sum;
  for (int j = 0; j < w; ++j) o += s_w[j];
#pragma unroll
  for (uint32_t q = 0; q < per; ++q) {
    s_ofs[tid * per + q] = o;
    o += v[q];
  }
  if (tid == kBlock - 1) s_ofs[kRsMaxW] = o;  // (the total: every count past W is 0)
  __syncthreads();
  const uint32_t total = s_ofs[kRsMaxW];
  if (blockIdx.x == 0) {
    for (uint32_t i = tid; i <= W; i += kBlock) rofs[i] = i < W ? s_ofs[i] : total;
    if (tid == 0) *nS = total;
  }
  const uint64_t nch = (uint64_t(total) + kWave - 1) / kWave;
  for (uint64_t ch = blockIdx.x * uint64_t(kBlock) + tid; ch < nch; ch += uint64_t(gridDim.x) * kBlock) {
    const uint32_t o0 = static_cast<uint32_t>(ch * kWave);
    uint32_t lo = 0, hi = W - 1;  // the last slice starting at or before o0 (empty slices share offsets)
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_ofs[mid] <= o0) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t end = lo + 1 < W ? s_ofs[lo + 1] : total;
    const uint64_t b = rbase[lo] + (o0 - s_ofs[lo]);
    cdesc[ch] = make_uint4(static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32), min(uint32_t(kWave), end - o0),
                           lo + 1);
  }
}

// heavy-row scratch, heavy records and the 2-bit codes of a superstep-0 launch (queued with the search's reset)
void queue_lcc_first_fills(Ctx& c) {
  if (c.ntiles == 0) return;
  if (c.nheavy) zero_later(c, c.d_hscr, 3 * size_t(c.nheavy) * sizeof(uint32_t));
  if (c.nheavy && c.d_hrec) zero_later(c, c.d_hrec, size_t(c.nheavy) * sizeof(uint4));
  if (!c.tcode_zeroed) zero_later(c, c.d_tcode, tcode_words(c.lr) * sizeof(uint32_t));
  c.k1_fills_queued = true;
}

// The codes' clear for the next search, on rstream after the first later superstep (their last reader) -- one
// context only (a sharded search exchanges codes in collectives on its stream).
void side_clear_codes(Ctx& c) {
  if (c.comm || c.ntiles == 0) return;
  if (!c.rstream) {
    PM_HIP_CHECK(hipStreamCreateWithFlags(&c.rstream, hipStreamNonBlocking));
    PM_HIP_CHECK(hipEventCreateWithFlags(&c.ev_rb, hipEventDisableTiming));
  }
  if (!c.ev_tz) {
    PM_HIP_CHECK(hipEventCreateWithFlags(&c.ev_tz0, hipEventDisableTiming));
    PM_HIP_CHECK(hipEventCreateWithFlags(&c.ev_tz, hipEventDisableTiming));
  }
  PM_HIP_CHECK(hipEventRecord(c.ev_tz0, c.stream));
  PM_HIP_CHECK(hipStreamWaitEvent(c.rstream, c.ev_tz0, 0));
  PM_HIP_CHECK(hipMemsetAsync(c.d_tcode, 0, tcode_words(c.lr) * sizeof(uint32_t), c.rstream));
  PM_HIP_CHECK(hipEventRecord(c.ev_tz, c.rstream));
  c.tcode_zeroed = true;
  c.tcode_zpending = true;
}

void launch_lcc_first(Ctx& c, uint64_t* d_slot, hipEvent_t ev0, hipEvent_t ev1) {
  if (c.ntiles == 0) {
    flush_zero(c);
    if (ev0) PM_HIP_CHECK(hipEventRecord(ev0, c.stream));
    if (ev1) PM_HIP_CHECK(hipEventRecord(ev1, c.stream));
    PM_HIP_CHECK(hipMemsetAsync(d_slot, 0, slot_words(c) * sizeof(uint64_t), c.stream));
    PM_HIP_CHECK(hipMemsetAsync(c.d_nS, 0, sizeof(uint32_t), c.stream));
    c.smask_valid = false;
    return;
  }
  const unsigned grid = c.k1_grid;
  if (!c.k1_fills_queued) queue_lcc_first_fills(c);
  flush_zero(c);
  c.k1_fills_queued = false;
  lcc_first_set_dense(c);
  c.slist_compacted = false;
  if (ev0) PM_HIP_CHECK(hipEventRecord(ev0, c.stream));
  launch_lcc_first_kernel(c, 0, grid, d_slot);
  if (ev1) PM_HIP_CHECK(hipEventRecord(ev1, c.stream));
  reduce_into(c, grid, d_slot);
  c.smask_valid = false;
  if (c.k1_records) {
    // slist = the records of the waves' slices (wave order), then the heavy survivors
    // the first later superstep reads the records in place (no copy); a sharded context whose labels need the
    // wide code exchange packs every survivor's T_pub from the records before that superstep, so it copies
    c.records_in_place = !c.comm || !c.xcode_wide;
    static const bool lib_scan = std::getenv("PM_RSCAN_LIB") && std::string(std::getenv("PM_RSCAN_LIB")) == "1";
    // (32-bit offsets: the records are light rows, fewer than 2^32)
    const bool one = c.records_in_place && c.rwaves <= kRsMaxW && c.rarea_cap < (1ull << 32) && !lib_scan;
    if (!one) {
      rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> rit(c.d_rcnt, Widen());
      size_t tb = c.rscan_tmp_bytes;
      PM_HIP_CHECK(rocprim::exclusive_scan(c.d_rscan_tmp, tb, rit, c.d_rofs, uint64_t(0), size_t(c.rwaves),
                                           rocprim::plus<uint64_t>(), c.stream));
    }
    if (c.records_in_place) {
      if (!c.d_cdesc) PM_HIP_CHECK(hipMalloc(&c.d_cdesc, (c.rarea_cap / kWave + 2) * sizeof(uint4)));
      if (one)  // (PM_RSCAN_LIB=1: the library scan and k_chunk_slices, A/B)
        hipLaunchKernelGGL(k_record_slices, dim3(grid_for(c.rarea_cap / kWave + 1, kBlock, 256)), dim3(kBlock), 0,
                           c.stream, c.d_rcnt, c.d_rbase, c.rwaves, c.d_rofs, c.d_cdesc, c.d_nS);
      else
        hipLaunchKernelGGL(k_chunk_slices, dim3(grid_for(c.rarea_cap / kWave + 1, kBlock, 1024)), dim3(kBlock), 0,
                           c.stream, c.d_rofs, c.d_rcnt, c.d_rbase, c.rwaves, c.d_rofs, c.d_cdesc, c.d_nS);
    } else {
      hipLaunchKernelGGL(k_slist_from_records, dim3(grid_for(c.rwaves, kWpb, 8192)), dim3(kBlock), 0, c.stream,
                         c.d_rarea, c.d_rbase, c.d_rcnt, c.d_rofs, c.rwaves, c.d_srec, c.d_slist, c.d_nS);
    }
    if (c.nheavy)
      hipLaunchKernelGGL(k_slist_heavy, dim3(grid_for(c.nheavy, kBlock, 1024)), dim3(kBlock), 0, c.stream, c.d_hrec,
                         c.nheavy, c.d_tst, c.d_srec, c.d_slist, c.d_nS);
    PM_HIP_CHECK(hipGetLastError());
    return;
  }
  // slist = survivors in label-major row order (tiles are in position order)
  rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> it(c.d_tcnt, Widen());
  size_t tmp = c.scan_tmp_bytes;
  PM_HIP_CHECK(rocprim::exclusive_scan(c.d_scan_tmp, tmp, it, c.d_tbase, uint64_t(0), size_t(c.ntiles), rocprim::plus<uint64_t>(), c.stream));
  c.smask_valid = false;
  hipLaunchKernelGGL(k_slist_write, dim3(grid_for(c.ntiles, kBlock, 8192)), dim3(kBlock), 0, c.stream, c.d_tcnt,
                     c.d_tstart, reinterpret_cast<const unsigned long long*>(c.d_tmask), c.d_tbase, c.ntiles, c.d_slist,
                     c.d_nS);
  PM_HIP_CHECK(hipGetLastError());
}

size_t slist_scan_tmp_bytes(uint64_t words) {
  rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> it(nullptr, Widen());
  size_t tmp = 0;
  PM_HIP_CHECK(rocprim::exclusive_scan(nullptr, tmp, it, static_cast<uint64_t*>(nullptr), uint64_t(0), size_t(std::max<uint64_t>(words, 1)), rocprim::plus<uint64_t>(), hipStream_t(0)));
  return tmp;
}

void launch_lcc_push(Ctx& c, uint64_t* d_slot) {
  if (!c.d_tn) {
    PM_HIP_CHECK(hipMalloc(&c.d_tn, c.n * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMemsetAsync(c.d_tn, 0, c.n * sizeof(uint32_t), c.stream));
  }
  // the long rows' piece lists of the send and of the verify (a row whose pieces do not fit is walked by its
  // own wave: slower, exact)
  const uint64_t want = 2 * uint64_t(c.nS_host) + 65536;
  if (c.push_cap < want) {
    if (c.d_push) (void)hipFree(c.d_push);
    c.d_push = nullptr;
    PM_HIP_CHECK(hipMalloc(&c.d_push, (2 * want + 2) * sizeof(unsigned long long)));
    c.push_cap = want;
  }
  const uint32_t P = c.nranks <= 1 ? 1 : c.nranks;
  PushArgs a{};
  a.offp = m_off(c);
  a.slist = c.d_slist;
  a.nS = c.d_nS;
  a.tcur = c.d_tpub[c.cur];
  a.tnxt = c.d_tpub[c.cur ^ 1];
  a.tst = c.d_tst;
  a.perm = c.d_perm;
  a.mcol = m_col(c);
  a.mlen = c.d_mlen;
  a.malive = c.d_malive;
  a.tn = c.d_tn;
  a.npieces = c.d_push;  // [0] the send's piece count, [1] the verify's
  a.pieces = c.d_push + 2;
  a.piece_cap = c.push_cap;
  PushArgs av = a;
  av.npieces = c.d_push + 1;
  av.pieces = c.d_push + 2 + c.push_cap;
  // no row of S longer than a piece (the last row compaction says so, c.push_long): no piece lists
  const bool pieces = c.push_long;
  if (pieces) PM_HIP_CHECK(hipMemsetAsync(c.d_push, 0, 2 * sizeof(unsigned long long), c.stream));
  // without the piece launches a long row must be walked by its own wave: no capacity, so push_pieces always
  // reports the list full (should the no-long-row stamp ever be wrong, the row is still sent and verified)
  if (!pieces) a.piece_cap = av.piece_cap = 0;
  const unsigned grid = grid_for((uint64_t(c.nS_host) + kWave - 1) / kWave, kWpb, 16384);
  auto* trav = reinterpret_cast<unsigned long long*>(d_slot + 2 * P);
  const OwnerArgs oa = owner_args(c);
  hipLaunchKernelGGL(k_lcc_push_rows<0>, dim3(grid), dim3(kBlock), 0, c.stream, a, c.pa, oa, partials(c, d_slot),
                     trav);
  if (pieces)
    hipLaunchKernelGGL(k_lcc_push_pieces<0>, dim3(kMaxGrid), dim3(kBlock), 0, c.stream, a, c.pa, oa,
                       partials(c, d_slot), uint64_t(0));
  hipLaunchKernelGGL(k_lcc_push_rows<1>, dim3(grid), dim3(kBlock), 0, c.stream, av, c.pa, oa, partials(c, d_slot),
                     trav);
  if (pieces)
    hipLaunchKernelGGL(k_lcc_push_pieces<1>, dim3(kMaxGrid), dim3(kBlock), 0, c.stream, av, c.pa, oa,
                       partials(c, d_slot), uint64_t(0));
  PM_HIP_CHECK(hipGetLastError());
  c.cur ^= 1;
  c.smask_valid = false;  // the pull kernel's live masks are not maintained here
}

void ensure_slist2(Ctx& c) {
  if (c.d_slist2) return;
  PM_HIP_CHECK(hipMalloc(&c.d_slist2, std::max<uint64_t>(c.n, 1) * sizeof(uint32_t)));
  PM_HIP_CHECK(hipMalloc(&c.d_nS2, 2 * sizeof(uint32_t)));  // [1]: long-row stamp (launch_compact_rows)
  PM_HIP_CHECK(hipMemset(c.d_nS2, 0, 2 * sizeof(uint32_t)));
}

static constexpr unsigned kLongGrid = 2048;  // blocks of the long rows' pieces launch (8192 waves)

void launch_lcc_step(Ctx& c, uint64_t* d_slot, bool first_after_ss0, bool last_of_call, bool pub_state) {
  if (!c.d_kmask) PM_HIP_CHECK(hipMalloc(&c.d_kmask, ((c.n + 63) / 64 + 1) * sizeof(uint64_t)));
  const uint64_t chunks = (uint64_t(c.nS_host) + kWave - 1) / kWave;
  // first later superstep (every slist entry live): one chunk per wave, the
  // latency-bound rows need waves in flight; afterwards few chunks are live
  // and a persistent-style grid skips the dead ones cheaply
  // (a compacted list is short: its all-live pass needs no more than a few waves per CU)
  const unsigned grid = grid_for(chunks, kWpb, c.smask_valid ? kMaxGrid : c.slist_compacted ? 2048 : 16384);
  const unsigned long long* min = c.smask_valid ? reinterpret_cast<const unsigned long long*>(c.d_smask[c.smask_cur])
                                                : nullptr;
  auto* mout = reinterpret_cast<unsigned long long*>(c.d_smask[c.smask_cur ^ 1]);
  RecSrc rs{};
  if (first_after_ss0 && c.k1_records && c.records_in_place)
    rs = RecSrc{c.d_rarea, c.d_rbase, c.d_rofs, c.d_cdesc, c.rwaves};
  // short rows: the previous search's mean |M| of this superstep's rows (the survivors of the one before;
  // the first search guesses long)
  const double mpr = c.cur_ss > 0 && c.cur_ss - 1 < c.m_per_row.size() ? c.m_per_row[c.cur_ss - 1] : 0.0;
  const bool short_rows = mpr > 0 && mpr <= 4.0;
  auto kern = short_rows ? k_lcc_step<3> : k_lcc_step<4>;
  // records and codes: the specialised instantiation (no spills at 6 waves per SIMD; budgets for 7 / 8 waves
  // spilled 13 / 31 VGPRs and ran 516-525 / 616-620 us against 513)
  if (first_after_ss0 && c.k1_records && c.d_srec) kern = short_rows ? k_lcc_step<3, true> : k_lcc_step<4, true>;
  // long rows in pieces (a second launch) where the previous search of this layout deferred some, or while that
  // is not known; the counter is the slot's word 2P + 4 (zeroed with the slots).  The call's last pull superstep
  // also packs them (k_long_pack) when the row compaction follows it.
  LongList ll{};
  const uint32_t P = c.nranks <= 1 ? 1 : c.nranks;
  const bool longs = !c.long_seen_off && (c.cur_ss >= c.long_seen.size() || c.long_seen[c.cur_ss]);
  const bool pack = longs && last_of_call && !c.no_row_compaction;
  if (longs) {
    if (!c.d_lrows) {
      c.lrows_cap = 1u << 16;
      PM_HIP_CHECK(hipMalloc(&c.d_lrows, uint64_t(c.lrows_cap) * sizeof(LongRow)));
    }
    ll = LongList{static_cast<LongRow*>(c.d_lrows), reinterpret_cast<unsigned long long*>(d_slot + 2 * P + 4),
                  c.lrows_cap, c.pull_long ? c.pull_long : kPullLong, nullptr, nullptr, 0};
    if (pack) {
      if (!c.d_lscr) {
        const uint64_t pieces =  // (PM_PACK_PIECES: tests; read per context)
            std::getenv("PM_PACK_PIECES") ? std::strtoull(std::getenv("PM_PACK_PIECES"), nullptr, 10) : (1u << 15);
        c.lscr_pieces = std::max<uint64_t>(pieces, 1);
        PM_HIP_CHECK(hipMalloc(&c.d_lscr, c.lscr_pieces * (kPullPiece + 1) * sizeof(uint32_t)));
      }
      ll.scr = static_cast<uint32_t*>(c.d_lscr);
      ll.pcnt = ll.scr + c.lscr_pieces * kPullPiece;
      ll.scr_pieces = c.lscr_pieces;
    }
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, c.stream, m_off(c), c.d_slist, c.d_nS, min, mout,
                     c.d_tpub[c.cur], c.d_tpub[c.cur ^ 1], c.d_tst, c.pa, owner_args(c), m_col(c), c.d_mlen,
                     c.d_malive, partials(c, d_slot), first_after_ss0 ? c.d_tcode : nullptr, c.lr,
                     c.diag_step, first_after_ss0 && c.k1_records ? c.d_srec : nullptr, c.dbase,
                     reinterpret_cast<unsigned long long*>(c.d_kmask), rs, c.d_slist, ll, pub_state ? 1 : 0,
                     pub_state && !last_of_call && !c.comm ? 1 : 0);
  PM_HIP_CHECK(hipGetLastError());
  if (longs) {
    hipLaunchKernelGGL(k_lcc_step_pieces, dim3(kLongGrid), dim3(kBlock), 0, c.stream, ll, c.d_tpub[c.cur],
                       c.d_tpub[c.cur ^ 1], c.d_tst, c.pa, owner_args(c), m_col(c), c.d_malive,
                       partials(c, d_slot), first_after_ss0 ? c.d_tcode : nullptr, c.lr,
                       first_after_ss0 && c.k1_records && c.d_srec ? 1 : 0, mout,
                       reinterpret_cast<unsigned long long*>(c.d_kmask),
                       pub_state && !(first_after_ss0 && c.k1_records && c.d_srec) ? 1 : 0);
    PM_HIP_CHECK(hipGetLastError());
    if (pack) {
      hipLaunchKernelGGL(k_long_pack, dim3(256), dim3(kBlock), 0, c.stream, ll, m_col(c), c.d_mlen);
      PM_HIP_CHECK(hipGetLastError());
    }
  }
  c.removed_cleared = first_after_ss0 && c.k1_records;  // (its removed rows cleared the T_pub they read)
  c.k1_dense = false;  // every M row of S is in its padded row from here on
  c.k1_records = false;
  reduce_into(c, grid, d_slot);
  c.cur ^= 1;
  c.smask_cur ^= 1;
  c.smask_valid = true;
}

// slist compaction after a later superstep: an entry stays iff it is live in
// the superstep's mask AND still in S (T_pub just written != 0); a live entry
// whose T_pub became 0 was removed by that superstep: the T_pub buffer that
// superstep read is cleared here (the other one holds its 0 already), so it
// need not stay live one more superstep.  One wave per 64-entry chunk: the
// keep ballot is the chunk's keep mask; then (after an exclusive scan of the
// chunk counts) the kept entries in their order, and the new count.
__global__ void k_live_keep(const uint32_t* __restrict__ slist, const unsigned long long* __restrict__ mask,
                            const uint32_t* __restrict__ nSp, uint64_t cap, const uint16_t* __restrict__ tnew,
                            uint16_t* __restrict__ told, unsigned long long* __restrict__ kmask,
                            uint32_t* __restrict__ cnt) {
  const uint64_t nS = *nSp;
  const int lane = lane_id();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;  // a multiple of kWave: a wave stays on one chunk
  // chunks of the device count only (cap: host upper bound; the scan reads counts below nch alone)
  const uint64_t end = min(cap, (nS + kWave - 1) / kWave) * kWave;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < end; i += stride) {
    const uint64_t c = i / kWave;
    bool keep = false;
    if (i < nS && ((mask[c] >> lane) & 1ull)) {
      const uint32_t u = slist[i];
      keep = tnew[u] != 0;
      if (!keep) told[u] = 0;
    }
    const uint64_t b = __ballot(keep);
    if (lane == 0) {
      kmask[c] = b;
      cnt[c] = static_cast<uint32_t>(__builtin_popcountll(b));
    }
  }
}

// The same from the superstep's own keep mask (k_lcc_step keep_out): no T_pub gather; the slist entries are
// read only for live entries that were not kept (removed now: the buffer the superstep read is cleared).
// One lane per chunk.
// PER_ENTRY: one thread per entry (the removed entries of a chunk cleared in parallel: after the second later
// superstep almost every entry goes); else one thread per chunk (after the first, whose removed rows cleared their
// T_pub themselves: few entries go, and a thread per entry would only read the masks).
template <bool PER_ENTRY>
__global__ void k_live_keep_masks(const uint32_t* __restrict__ slist, const unsigned long long* __restrict__ mask,
                                  const unsigned long long* __restrict__ keep, const uint32_t* __restrict__ nSp,
                                  uint64_t cap, uint16_t* __restrict__ told, uint32_t* __restrict__ cnt) {
  const uint64_t nch = min(cap, (static_cast<uint64_t>(*nSp) + kWave - 1) / kWave);
  const uint64_t n = PER_ENTRY ? nch * kWave : nch;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    if (PER_ENTRY) {
      const uint64_t c = i / kWave;
      const uint32_t b = static_cast<uint32_t>(i % kWave);
      const unsigned long long k = keep[c];
      if (b == 0) cnt[c] = static_cast<uint32_t>(__builtin_popcountll(k));
      if (((mask[c] & ~k) >> b) & 1ull) told[slist[i]] = 0;
    } else {
      const unsigned long long k = keep[i];
      cnt[i] = static_cast<uint32_t>(__builtin_popcountll(k));
      unsigned long long gone = mask[i] & ~k;
      while (gone) {
        const int b = __builtin_ctzll(gone);
        gone &= gone - 1;
        told[slist[i * kWave + b]] = 0;
      }
    }
  }
}

// Exclusive scan of the kept counts cnt[0, n) into base, n = the device's chunk count (ceil(*nSp / 64)); the host
// holds only a bound (the list length before the superstep is not read back), and a library scan over the bound
// cost 17-31 us at S=28 where the list had 153 k / 12.5 k chunks.  kScanBlocks blocks: block sums, then every
// block scans its range from the sum of the blocks before it.
static constexpr unsigned kScanBlocks = 256;
__global__ __launch_bounds__(kBlock) void k_chunk_scan_sums(const uint32_t* __restrict__ cnt,
                                                            const uint32_t* __restrict__ nSp,
                                                            uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s_w[kWpb];
  const uint64_t n = (static_cast<uint64_t>(*nSp) + kWave - 1) / kWave;
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = min(n, uint64_t(blockIdx.x) * per), hi = min(n, lo + per);
  uint64_t x = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) x += cnt[i];
  x = wave_sum(x);
  if (lane_id() == 0) s_w[threadIdx.x / kWave] = static_cast<uint32_t>(x);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int j = 0; j < kWpb; ++j) t += s_w[j];
    bsum[blockIdx.x] = t;
  }
}
__global__ __launch_bounds__(kBlock) void k_chunk_scan_write(const uint32_t* __restrict__ cnt,
                                                             const uint32_t* __restrict__ nSp,
                                                             const uint32_t* __restrict__ bsum,
                                                             uint32_t* __restrict__ base) {
  __shared__ uint32_t s_w[kWpb];
  const int w = threadIdx.x / kWave;
  const uint64_t n = (static_cast<uint64_t>(*nSp) + kWave - 1) / kWave;
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = min(n, uint64_t(blockIdx.x) * per), hi = min(n, lo + per);
  if (lo >= hi) return;  // (block-uniform)
  uint64_t o = 0;
  for (uint32_t j = threadIdx.x; j < blockIdx.x; j += blockDim.x) o += bsum[j];
  o = wave_sum(o);
  if (lane_id() == 0) s_w[w] = static_cast<uint32_t>(o);
  __syncthreads();
  uint32_t carry = 0;
  for (int j = 0; j < kWpb; ++j) carry += s_w[j];
  __syncthreads();
  for (uint64_t t0 = lo; t0 < hi; t0 += blockDim.x) {
    const uint64_t i = t0 + threadIdx.x;
    const uint32_t v = i < hi ? cnt[i] : 0u;
    const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(v));
    if (lane_id() == kWave - 1) s_w[w] = incl;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (int j = 0; j < kWpb; ++j) {
      wpre += j < w ? s_w[j] : 0u;
      tot += s_w[j];
    }
    if (i < hi) base[i] = carry + wpre + incl - v;
    carry += tot;
    __syncthreads();
  }
}

__global__ void k_live_write(const uint32_t* __restrict__ slist, const unsigned long long* __restrict__ kmask,
                             const uint32_t* __restrict__ nSp, const uint32_t* __restrict__ cnt,
                             const uint32_t* __restrict__ base, uint32_t* __restrict__ out,
                             uint32_t* __restrict__ nS_out) {
  const uint64_t nS = *nSp;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nS; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t c = i / kWave;
    const uint32_t b = static_cast<uint32_t>(i % kWave);
    const unsigned long long m = kmask[c];
    if ((m >> b) & 1ull) out[base[c] + __builtin_popcountll(m & ((1ull << b) - 1))] = slist[i];
    if (i == nS - 1) *nS_out = base[c] + cnt[c];
  }
  if (nS == 0 && blockIdx.x == 0 && threadIdx.x == 0) *nS_out = 0;
}

// List compaction in two launches (round 6; the four above: keep counts, the two scan passes, the write).
// k_compact_scan: tile b = chunks [256 b, 256 b + 256): their kept counts and block scan, the tile's offset in the
// new list by a decoupled look-back over the tiles before it, each chunk's first kept slot (cbase) and, after the
// first later superstep, the T_pub clears of its few removed entries.  Status word of a tile: epoch << 40 | flag << 38
// | value (flag 1: the tile's own count, 2: its inclusive offset); the epoch (the launch's number, never 0) tells a
// word of this launch from an older one, so the words are never cleared.  (A block ticket taken with one atomic per
// block -- the usual way to order the look-back -- cost 60 us for 600 blocks: same-address atomics serialise; the
// grid is a cooperative launch instead, every block resident, each walking its tiles in increasing order.)
// k_compact_write: the kept entries to the new list (and, PER_ENTRY, the clears of the removed ones) with every CU
// busy: a wave takes 16 chunks and requests their 16 entries per lane before any store.  (One launch doing both ran
// 83-86 us per compaction at S=28: 49-600 blocks walking their entries could not keep the memory system busy.)
static constexpr uint32_t kClEpochBits = 24;
__device__ __forceinline__ unsigned long long cl_word(uint64_t epoch, uint32_t flag, uint64_t v) {
  return (epoch << 40) | (uint64_t(flag) << 38) | v;
}
template <bool PER_ENTRY>
__global__ __launch_bounds__(kBlock) void k_compact_scan(const uint32_t* __restrict__ slist,
                                                         const unsigned long long* __restrict__ mask,
                                                         const unsigned long long* __restrict__ keep,
                                                         const uint32_t* __restrict__ nSp, uint64_t cap,
                                                         uint16_t* __restrict__ told, uint32_t* __restrict__ cbase,
                                                         uint32_t* __restrict__ nS_out, unsigned long long* status,
                                                         uint64_t epoch) {
  __shared__ uint32_t s_w[kWpb];
  __shared__ uint64_t s_base;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const uint64_t nch = min(cap, (static_cast<uint64_t>(*nSp) + kWave - 1) / kWave);
  const uint64_t nblk = (nch + kBlock - 1) / kBlock;
  if (nch == 0 && blockIdx.x == 0 && tid == 0) *nS_out = 0;
  // tiles of 256 chunks in increasing order per block; the grid is co-resident (cooperative launch), so the tile a
  // look-back waits for is always being worked on
  for (uint64_t bid = blockIdx.x; bid < nblk; bid += gridDim.x) {
    const uint64_t c = bid * kBlock + tid;
    unsigned long long k = 0, g = 0;
    if (c < nch) {  // (mask and keep bits of entries past the list's end are 0)
      k = keep[c];
      g = mask[c] & ~k;
    }
    const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(k));
    const uint32_t incl = static_cast<uint32_t>(wave_incl_scan(cnt));
    if (lane == kWave - 1) s_w[w] = incl;
    __syncthreads();
    uint32_t wpre = 0, agg = 0;
    for (int j = 0; j < kWpb; ++j) {
      wpre += j < w ? s_w[j] : 0u;
      agg += s_w[j];
    }
    if (w == 0) {  // look-back: 64 tiles per poll, back to the nearest one whose inclusive offset is out
      uint64_t excl = 0;
      if (bid > 0) {
        if (lane == 0)
          __hip_atomic_store(&status[bid], cl_word(epoch, 1, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t top = int64_t(bid) - 1;
        for (;;) {
          const int64_t j = top - lane;
          const unsigned long long sw =
              j >= 0 ? __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : cl_word(epoch, 2, 0);
          const uint32_t fl = static_cast<uint32_t>(sw >> 38) & 3u;
          const bool ready = (sw >> 40) == epoch && fl != 0;
          const uint64_t pm = __ballot(ready && fl == 2);
          const uint64_t rm = __ballot(ready);
          const int fp = pm ? __builtin_ctzll(pm) : kWave;  // nearest tile with its offset out
          const uint64_t need = fp >= kWave - 1 ? ~0ull : ((2ull << fp) - 1ull);
          if ((rm & need) != need) {
            __builtin_amdgcn_s_sleep(1);
            continue;  // a tile up to there has not published yet
          }
          excl += wave_sum(lane <= fp ? (sw & ((1ull << 38) - 1ull)) : 0ull);
          if (fp < kWave) break;
          top -= kWave;
        }
      }
      if (lane == 0) {
        __hip_atomic_store(&status[bid], cl_word(epoch, 2, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_base = excl;
        if (bid == nblk - 1) *nS_out = static_cast<uint32_t>(excl + agg);
      }
    }
    __syncthreads();
    if (c < nch) cbase[c] = static_cast<uint32_t>(s_base + wpre + incl - cnt);
    if (!PER_ENTRY) {  // few entries leave: one thread per chunk
      while (g) {
        const int b = __builtin_ctzll(g);
        g &= g - 1;
        told[slist[c * kWave + b]] = 0;
      }
    }
    __syncthreads();  // (s_w and s_base are reused by the next tile)
  }
}

template <bool PER_ENTRY>
__global__ __launch_bounds__(kBlock) void k_compact_write(const uint32_t* __restrict__ slist,
                                                          const unsigned long long* __restrict__ mask,
                                                          const unsigned long long* __restrict__ keep,
                                                          const uint32_t* __restrict__ cbase,
                                                          const uint32_t* __restrict__ nSp, uint64_t cap,
                                                          uint16_t* __restrict__ told, uint32_t* __restrict__ out,
                                                          uint64_t lcap) {
  constexpr int kR = 16;
  const int lane = lane_id();
  const uint64_t nch = min(cap, (static_cast<uint64_t>(*nSp) + kWave - 1) / kWave);
  const uint64_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * kWpb + threadIdx.x / kWave);
  const uint64_t nw = uint64_t(gridDim.x) * kWpb;
  for (uint64_t g0 = wv * kR; g0 < nch; g0 += nw * kR) {
    uint32_t u[kR], b[kR];
    unsigned long long kk[kR], gg[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const uint64_t c = g0 + q;
      const bool valid = c < nch;  // (wave-uniform)
      kk[q] = valid ? keep[c] : 0ull;
      gg[q] = PER_ENTRY && valid ? mask[c] & ~kk[q] : 0ull;
      b[q] = valid ? cbase[c] : 0u;
      // (unconditional, clamped to the list's allocation: one wait for all 16, not one per store)
      u[q] = slist[min(c * kWave + lane, lcap - 1)];
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      if ((kk[q] >> lane) & 1ull) out[b[q] + __builtin_popcountll(kk[q] & ((1ull << lane) - 1ull))] = u[q];
      if (PER_ENTRY && ((gg[q] >> lane) & 1ull)) told[u[q]] = 0;
    }
  }
}

void launch_compact_slist(Ctx& c) {
  ensure_slist2(c);
  const uint64_t cap = (uint64_t(c.nS_host) + kWave - 1) / kWave;  // nS_host: upper bound of the device count
  if (!cap || !c.smask_valid) return;
  if (c.ccap < cap) {
    if (c.d_ccnt) (void)hipFree(c.d_ccnt);
    if (c.d_cbase) (void)hipFree(c.d_cbase);
    if (c.d_ctmp) (void)hipFree(c.d_ctmp);
    c.d_ccnt = c.d_cbase = nullptr;
    c.d_ctmp = nullptr;
    const uint64_t words = std::max<uint64_t>(cap, (c.n + kWave - 1) / kWave);
    PM_HIP_CHECK(hipMalloc(&c.d_ccnt, words * sizeof(uint32_t)));
    PM_HIP_CHECK(hipMalloc(&c.d_cbase, words * sizeof(uint32_t)));
    c.ctmp_bytes = kScanBlocks * sizeof(uint32_t);  // the block sums of k_chunk_scan_*
    PM_HIP_CHECK(hipMalloc(&c.d_ctmp, c.ctmp_bytes));
    c.ccap = words;
  }
  const auto* mask = reinterpret_cast<const unsigned long long*>(c.d_smask[c.smask_cur]);
  // the pull superstep wrote its survivors per chunk (d_kmask): the keep masks; the T_pub buffer it read is
  // cleared at its live entries that were not kept (after launch_lcc_step: tpub[cur] was just written,
  // tpub[cur ^ 1] was read)
  auto* kmask = reinterpret_cast<unsigned long long*>(c.d_kmask);
  static const bool four = std::getenv("PM_COMPACT4") && std::string(std::getenv("PM_COMPACT4")) == "1";
  if (!four) {  // two launches (PM_COMPACT4=1: the four-launch form below, A/B)
    const uint64_t blocks = (cap + kBlock - 1) / kBlock;
    if (c.clstat_cap < blocks) {
      if (c.d_clstat) (void)hipFree(c.d_clstat);
      c.d_clstat = nullptr;
      c.clstat_cap = std::max<uint64_t>(blocks, ((c.n + kWave - 1) / kWave + kBlock - 1) / kBlock);
      PM_HIP_CHECK(hipMalloc(&c.d_clstat, c.clstat_cap * sizeof(unsigned long long) + 64));
      PM_HIP_CHECK(hipMemsetAsync(c.d_clstat, 0, c.clstat_cap * sizeof(unsigned long long) + 64, c.stream));
      c.cl_epoch = 0;
    }
    if (++c.cl_epoch >= (1ull << kClEpochBits)) {  // epochs wrapped: the words are cleared and counting restarts
      PM_HIP_CHECK(hipMemsetAsync(c.d_clstat, 0, c.clstat_cap * sizeof(unsigned long long), c.stream));
      c.cl_epoch = 1;
    }
    auto* st = static_cast<unsigned long long*>(c.d_clstat);
    auto scan = c.removed_cleared ? k_compact_scan<false> : k_compact_scan<true>;
    if (!c.cl_grid) {  // co-resident blocks of the scan (a cooperative launch checks it)
      int per_cu = 0;
      PM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_compact_scan<true>, kBlock, 0));
      int per_cu2 = 0;
      PM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, k_compact_scan<false>, kBlock, 0));
      hipDeviceProp_t prop;
      PM_HIP_CHECK(hipGetDeviceProperties(&prop, c.device));
      c.cl_grid = static_cast<unsigned>(std::max(1, std::min({per_cu, per_cu2, 4}) * prop.multiProcessorCount));
    }
    const unsigned sgrid = static_cast<unsigned>(std::min<uint64_t>(blocks, c.cl_grid));
    const uint32_t* a_slist = c.d_slist;
    const uint32_t* a_nS = c.d_nS;
    uint16_t* a_told = c.d_tpub[c.cur ^ 1];
    uint32_t* a_cbase = c.d_cbase;
    uint32_t* a_nSo = c.d_nS2;
    uint64_t a_cap = cap, a_epoch = c.cl_epoch;
    void* sargs[] = {&a_slist, &mask, &kmask, &a_nS, &a_cap, &a_told, &a_cbase, &a_nSo, &st, &a_epoch};
    // (one context on the device: an ordinary launch of the co-resident grid, Ctx::coop)
    if (!c.coop)
      PM_HIP_CHECK(hipLaunchKernel(reinterpret_cast<const void*>(scan), dim3(sgrid), dim3(kBlock), sargs, 0, c.stream));
    else
      PM_HIP_CHECK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(scan), dim3(sgrid), dim3(kBlock), sargs, 0,
                                              c.stream));
    auto write = c.removed_cleared ? k_compact_write<false> : k_compact_write<true>;
    hipLaunchKernelGGL(write, dim3(grid_for((cap + 15) / 16, kWpb, 2048)), dim3(kBlock), 0, c.stream, c.d_slist, mask,
                       kmask, c.d_cbase, c.d_nS, cap, c.d_tpub[c.cur ^ 1], c.d_slist2, std::max<uint64_t>(c.n, 1));
    PM_HIP_CHECK(hipGetLastError());
    std::swap(c.d_slist, c.d_slist2);
    std::swap(c.d_nS, c.d_nS2);
    c.smask_valid = false;
    c.slist_compacted = true;
    return;
  }
  if (c.removed_cleared)
    hipLaunchKernelGGL(k_live_keep_masks<false>, dim3(grid_for(cap, kBlock, 2048)), dim3(kBlock), 0, c.stream,
                       c.d_slist, mask, kmask, c.d_nS, cap, c.d_tpub[c.cur ^ 1], c.d_ccnt);
  else
    hipLaunchKernelGGL(k_live_keep_masks<true>, dim3(grid_for(cap * kWave, kBlock, 8192)), dim3(kBlock), 0, c.stream,
                       c.d_slist, mask, kmask, c.d_nS, cap, c.d_tpub[c.cur ^ 1], c.d_ccnt);
  auto* bsum = static_cast<uint32_t*>(c.d_ctmp);
  hipLaunchKernelGGL(k_chunk_scan_sums, dim3(kScanBlocks), dim3(kBlock), 0, c.stream, c.d_ccnt, c.d_nS, bsum);
  hipLaunchKernelGGL(k_chunk_scan_write, dim3(kScanBlocks), dim3(kBlock), 0, c.stream, c.d_ccnt, c.d_nS, bsum,
                     c.d_cbase);
  hipLaunchKernelGGL(k_live_write, dim3(grid_for(uint64_t(c.nS_host), kBlock, 2048)), dim3(kBlock), 0, c.stream,
                     c.d_slist, kmask, c.d_nS, c.d_ccnt, c.d_cbase, c.d_slist2, c.d_nS2);
  PM_HIP_CHECK(hipGetLastError());
  std::swap(c.d_slist, c.d_slist2);
  std::swap(c.d_nS, c.d_nS2);
  c.smask_valid = false;  // every entry of the new list is live
  c.slist_compacted = true;
}

// Batched zero fills (16-B stores in the aligned middle of each range) and the T_pub clear at the slist
// entries; the block that finishes last zeroes *np (read by every block's clear) and re-arms the ticket.
struct ZeroBatch {
  uint32_t* p[8];
  uint64_t words[8];
  int n;
  const uint32_t* list;
  uint32_t* np;
  uint64_t cap;
  uint16_t* t0;
  uint16_t* t1;
  uint32_t* ticket;
  uint32_t cblocks;  // blocks that clear (their last one zeroes *np): few, so the ticket atomics do not queue
};

__global__ __launch_bounds__(kBlock) void k_zero_batch(ZeroBatch b) {
  const uint64_t tid = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  const uint64_t nt = uint64_t(gridDim.x) * blockDim.x;
  for (int r = 0; r < b.n; ++r) {
    uint32_t* p = b.p[r];
    const uint64_t w = b.words[r];
    const uint64_t head = min<uint64_t>(w, ((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4);
    const uint64_t nv = (w - head) / 4;
    if (tid < head) p[tid] = 0u;
    uint4* v = reinterpret_cast<uint4*>(p + head);
    for (uint64_t i = tid; i < nv; i += nt) v[i] = make_uint4(0u, 0u, 0u, 0u);
    const uint64_t tail = head + nv * 4;
    if (tail + tid < w) p[tail + tid] = 0u;
  }
  if (!b.list || blockIdx.x >= b.cblocks) return;
  const uint64_t n = min(static_cast<uint64_t>(*b.np), b.cap);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(b.cblocks) * blockDim.x) {
    const uint32_t q = b.list[i];
    b.t0[q] = 0;
    b.t1[q] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(b.ticket, 1u) == b.cblocks - 1) {
      *b.np = 0u;
      *b.ticket = 0u;
    }
  }
}

void zero_later(Ctx& c, void* p, uint64_t bytes) {
  if (!bytes) return;
  if ((bytes & 3) || (reinterpret_cast<uintptr_t>(p) & 3)) throw std::runtime_error("internal: unaligned zero fill");
  if (c.nzq == 8) flush_zero(c);
  c.zq[c.nzq++] = Ctx::ZeroRange{p, bytes};
}

void stream_wait(hipStream_t s) {
  static const bool spin = !std::getenv("PM_SPIN") || std::string(std::getenv("PM_SPIN")) != "0";
  if (!spin) {
    PM_HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  // poll for a bounded time (the driver loop's read-backs are due within microseconds), then hand the core back
  // between polls: a long wait (a 140 ms NLC search, a collective's partner) does not hold a CPU the other
  // shards' host threads need
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 1;; ++k) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) PM_HIP_CHECK(e);
    if ((k & 63) == 0) {
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt > std::chrono::milliseconds(20)) {
        PM_HIP_CHECK(hipStreamSynchronize(s));
        return;
      }
      if (dt > std::chrono::microseconds(200)) std::this_thread::yield();
    }
  }
}

void flush_zero(Ctx& c) {
  if (!c.nzq && !c.clear_pending) return;
  ZeroBatch b{};
  uint64_t most = 0;
  for (int r = 0; r < c.nzq; ++r) {
    b.p[r] = static_cast<uint32_t*>(c.zq[r].p);
    b.words[r] = c.zq[r].bytes / 4;
    most = std::max(most, b.words[r] / 4);
  }
  b.n = c.nzq;
  if (c.clear_pending) {
    if (!c.d_zticket) {
      PM_HIP_CHECK(hipMalloc(&c.d_zticket, sizeof(uint32_t)));
      PM_HIP_CHECK(hipMemsetAsync(c.d_zticket, 0, sizeof(uint32_t), c.stream));
    }
    b.list = c.d_slist;
    b.np = c.d_nS;
    b.cap = c.clear_cap;
    b.t0 = c.d_tpub[0];
    b.t1 = c.d_tpub[1];
    b.ticket = c.d_zticket;
    most = std::max<uint64_t>(most, c.clear_cap);
  }
  const unsigned grid = grid_for(most, kBlock, 2048);
  b.cblocks = std::min<unsigned>(grid, grid_for(b.cap, 16 * kBlock, 2048));  // ~16 entries per thread
  hipLaunchKernelGGL(k_zero_batch, dim3(grid), dim3(kBlock), 0, c.stream, b);
  PM_HIP_CHECK(hipGetLastError());
  c.nzq = 0;
  c.clear_pending = false;
}

__global__ void k_clear_tpub(const uint32_t* __restrict__ list, const uint32_t* __restrict__ np, uint64_t cap,
                             uint16_t* __restrict__ t0, uint16_t* __restrict__ t1) {
  const uint64_t n = min(static_cast<uint64_t>(*np), cap);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t p = list[i];
    t0[p] = 0;
    t1[p] = 0;
  }
}

// End of an LCC call: the rows of S that are mostly dead entries (written length mlen above twice the alive count
// plus 64) are compacted in place, alive entries to the front in order (rows stay in neighbour-id order, flags kept),
// and mlen becomes the alive count.  Every later reader walks [offp, offp + mlen): without this a hub row kept
// its superstep-0 length (10^5 entries at C5 S=27 with a few thousand alive) for every later superstep and
// every NLC line position.  One wave per row with dead entries (reads precede the writes of each 64-entry
// step, and a write never passes its lane's read position).
__global__ __launch_bounds__(kBlock) void k_compact_rows(const uint32_t* __restrict__ slist,
                                                         const uint32_t* __restrict__ nSp,
                                                         const uint16_t* __restrict__ tcur,
                                                         const uint64_t* __restrict__ offp, uint32_t* __restrict__ mcol,
                                                         uint32_t* __restrict__ mlen,
                                                         const uint32_t* __restrict__ malive,
                                                         uint32_t* __restrict__ long_stamp, uint32_t stamp) {
  const int lane = lane_id();
  const uint64_t gw = blockIdx.x * uint64_t(kWpb) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t nw = uint64_t(gridDim.x) * kWpb;
  const uint64_t nS = *nSp;
  for (uint64_t c0 = gw * kWave; c0 < nS; c0 += nw * kWave) {
    const uint64_t i = c0 + lane;
    uint32_t v = 0;
    bool dead = false;
    if (i < nS) {
      v = slist[i];
      if (tcur[v]) {
        const uint32_t L = mlen[v];
        dead = L > 2 * malive[v] + kWave;  // (a row mostly alive is left as it is)
        // a row longer than a push-form piece after the compaction: the next call needs its piece lists
        if (!dead && L > kPushLong) *long_stamp = stamp;
      }
    }
    uint64_t bal = __ballot(dead);
    while (bal) {
      const int r = __ffsll(static_cast<long long>(bal)) - 1;
      bal &= bal - 1;
      const uint32_t u = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), r));
      const uint64_t b = offp[u];
      const uint32_t L = mlen[u];
      uint32_t cnt = 0;
      for (uint32_t j0 = 0; j0 < L; j0 += kWave) {
        const uint32_t j = j0 + lane;
        const uint32_t m = j < L ? mcol[b + j] : 0u;
        const bool keep = (m & kAlive) != 0;
        const uint64_t km = __ballot(keep);
        if (keep) mcol[b + cnt + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(km >> 32),
                                                           __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(km), 0u))] = m;
        cnt += static_cast<uint32_t>(__popcll(km));
      }
      if (lane == 0) {
        mlen[u] = cnt;
        if (cnt > kPushLong) *long_stamp = stamp;
      }
    }
  }
}

// (the long-row stamp goes to the word after the list count, read back with it: c.d_nS[1] == stamp <=> some row
// of S is longer than a push-form piece)
void launch_compact_rows(Ctx& c, uint32_t stamp) {
  if (!c.nS_host) return;
  hipLaunchKernelGGL(k_compact_rows, dim3(grid_for((uint64_t(c.nS_host) + kWave - 1) / kWave, kWpb, 4096)),
                     dim3(kBlock), 0, c.stream, c.d_slist, c.d_nS, c.d_tpub[c.cur], m_off(c), m_col(c), c.d_mlen,
                     c.d_malive, c.d_nS + 1, stamp);
  PM_HIP_CHECK(hipGetLastError());
}

void launch_clear_tpub(Ctx& c) {
  if (c.nS_host)
    hipLaunchKernelGGL(k_clear_tpub, dim3(grid_for(c.nS_host, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_slist,
                       c.d_nS, uint64_t(c.nS_host), c.d_tpub[0], c.d_tpub[1]);
  PM_HIP_CHECK(hipGetLastError());
}

void launch_count_state(Ctx& c, uint64_t* d_slot) {
  const unsigned grid = grid_for(c.nS_host, kBlock, kMaxGrid);
  hipLaunchKernelGGL(k_count_state, dim3(grid), dim3(kBlock), 0, c.stream, c.d_slist, c.d_nS, c.d_tpub[c.cur],
                     c.d_malive, owner_args(c), partials(c, d_slot));
  PM_HIP_CHECK(hipGetLastError());
  reduce_into(c, grid, d_slot);
}

// ===========================================================================
// Token passing.
//
// Both NLCC variants are run level-synchronously over all sources at once.
// Path/cycle (nem_1): a token (u, s, parent) at walk position k.  The
// reference's per-(vertex,source) first-arrival dedup (nem_1.hpp:131-139,
// :270-285) keeps the lowest position; tokens reaching (u,s) at that position
// from several parents forward to M[u] minus the parent when exactly one
// parent arrived, and to all of M[u] otherwise (identical to the reference
// whenever the NLC line is order-free).
// TDS (tds_batch_1): exhaustive walk enumeration, no dedup.

LineArgs make_line_args(const Ctx& c, const NlcLine& line) {
  LineArgs la{};
  const int n = static_cast<int>(line.cycle_length + 2);
  la.C = static_cast<int32_t>(line.cycle_length);
  la.VC = line.valid_cycle ? 1 : 0;
  la.ilast = static_cast<uint16_t>(line.indices.back());
  la.sv = line.selected_vertices ? 1 : 0;
  for (int k = 0; k < n; ++k) {
    la.I[k] = static_cast<uint16_t>(line.indices[k]);
    const uint64_t t = line.indices[k];
    la.lok[k] = (t < c.pattern.graph.vertex_data.size() && c.pattern.graph.vertex_data[t] == line.labels[k]) ? 1 : 0;
    la.E[k] = k < static_cast<int>(line.enumeration.size()) ? static_cast<uint16_t>(line.enumeration[k]) : 0xFFFF;
  }
  return la;
}

// Source selection, nem_1.hpp:387-479 / tds_batch_1.hpp:1067-1135 (over S:
// T_pub != 0 only for members of S).  Stream compaction of slist (rocPRIM).
struct SourcePred {
  const uint16_t* tpub;
  LineArgs la;
  int tds;
  __device__ bool operator()(uint32_t u) const {
    const uint16_t T = tpub[u];
    if (!T || !pos_ok(T, 0, la)) return false;
    if (!tds && !la.VC && !la.sv && !((T >> la.ilast) & 1u)) return false;
    return true;
  }
};

// Selected-vertices lines verify the active vertices with the line's last
// label (nem_1.hpp:409-436; they initiate no tokens).
struct DestPred {
  const uint16_t* tpub;
  const uint64_t* labs;
  uint64_t last;
  __device__ bool operator()(uint32_t u) const { return tpub[u] != 0 && labs[u] == last; }
};

__global__ void k_mark_sources(const uint32_t* __restrict__ sources, const int* __restrict__ nsrc,
                               uint8_t* __restrict__ tsm) {
  const uint64_t n = static_cast<uint64_t>(*nsrc);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    tsm[sources[i]] = 1;
}

// Number of alive entries of M[u] (excluding `skip`) -> outputs per item.
__global__ void k_row_alive(const uint32_t* __restrict__ items, uint64_t nitems, int stride, int pos,
                            const uint64_t* __restrict__ offp, const uint32_t* __restrict__ malive,
                            uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nitems; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = malive[items[i * stride + pos]];
}

// Level-1 tokens of path/cycle lines: (v, s, parent = s) for v in M[s].
__global__ void k_tp_init(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint64_t* __restrict__ obase,
                          const uint64_t* __restrict__ offp, const uint32_t* __restrict__ mcol,
                          const uint32_t* __restrict__ mlen,
                          uint32_t* __restrict__ tu, uint32_t* __restrict__ ts, uint32_t* __restrict__ tp) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    uint64_t o = obase[i];
    const uint64_t b = offp[s], L = mlen[s];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mcol[e] & kAlive)) continue;
      tu[o] = mcol[e] & kPosMask;
      ts[o] = s;
      tp[o] = s;
      ++o;
    }
  }
}

// Arrival filter at non-terminal position k (nem_1.hpp:172-297, :540-660).
__global__ void k_tp_filter(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ts, uint64_t ntok, int k,
                            LineArgs la, const uint16_t* __restrict__ tpub, unsigned long long* __restrict__ keys) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < ntok; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = tu[i], s = ts[i];
    const bool ok = (u != s) && pos_ok(tpub[u], k, la);
    keys[i] = ok ? ((static_cast<unsigned long long>(s) << 32) | u) : ~0ull;
  }
}

__device__ __forceinline__ bool sorted_contains(const unsigned long long* a, uint64_t n, unsigned long long key) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == key;
}

struct SeenSet {
  const unsigned long long* keys[16];
  uint64_t n[16];
  int count;
};

// Marks segment heads of the sorted (key, parent) list that are new (not seen
// at a lower position) and computes the forwarding exclusion.
__global__ void k_tp_unique(const unsigned long long* __restrict__ keys, const uint32_t* __restrict__ par,
                            uint64_t ntok, SeenSet seen, uint8_t* __restrict__ head, uint32_t* __restrict__ excl) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < ntok; i += uint64_t(gridDim.x) * blockDim.x) {
    const unsigned long long k = keys[i];
    uint8_t h = 0;
    uint32_t x = kNone;
    if (k != ~0ull && (i == 0 || keys[i - 1] != k)) {
      bool old = false;
      for (int l = 0; l < seen.count && !old; ++l) old = sorted_contains(seen.keys[l], seen.n[l], k);
      if (!old) {
        h = 1;
        x = par[i];
        for (uint64_t j = i + 1; j < ntok && keys[j] == k; ++j)
          if (par[j] != x) {
            x = kNone;
            break;
          }
      }
    }
    head[i] = h;
    excl[i] = x;
  }
}

// Expansion count: alive entries of M[u] other than the excluded parent.
__global__ void k_tp_expand_count(const unsigned long long* __restrict__ fk, const uint32_t* __restrict__ fx,
                                  uint64_t nf, const uint64_t* __restrict__ offp, const uint32_t* __restrict__ mcol,
                                  const uint32_t* __restrict__ mlen,
                                  const uint32_t* __restrict__ malive, uint32_t* __restrict__ cnt,
                                  unsigned long long* __restrict__ trav) {
  uint64_t t = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nf; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = static_cast<uint32_t>(fk[i] & 0xFFFFFFFFull);
    const uint32_t x = fx[i];
    const uint64_t b = offp[u], L = mlen[u];
    uint32_t c = 0;
    for (uint64_t e = b; e < b + L; ++e)
      if ((mcol[e] & kAlive) && (mcol[e] & kPosMask) != x) ++c;
    cnt[i] = c;
    t += malive[u];
  }
  block_atomic_add(trav, t);
}

__global__ void k_tp_expand_write(const unsigned long long* __restrict__ fk, const uint32_t* __restrict__ fx,
                                  uint64_t nf, const uint64_t* __restrict__ obase, const uint64_t* __restrict__ offp,
                                  const uint32_t* __restrict__ mcol, const uint32_t* __restrict__ mlen,
                                  uint32_t* __restrict__ tu,
                                  uint32_t* __restrict__ ts, uint32_t* __restrict__ tp) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nf; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = static_cast<uint32_t>(fk[i] & 0xFFFFFFFFull);
    const uint32_t s = static_cast<uint32_t>(fk[i] >> 32);
    const uint32_t x = fx[i];
    uint64_t o = obase[i];
    const uint64_t b = offp[u], L = mlen[u];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mcol[e] & kAlive)) continue;
      const uint32_t w = mcol[e] & kPosMask;
      if (w == x) continue;
      tu[o] = w;
      ts[o] = s;
      tp[o] = u;
      ++o;
    }
  }
}

// Terminal position C+1 (nem_1.hpp:661-791): path -> ack the source when the
// walk does not end on it; cycle -> mark the source and the closing edge.
__global__ void k_tp_terminal(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ts,
                              const uint32_t* __restrict__ tp, uint64_t ntok, LineArgs la,
                              const uint16_t* __restrict__ tpub, const uint64_t* __restrict__ offp,
                              uint32_t* __restrict__ mcol, const uint32_t* __restrict__ mlen,
                              const uint32_t* __restrict__ perm, uint8_t* __restrict__ tsm) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < ntok; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = tu[i], s = ts[i];
    if (!pos_ok(tpub[u], la.C + 1, la)) continue;
    if (!la.VC) {
      if (u == s) continue;
      if (tpub[s]) tsm[s] = 2;  // ack visitor needs an active source (nem_1.hpp:101, :326-336)
    } else {
      if (u != s) continue;
      tsm[s] = 2;
      // mark M[s][parent]: rows hold positions in neighbour-id order
      const uint32_t p = tp[i], pid = perm[p];
      uint64_t lo = offp[s], hi = offp[s] + mlen[s];
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (perm[mcol[mid] & kPosMask] < pid) lo = mid + 1; else hi = mid;
      }
      if (lo < offp[s] + mlen[s] && (mcol[lo] & kPosMask) == p && (mcol[lo] & kAlive)) mcol[lo] |= kFlag;
    }
  }
}

// Selected-vertices terminal (nem_1.hpp:680-719): a path reaching a verified
// vertex u from source s confirms u iff s is in u's token-source set.  The
// reference registers u when its own init visit runs and, on one rank, drains
// every source's tokens before visiting the next vertex
// (visitor_queue.hpp:221-251): u is registered for s's tokens iff id(u) <
// id(s) ("selected vertices").
__global__ void k_tp_terminal_sv(const uint32_t* __restrict__ tu, const uint32_t* __restrict__ ts, uint64_t ntok,
                                 LineArgs la, const uint16_t* __restrict__ tpub, const uint32_t* __restrict__ perm,
                                 uint8_t* __restrict__ tsm, SeenSet seen) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < ntok; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = tu[i], s = ts[i];
    if (u == s || !pos_ok(tpub[u], la.C + 1, la)) continue;
    if (tsm[u] == 0 || perm[u] >= perm[s]) continue;  // not a registered selected vertex yet
    const unsigned long long key = (static_cast<unsigned long long>(s) << 32) | u;
    bool found = false;
    for (int l = 0; l < seen.count && !found; ++l) found = sorted_contains(seen.keys[l], seen.n[l], key);
    if (found) tsm[u] = 2;
  }
}

// Position-1 walks of the sources; only each source's walks [clo, chi) are written (a source with more walks
// than a chunk holds is enumerated in windows of its walks).
__global__ void k_tds_init(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint64_t* __restrict__ obase,
                           uint64_t obase0, const uint64_t* __restrict__ offp, const uint32_t* __restrict__ mcol,
                           const uint32_t* __restrict__ mlen, int stride,
                           uint32_t* __restrict__ walks, uint64_t clo, uint64_t chi) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    uint64_t o = obase[i] - obase0, j = 0;
    const uint64_t b = offp[s], L = mlen[s];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mcol[e] & kAlive)) continue;
      if (j >= clo && j < chi) {
        walks[o * stride + 0] = s;
        walks[o * stride + 1] = mcol[e] & kPosMask;
        ++o;
      }
      ++j;
    }
  }
}

// Non-terminal position k: receiver checks, then sender-side filter per
// neighbour.  pass 0 counts, pass 1 writes each walk's children [clo, chi)
// (a walk with more children than a chunk holds is expanded in windows).
template <int PASS>
__global__ void k_tds_expand(const uint32_t* __restrict__ win, uint64_t nw, int k, int stride, LineArgs la,
                             const uint16_t* __restrict__ tpub, const uint64_t* __restrict__ offp,
                             const uint32_t* __restrict__ mcol,
                             const uint32_t* __restrict__ mlen, const uint32_t* __restrict__ malive,
                             uint32_t* __restrict__ cnt, const uint64_t* __restrict__ obase, uint64_t obase0,
                             uint32_t* __restrict__ wout, unsigned long long* __restrict__ trav, uint64_t clo = 0,
                             uint64_t chi = ~0ull) {
  uint64_t t = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nw; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t* w = win + i * stride;
    const uint32_t u = w[k];
    uint32_t c = 0;
    if (pos_ok(tpub[u], k, la) && enum_ok(w, k, u, la)) {
      const uint32_t s = w[0];
      const uint64_t b = offp[u], L = mlen[u];
      uint64_t o = PASS ? obase[i] - obase0 : 0;
      for (uint64_t e = b; e < b + L; ++e) {
        if (!(mcol[e] & kAlive)) continue;
        const uint32_t nb = mcol[e] & kPosMask;
        if (k == la.C) {
          if (la.VC) {
            if (nb != s) continue;
          } else {
            if (nb == s) continue;
            if (!enum_ok(w, k + 1, nb, la)) continue;
          }
        } else {
          if (!enum_ok(w, k + 1, nb, la)) continue;
        }
        if (PASS && c >= clo && c < chi) {
          uint32_t* d = wout + o * stride;
          for (int p = 0; p <= k; ++p) d[p] = w[p];
          d[k + 1] = nb;
          ++o;
        }
        ++c;
      }
      if (!PASS) t += malive[u];
    }
    if (!PASS) cnt[i] = c;
  }
  if (!PASS) block_atomic_add(trav, t);
}

// Terminal position C+1 (tds_batch_1.hpp:641-758).
__global__ void k_tds_terminal(const uint32_t* __restrict__ win, uint64_t nw, int stride, LineArgs la,
                               const uint16_t* __restrict__ tpub, uint8_t* __restrict__ tsm,
                               uint8_t* __restrict__ keep) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nw; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t* w = win + i * stride;
    const int k = la.C + 1;
    const uint32_t u = w[k], s = w[0];
    uint8_t kp = 0;
    if (pos_ok(tpub[u], k, la)) {
      if (!la.VC) {
        if (u != s) {
          kp = 1;
          if (tpub[s]) tsm[s] = 2;
        }
      } else if (u == s) {
        kp = 1;
        tsm[s] = 2;
      }
    }
    keep[i] = kp;
  }
}
__global__ void k_tp_post(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint8_t* __restrict__ tsm,
                          uint16_t* __restrict__ tpub, int i0, unsigned long long* __restrict__ out) {
  uint64_t acked = 0, deleted = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    if (tsm[s] == 2) {
      ++acked;
      continue;
    }
    uint16_t T = tpub[s];
    if (!T) continue;
    if ((T >> i0) & 1u) {
      T &= static_cast<uint16_t>(~(1u << i0));
      tpub[s] = T;  // T == 0: vertex_active = false and erased from the state map
    }
    ++deleted;
  }
  block_atomic_add(&out[0], acked);
  block_atomic_add(&out[1], deleted);
}

__global__ void k_clear_tsm(const uint32_t* __restrict__ sources, uint64_t nsrc, uint8_t* __restrict__ tsm) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x)
    tsm[sources[i]] = 0;
}

// ---------------------------------------------------------------------------
// host helpers for token passing
template <typename T>
static T* arena_alloc(Ctx& c, uint64_t n) {
  return static_cast<T*>(c.arena.get(std::max<uint64_t>(1, n) * sizeof(T)));
}

static uint64_t exclusive_scan_u32_to_u64(Ctx& c, const uint32_t* in, uint64_t* out, uint64_t n) {
  // out[0..n] = exclusive prefix; returns total (synchronizes the stream).
  if (n == 0) return 0;
  rocprim::transform_iterator<const uint32_t*, Widen, uint64_t> it(in, Widen());
  size_t tmp = 0;
  PM_HIP_CHECK(rocprim::inclusive_scan(nullptr, tmp, it, out + 1, size_t(n), rocprim::plus<uint64_t>(), c.stream));
  void* d_tmp = c.arena.get(tmp);
  PM_HIP_CHECK(rocprim::inclusive_scan(d_tmp, tmp, it, out + 1, size_t(n), rocprim::plus<uint64_t>(), c.stream));
  PM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(uint64_t), c.stream));
  uint64_t total = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&total, out + n, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return total;
}

// d_sources / c.nsources: the token_source_map keys of the line (marked 1 in
// tsm): its sources, or for a selected-vertices line the vertices it
// verifies, whose token initiators are returned in *init / *ninit (arena).
static void ensure_sources(Ctx& c, const LineArgs& la, int tds, const NlcLine& line, uint32_t** init = nullptr,
                           uint64_t* ninit = nullptr) {
  // previous line's sources are cleared from tsm first
  if (c.d_sources && c.nsources) {
    hipLaunchKernelGGL(k_clear_tsm, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                       c.nsources, c.d_tsm);
  }
  SourcePred pred{c.d_tpub[c.cur], la, tds};
  DestPred dpred{c.d_tpub[c.cur], c.d_labs, line.labels.back()};
  int* d_ns = arena_alloc<int>(c, 2);
  uint32_t* ilist = la.sv ? arena_alloc<uint32_t>(c, std::max<uint32_t>(c.nS_host, 1)) : nullptr;
  size_t tmp = 0, tmp2 = 0;
  const int nitems = static_cast<int>(std::max<uint32_t>(c.nS_host, 1));
  PM_HIP_CHECK(hipMemsetAsync(d_ns, 0, 2 * sizeof(int), c.stream));
  if (c.nS_host) {
    PM_HIP_CHECK(rocprim::select(nullptr, tmp, c.d_slist, c.d_sources, d_ns, nitems, pred, c.stream));
    PM_HIP_CHECK(rocprim::select(nullptr, tmp2, c.d_slist, c.d_sources, d_ns, nitems, dpred, c.stream));
    void* d_tmp = c.arena.get(std::max(tmp, tmp2));
    if (la.sv) {
      PM_HIP_CHECK(rocprim::select(d_tmp, tmp, c.d_slist, ilist, d_ns + 1, nitems, pred, c.stream));
      tmp2 = std::max(tmp, tmp2);
      PM_HIP_CHECK(rocprim::select(d_tmp, tmp2, c.d_slist, c.d_sources, d_ns, nitems, dpred, c.stream));
    } else {
      PM_HIP_CHECK(rocprim::select(d_tmp, tmp, c.d_slist, c.d_sources, d_ns, nitems, pred, c.stream));
    }
    hipLaunchKernelGGL(k_mark_sources, dim3(grid_for(c.nS_host, kBlock, 1024)), dim3(kBlock), 0, c.stream,
                       c.d_sources, d_ns, c.d_tsm);
    PM_HIP_CHECK(hipGetLastError());
  }
  int ns[2] = {0, 0};
  PM_HIP_CHECK(hipMemcpyAsync(ns, d_ns, sizeof(ns), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.nsources = static_cast<uint64_t>(ns[0]);
  if (init) {
    *init = la.sv ? ilist : c.d_sources;
    *ninit = la.sv ? static_cast<uint64_t>(ns[1]) : c.nsources;
  }
}

// Token-source sets across lines: the start of a line keeps (selected-vertices
// line) or drops (any other line) the previous line's entries.
__global__ void k_pseen_keep(const unsigned long long* __restrict__ keys, uint64_t n, const uint16_t* __restrict__ tpub,
                             const uint64_t* __restrict__ labs, uint64_t last, uint8_t* __restrict__ keep) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = static_cast<uint32_t>(keys[i] & 0xFFFFFFFFull);
    keep[i] = tpub[u] != 0 && labs[u] == last;
  }
}

static uint64_t pseen_start(Ctx& c, const NlcLine& line, const unsigned long long** out) {
  *out = nullptr;
  if (!line.selected_vertices || c.npseen == 0) return 0;
  auto* keep = arena_alloc<uint8_t>(c, c.npseen);
  auto* kept = arena_alloc<unsigned long long>(c, c.npseen);
  auto* d_n = arena_alloc<int>(c, 1);
  hipLaunchKernelGGL(k_pseen_keep, dim3(grid_for(c.npseen, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_pseen,
                     c.npseen, c.d_tpub[c.cur], c.d_labs, line.labels.back(), keep);
  size_t tmp = 0;
  PM_HIP_CHECK(rocprim::select(nullptr, tmp, c.d_pseen, keep, kept, d_n, size_t(c.npseen),
                                             c.stream));
  void* d_tmp = c.arena.get(tmp);
  PM_HIP_CHECK(rocprim::select(d_tmp, tmp, c.d_pseen, keep, kept, d_n, size_t(c.npseen),
                                             c.stream));
  int n = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&n, d_n, sizeof(n), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  *out = kept;
  return static_cast<uint64_t>(n);
}

// End of a line: the sets become the line's start entries plus every
// (source, vertex) a relay accepted during the line (sorted, unique).
static void pseen_end(Ctx& c, const SeenSet& seen) {
  uint64_t total = 0;
  for (int l = 0; l < seen.count; ++l) total += seen.n[l];
  c.npseen = 0;
  if (!total) return;
  auto* cat = arena_alloc<unsigned long long>(c, total);
  uint64_t o = 0;
  for (int l = 0; l < seen.count; ++l) {
    if (seen.n[l])
      PM_HIP_CHECK(hipMemcpyAsync(cat + o, seen.keys[l], seen.n[l] * sizeof(unsigned long long),
                                  hipMemcpyDeviceToDevice, c.stream));
    o += seen.n[l];
  }
  auto* sorted = arena_alloc<unsigned long long>(c, total);
  size_t tmp = 0;
  PM_HIP_CHECK(rocprim::radix_sort_keys(nullptr, tmp, cat, sorted, size_t(total), 0, 64, c.stream));
  void* d_tmp = c.arena.get(tmp);
  PM_HIP_CHECK(rocprim::radix_sort_keys(d_tmp, tmp, cat, sorted, size_t(total), 0, 64, c.stream));
  if (c.pseen_cap < total) {
    if (c.d_pseen) (void)hipFree(c.d_pseen);
    c.pseen_cap = std::max<uint64_t>(total, 2 * c.pseen_cap);
    PM_HIP_CHECK(hipMalloc(&c.d_pseen, c.pseen_cap * sizeof(unsigned long long)));
  }
  auto* d_n = arena_alloc<int>(c, 1);
  tmp = 0;
  PM_HIP_CHECK(rocprim::unique(nullptr, tmp, sorted, c.d_pseen, d_n, size_t(total), rocprim::equal_to<unsigned long long>(), c.stream));
  d_tmp = c.arena.get(tmp);
  PM_HIP_CHECK(rocprim::unique(d_tmp, tmp, sorted, c.d_pseen, d_n, size_t(total), rocprim::equal_to<unsigned long long>(), c.stream));
  int n = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&n, d_n, sizeof(n), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.npseen = static_cast<uint64_t>(n);
}

// The tokens of initiators init[0, ninit) through the line's positions (one launch + sync per position) and the
// terminal check; the line's seen sets are appended to `seen`.  Returns the batch's tokens and its traversed edges
// (level-1 scans included).  Every device buffer comes from the arena: a batch that does not fit throws ArenaFull
// before its terminal launch, with no effect outside the arena (its traversal counter is its own).
static void path_batch(Ctx& c, const LineArgs& la, const uint32_t* init, uint64_t ninit, SeenSet& seen,
                       uint64_t& tokens_out, uint64_t& edges_out) {
  const uint16_t* tpub = c.d_tpub[c.cur];
  auto* d_trav = arena_alloc<unsigned long long>(c, 1);
  PM_HIP_CHECK(hipMemsetAsync(d_trav, 0, sizeof(unsigned long long), c.stream));
  uint64_t tokens = 0;
  // level 1 tokens
  auto* cnt = arena_alloc<uint32_t>(c, ninit);
  auto* obase = arena_alloc<uint64_t>(c, ninit + 1);
  hipLaunchKernelGGL(k_row_alive, dim3(grid_for(ninit, kBlock, 4096)), dim3(kBlock), 0, c.stream, init, ninit, 1, 0,
                     m_off(c), c.d_malive, cnt);
  uint64_t ntok = exclusive_scan_u32_to_u64(c, cnt, obase, ninit);
  const uint64_t trav_init = ntok;  // sources scan all of M[s]
  auto* tu = arena_alloc<uint32_t>(c, ntok);
  auto* ts = arena_alloc<uint32_t>(c, ntok);
  auto* tp = arena_alloc<uint32_t>(c, ntok);
  hipLaunchKernelGGL(k_tp_init, dim3(grid_for(ninit, kBlock, 4096)), dim3(kBlock), 0, c.stream, init, ninit, obase,
                     m_off(c), m_col(c), c.d_mlen, tu, ts, tp);
  PM_HIP_CHECK(hipGetLastError());
  tokens += ntok;
  const int C = la.C;
  for (int k = 1; k <= C && ntok > 0; ++k) {
    auto* keys = arena_alloc<unsigned long long>(c, ntok);
    hipLaunchKernelGGL(k_tp_filter, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, tu, ts, ntok, k,
                       la, tpub, keys);
    auto* keys_s = arena_alloc<unsigned long long>(c, ntok);
    auto* par_s = arena_alloc<uint32_t>(c, ntok);
    size_t tmp = 0;
    PM_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp, keys, keys_s, tp, par_s, size_t(ntok), 0,
                                                    64, c.stream));
    void* d_tmp = c.arena.get(tmp);
    PM_HIP_CHECK(rocprim::radix_sort_pairs(d_tmp, tmp, keys, keys_s, tp, par_s, size_t(ntok), 0,
                                                    64, c.stream));
    auto* head = arena_alloc<uint8_t>(c, ntok);
    auto* excl = arena_alloc<uint32_t>(c, ntok);
    hipLaunchKernelGGL(k_tp_unique, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, keys_s, par_s,
                       ntok, seen, head, excl);
    // compact heads (stable: keeps keys sorted)
    auto* fk = arena_alloc<unsigned long long>(c, ntok);
    auto* fx = arena_alloc<uint32_t>(c, ntok);
    auto* d_nsel = arena_alloc<int>(c, 1);
    tmp = 0;
    PM_HIP_CHECK(rocprim::select(nullptr, tmp, keys_s, head, fk, d_nsel, size_t(ntok), c.stream));
    d_tmp = c.arena.get(tmp);
    PM_HIP_CHECK(rocprim::select(d_tmp, tmp, keys_s, head, fk, d_nsel, size_t(ntok), c.stream));
    PM_HIP_CHECK(rocprim::select(d_tmp, tmp, excl, head, fx, d_nsel, size_t(ntok), c.stream));
    int nsel = 0;
    PM_HIP_CHECK(hipMemcpyAsync(&nsel, d_nsel, sizeof(int), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    const uint64_t nf = static_cast<uint64_t>(nsel);
    if (seen.count < 16) {
      seen.keys[seen.count] = fk;
      seen.n[seen.count] = nf;
      seen.count++;
    }
    if (nf == 0) {
      ntok = 0;
      break;
    }
    auto* ecnt = arena_alloc<uint32_t>(c, nf);
    hipLaunchKernelGGL(k_tp_expand_count, dim3(grid_for(nf, kBlock, 1024)), dim3(kBlock), 0, c.stream, fk, fx, nf,
                       m_off(c), m_col(c), c.d_mlen, c.d_malive, ecnt, d_trav);
    auto* eb = arena_alloc<uint64_t>(c, nf + 1);
    const uint64_t nnext = exclusive_scan_u32_to_u64(c, ecnt, eb, nf);
    tu = arena_alloc<uint32_t>(c, nnext);
    ts = arena_alloc<uint32_t>(c, nnext);
    tp = arena_alloc<uint32_t>(c, nnext);
    hipLaunchKernelGGL(k_tp_expand_write, dim3(grid_for(nf, kBlock, 1024)), dim3(kBlock), 0, c.stream, fk, fx, nf, eb,
                       m_off(c), m_col(c), c.d_mlen, tu, ts, tp);
    PM_HIP_CHECK(hipGetLastError());
    ntok = nnext;
    tokens += ntok;
  }
  if (ntok > 0 && la.sv) {  // the terminal vertex is verified here
    hipLaunchKernelGGL(k_tp_terminal_sv, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, tu, ts, ntok,
                       la, tpub, c.d_perm, c.d_tsm, seen);
    PM_HIP_CHECK(hipGetLastError());
  } else if (ntok > 0) {
    hipLaunchKernelGGL(k_tp_terminal, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, tu, ts, tp, ntok,
                       la, tpub, m_off(c), m_col(c), c.d_mlen, c.d_perm, c.d_tsm);
    PM_HIP_CHECK(hipGetLastError());
  }
  unsigned long long trav = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&trav, d_trav, sizeof(trav), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  tokens_out = tokens;
  edges_out = trav + trav_init;
}

// nem_1.hpp path / cycle check on the exact path.  The initiators run in batches: all of them while their tokens
// fit the arena, otherwise halves, quarters, ... (a batch that ran out of room is discarded -- nothing outside the
// arena was written -- and its first half runs again).  A (source, vertex) key carries its source, so batches never
// share a dedup entry, and each source's acknowledgement comes from its own batch: the result is the unbatched one.
// The token-source sets a later selected-vertices line reads (pseen) are kept only when the line ran in one batch;
// a pattern with such a line whose line needs batches fails with the arena message.
TpResult run_path_line(Ctx& c, const NlcLine& line) {
  TpResult res;
  c.arena.reset();
  const LineArgs la = make_line_args(c, line);
  SeenSet seen0{};
  seen0.count = 0;
  const unsigned long long* p0 = nullptr;
  const uint64_t np0 = pseen_start(c, line, &p0);  // the token-source sets this line starts from
  if (np0) {
    seen0.keys[0] = p0;
    seen0.n[0] = np0;
    seen0.count = 1;
  }
  uint32_t* init = nullptr;  // token initiators
  uint64_t ninit = 0;
  ensure_sources(c, la, 0, line, &init, &ninit);
  res.sources = c.nsources;
  if (ninit == 0) {
    pseen_end(c, seen0);
    return res;
  }
  const size_t mark = c.arena.used;
  const char* fe = std::getenv("PM_PATH_BATCH");  // PM_PATH_BATCH=<initiators> (tests): batches of at most this many
  const uint64_t forced = fe ? std::max<uint64_t>(1, std::strtoull(fe, nullptr, 10)) : 0;
  uint64_t batch = forced ? std::min(forced, ninit) : ninit;
  SeenSet seen = seen0;
  for (uint64_t i0 = 0; i0 < ninit;) {
    const uint64_t n = std::min(batch, ninit - i0);
    if (n < ninit && c.any_sv)
      throw std::runtime_error("device scratch arena exhausted (a path line of a pattern with selected-vertices "
                               "lines needs source batches)");
    seen = seen0;
    uint64_t tokens = 0, edges = 0;
    try {
      path_batch(c, la, init + i0, n, seen, tokens, edges);
    } catch (const ArenaFull&) {
      PM_HIP_CHECK(hipStreamSynchronize(c.stream));  // (the batch's queued kernels write the arena it reuses)
      c.arena.used = mark;
      if (n == 1) throw std::runtime_error("device scratch arena exhausted (one source's tokens of a path line)");
      batch = (n + 1) / 2;
      ++res.batch_retries;
      continue;
    }
    res.tokens += tokens;
    res.edges += edges;
    ++res.batches;
    i0 += n;
    if (i0 < ninit) c.arena.used = mark;
  }
  if (res.batches == 1) pseen_end(c, seen);
  else c.npseen = 0;  // (no selected-vertices line reads them: any_sv is false here)
  return res;
}

// TDS line (tds_batch_1.hpp:976-1324) on the exact path: a depth-first enumeration over bounded chunks.  The
// reference enumerates in source batches (the batch loop at :1181) so that a batch's tokens fit; here every
// level of the walk tree is cut into chunks whose children number at most `cap` walks, and a chunk's whole
// subtree is enumerated (down to the terminal, whose kept walks go to the sink) before the next chunk is
// expanded.  Device memory is then bounded by (C + 1) levels of at most cap walks, whatever the total
// frontier; a level's pass-0 count (and its traversed-edge counter) still covers the level's whole walk set,
// and the kept walks come out in the order of the unbatched enumeration (lexicographic by the children's
// indices), for every cap.  A single walk (or source) with more than cap children is expanded in windows of
// cap of its children, so the bound holds for hubs at any position too.  PM_TDS_CAP=<walks> forces a small cap
// (tests).
namespace {
struct TdsRun {
  Ctx& c;
  LineArgs la;
  int C, stride;
  uint64_t cap;
  const uint16_t* tpub;
  unsigned long long* d_trav;
  TpResult& res;
  const TdsSink& sink;
  uint64_t chunks = 0, kept = 0;

  // children of the walks at position k: count, scan, then chunk by chunk
  void expand(int k, const uint32_t* walks, uint64_t nw) {
    if (k > C) return terminal(walks, nw);
    const size_t mark = c.arena.used;
    auto* wc = arena_alloc<uint32_t>(c, nw);
    hipLaunchKernelGGL(k_tds_expand<0>, dim3(grid_for(nw, kBlock, 1024)), dim3(kBlock), 0, c.stream, walks, nw, k,
                       stride, la, tpub, m_off(c), m_col(c), c.d_mlen, c.d_malive, wc,
                       static_cast<const uint64_t*>(nullptr), uint64_t(0), static_cast<uint32_t*>(nullptr), d_trav,
                       uint64_t(0), ~0ull);
    auto* wb = arena_alloc<uint64_t>(c, nw + 1);
    const uint64_t nnext = exclusive_scan_u32_to_u64(c, wc, wb, nw);
    res.tokens += nnext;
    if (nnext) {
      std::vector<uint64_t> hb;  // host copy of the scan when the level is split
      if (nnext > cap) {
        hb.resize(nw + 1);
        PM_HIP_CHECK(hipMemcpyAsync(hb.data(), wb, (nw + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        PM_HIP_CHECK(hipStreamSynchronize(c.stream));
      }
      for (uint64_t i0 = 0; i0 < nw;) {
        uint64_t i1 = nw, b0 = 0, n = nnext;
        if (!hb.empty()) {  // the longest run of walks whose children fit the cap (at least one walk)
          b0 = hb[i0];
          i1 = static_cast<uint64_t>(std::upper_bound(hb.begin() + i0 + 1, hb.end(), b0 + cap) - hb.begin()) - 1;
          i1 = std::max(i1, i0 + 1);
          n = hb[i1] - b0;
        }
        // (one walk with more than cap children, i1 == i0 + 1: its children in windows of cap, in order)
        for (uint64_t c0 = 0; c0 < n; c0 += cap) {
          const uint64_t nn = std::min(cap, n - c0);
          const size_t cm = c.arena.used;
          auto* child = arena_alloc<uint32_t>(c, nn * stride);
          hipLaunchKernelGGL(k_tds_expand<1>, dim3(grid_for(i1 - i0, kBlock, 1024)), dim3(kBlock), 0, c.stream,
                             walks + i0 * stride, i1 - i0, k, stride, la, tpub, m_off(c), m_col(c), c.d_mlen,
                             c.d_malive, wc + i0, wb + i0, b0, child, d_trav, c0, n > cap ? c0 + nn : ~0ull);
          PM_HIP_CHECK(hipGetLastError());
          ++chunks;
          expand(k + 1, child, nn);
          c.arena.used = cm;
        }
        i0 = i1;
      }
    }
    c.arena.used = mark;
  }

  // terminal position C+1 (tds_batch_1.hpp:641-758): kept walks to the sink, in order
  void terminal(const uint32_t* walks, uint64_t nw) {
    if (!nw) return;
    const size_t mark = c.arena.used;
    auto* keep = arena_alloc<uint8_t>(c, nw);
    hipLaunchKernelGGL(k_tds_terminal, dim3(grid_for(nw, kBlock, 1024)), dim3(kBlock), 0, c.stream, walks, nw, stride,
                       la, tpub, c.d_tsm, keep);
    PM_HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> all(nw * stride), out;
    std::vector<uint8_t> kp(nw);
    PM_HIP_CHECK(hipMemcpyAsync(all.data(), walks, nw * stride * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipMemcpyAsync(kp.data(), keep, nw, hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    for (uint64_t i = 0; i < nw; ++i)
      if (kp[i]) out.insert(out.end(), all.begin() + i * stride, all.begin() + (i + 1) * stride);
    const uint64_t nk = out.size() / stride;
    kept += nk;
    if (nk) sink(out.data(), nk);
    c.arena.used = mark;
  }
};
}  // namespace

uint64_t tds_walk_cap(const Ctx& c, int stride) {
  // (C + 1) levels of at most cap walks: the walks (4 B per position), their child counts (4 B) and scan (8 B)
  const uint64_t free_b = c.arena.cap > c.arena.used ? c.arena.cap - c.arena.used : 0;
  uint64_t cap = free_b / (uint64_t(stride) * (4ull * stride + 16) * 5 / 4);
  if (const char* e = std::getenv("PM_TDS_CAP")) cap = std::min<uint64_t>(cap, std::strtoull(e, nullptr, 10));
  return std::max<uint64_t>(cap, 1);
}

TpResult run_tds_line(Ctx& c, const NlcLine& line, uint32_t& stride_out, const TdsSink& sink) {
  TpResult res;
  c.arena.reset();
  const LineArgs la = make_line_args(c, line);
  const int C = la.C;
  const int stride = C + 2;
  stride_out = static_cast<uint32_t>(stride);
  c.last_tds_chunks = 0;
  if (line.enumeration.size() < static_cast<size_t>(stride))
    throw std::runtime_error("pattern_non_local_constraint enumeration shorter than the TDS walk");
  auto* d_trav = arena_alloc<unsigned long long>(c, 1);
  PM_HIP_CHECK(hipMemsetAsync(d_trav, 0, sizeof(unsigned long long), c.stream));
  c.npseen = 0;  // token-source sets are dropped at the start of a non-selected line (beta.cpp:791-793)
  ensure_sources(c, la, 1, line);
  res.sources = c.nsources;
  if (c.nsources == 0) return res;
  TdsRun run{c, la, C, stride, 0, c.d_tpub[c.cur], d_trav, res, sink};
  // the sources' position-1 walks [s, w] (w alive in M[s]) in source batches of at most cap walks
  auto* cnt = arena_alloc<uint32_t>(c, c.nsources);
  auto* obase = arena_alloc<uint64_t>(c, c.nsources + 1);
  hipLaunchKernelGGL(k_row_alive, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, 1, 0, m_off(c), c.d_malive, cnt);
  const uint64_t nw1 = exclusive_scan_u32_to_u64(c, cnt, obase, c.nsources);
  const uint64_t trav_init = nw1;  // sources scan all of M[s]
  res.tokens += nw1;
  run.cap = tds_walk_cap(c, stride);
  std::vector<uint64_t> hb;
  if (nw1 > run.cap) {
    hb.resize(c.nsources + 1);
    PM_HIP_CHECK(hipMemcpyAsync(hb.data(), obase, hb.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  }
  for (uint64_t i0 = 0; i0 < c.nsources;) {
    uint64_t i1 = c.nsources, b0 = 0, n = nw1;
    if (!hb.empty()) {
      b0 = hb[i0];
      i1 = static_cast<uint64_t>(std::upper_bound(hb.begin() + i0 + 1, hb.end(), b0 + run.cap) - hb.begin()) - 1;
      i1 = std::max(i1, i0 + 1);
      n = hb[i1] - b0;
    }
    // (one source with more than cap walks, i1 == i0 + 1: its walks in windows of cap, in order)
    for (uint64_t c0 = 0; c0 < n; c0 += run.cap) {
      const uint64_t nn = std::min(run.cap, n - c0);
      const size_t mark = c.arena.used;
      auto* walks = arena_alloc<uint32_t>(c, nn * stride);
      hipLaunchKernelGGL(k_tds_init, dim3(grid_for(i1 - i0, kBlock, 4096)), dim3(kBlock), 0, c.stream,
                         c.d_sources + i0, i1 - i0, obase + i0, b0, m_off(c), m_col(c), c.d_mlen, stride, walks, c0,
                         n > run.cap ? c0 + nn : ~0ull);
      PM_HIP_CHECK(hipGetLastError());
      ++run.chunks;
      run.expand(1, walks, nn);
      c.arena.used = mark;
    }
    i0 = i1;
  }
  c.last_tds_chunks = run.chunks;
  res.walks = run.kept;
  unsigned long long trav = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&trav, d_trav, sizeof(trav), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  res.edges = trav + trav_init;
  return res;
}

TpResult run_tds_line(Ctx& c, const NlcLine& line, std::vector<uint32_t>& walks_out, uint32_t& stride_out) {
  walks_out.clear();
  return run_tds_line(c, line, stride_out,
                      [&](const uint32_t* w, uint64_t n) { walks_out.insert(walks_out.end(), w, w + n * stride_out); });
}

uint32_t launch_post_tp(Ctx& c, const NlcLine& line) {
  if (c.nsources == 0) return 0;
  auto* out = arena_alloc<unsigned long long>(c, 2);
  PM_HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_tp_post, dim3(grid_for(c.nsources, kBlock, 1024)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, c.d_tsm, c.d_tpub[c.cur],
                     static_cast<int>(line.selected_vertices ? line.indices.back() : line.indices[0]), out);
  PM_HIP_CHECK(hipGetLastError());
  unsigned long long h[2] = {0, 0};
  PM_HIP_CHECK(hipMemcpyAsync(h, out, sizeof(h), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.last_acked = h[0];
  return h[1] ? 1u : 0u;
}

}  // namespace pm
