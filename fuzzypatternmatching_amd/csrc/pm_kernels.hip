// HIP kernels (gfx950 / CDNA4) for the label-constrained pattern-matching path.
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   off[V+1] u64, col[E] u32      CSR, rows sorted by target (duplicates adjacent)
//   tl[V] u16                     template bits whose label equals the vertex label
//   tpub[2][V] u16                template_vertices (T_pub), ping-pong per superstep;
//                                 0 <=> vertex not in the state map S
//   tst[V] u16                    vertex_state.template_vertices (T_state)
//   mcol[E] u32, mst[E] u8        active-edge map M[v], stored in v's own CSR slot
//                                 [off[v], off[v]+mlen[v]) so no prefix scan is needed;
//                                 mst bit0 = alive, bit1 = edge flag
//   mlen[V], malive[V] u32        written length / alive count of M[v]
//   slist[nS] u32                 vertices that entered S in superstep 0 (S only shrinks)
//
// Every LCC kernel is row-per-lane scheduled through "strips": a wave owns 64
// consecutive rows (vertices or slist entries), prefix-sums their lengths and
// then walks the concatenated entries 64 at a time, one entry per lane, so the
// adjacency reads are coalesced regardless of degree; per-row OR / count
// reductions are segmented wave scans (no LDS or global atomics per entry).
// This is an irregular gather: no MFMA (north_star).

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>

#include "pm_internal.hpp"

namespace pm {

static constexpr int kWave = 64;
static constexpr int kBlock = 256;
static constexpr int kWpb = kBlock / kWave;
static constexpr uint32_t kNone = 0xFFFFFFFFu;
static constexpr unsigned kMaxGrid = 1024;  // persistent-style grids: 4 blocks per CU
static constexpr int kU = 8;                // strip unroll: independent loads in flight per lane

struct PopcOp {
  __host__ __device__ uint64_t operator()(unsigned long long m) const {
    return static_cast<uint64_t>(__builtin_popcountll(m));
  }
};

// ---------------------------------------------------------------------------
// helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ uint16_t nbr_mask(uint16_t T, const PatArgs& pa) {
  uint16_t m = 0;
  while (T) {
    const int t = __ffs(static_cast<int>(T)) - 1;
    m |= pa.adj[t];
    T &= static_cast<uint16_t>(T - 1);
  }
  return m;
}

// global verify_and_update_vertex_state bit test (nonunique_ee.hpp:901-939):
// keep bit t iff adj[t] != 0 and adj[t] is a subset of TN.
__device__ __forceinline__ uint16_t keep_bits(uint16_t T, uint16_t TN, const PatArgs& pa) {
  uint16_t out = T, x = T;
  while (x) {
    const int t = __ffs(static_cast<int>(x)) - 1;
    x &= static_cast<uint16_t>(x - 1);
    const uint16_t a = pa.adj[t];
    if (a == 0 || (a & static_cast<uint16_t>(~TN))) out &= static_cast<uint16_t>(~(1u << t));
  }
  return out;
}

__device__ __forceinline__ uint32_t owner_of(uint64_t v, const OwnerArgs& oa) {
  if (oa.nranks <= 1) return 0;
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

// Segmented inclusive scan over lanes whose row ids are non-decreasing:
// OR of the low 16 bits, sum of the high 16 bits.
__device__ __forceinline__ uint32_t seg_scan_orsum(uint32_t x, int row) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, kWave);
    const int ry = __shfl_up(row, d, kWave);
    if (lane >= d && ry == row) x = ((x | y) & 0xFFFFu) + (((x >> 16) + (y >> 16)) << 16);
  }
  return x;
}

// Per-block counter partials (no same-address global atomics: a wave-level
// atomic per chunk on one word serialises at one L2 channel).  Layout of one
// block's W = 2P + 4 words: [vertices per rank | edges per rank | traversed |
// matching rows | removed flag | asymmetry flag]; k_reduce_partials sums them.
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

// All threads of the block must call this (after their loops).
__device__ __forceinline__ void flush_block(BlockAcc a, const OwnerArgs& oa, unsigned long long* s_hist,
                                            unsigned long long* s_red, unsigned long long* __restrict__ part) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t v[6] = {wave_sum(a.trav), wave_sum(a.match), wave_sum(a.vs), wave_sum(a.es),
                         wave_sum(a.removed), wave_sum(a.asym)};
  if (lane == 0)
    for (int i = 0; i < 6; ++i) s_red[w * 6 + i] = v[i];
  __syncthreads();
  const uint32_t P = oa.nranks <= 1 ? 1 : oa.nranks;
  const uint32_t W = 2 * P + 4;
  unsigned long long* out = part + uint64_t(blockIdx.x) * W;
  if (threadIdx.x < 6) {
    unsigned long long t = 0;
    for (int i = 0; i < kWpb; ++i) t += s_red[i * 6 + threadIdx.x];
    const int j = threadIdx.x;
    if (j == 0) out[2 * P] = t;
    if (j == 1) out[2 * P + 1] = t;
    if (j == 4) out[2 * P + 2] = t;
    if (j == 5) out[2 * P + 3] = t;
    if (oa.nranks <= 1) {
      if (j == 2) out[0] = t;
      if (j == 3) out[1] = t;
    }
  }
  if (oa.nranks > 1)
    for (uint32_t i = threadIdx.x; i < 2 * P; i += blockDim.x) out[i] = s_hist[i];
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

// One block: thread t sums blocks t, t+256, ... of every word (independent
// loads in flight), then a wave + LDS reduction per word.
__global__ __launch_bounds__(kBlock) void k_reduce_partials(const unsigned long long* __restrict__ part,
                                                            uint32_t nblocks, uint32_t W,
                                                            unsigned long long* __restrict__ slot) {
  __shared__ unsigned long long s_w[kWpb];
  for (uint32_t j = 0; j < W; ++j) {
    unsigned long long t = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += blockDim.x) t += part[uint64_t(b) * W + j];
    t = wave_sum(t);
    if (lane_id() == 0) s_w[threadIdx.x / kWave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long s = 0;
      for (int i = 0; i < kWpb; ++i) s += s_w[i];
      slot[j] = s;
    }
    __syncthreads();
  }
}

// Last row r (0..63) of a wave's strip space whose start <= j.
__device__ __forceinline__ int find_row(const uint64_t* rs, uint64_t j) {
  int lo = 0, hi = kWave - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rs[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ---------------------------------------------------------------------------
// K0: labels.
// vertex_data_db_degree.hpp:109  label = ceil(log2(degree + 1)) == bit_width(degree)
__global__ void k_degree_labels(const uint64_t* __restrict__ off, uint64_t n, uint64_t* __restrict__ labels) {
  for (uint64_t v = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; v < n; v += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t d = off[v + 1] - off[v];
    labels[v] = d ? static_cast<uint64_t>(64 - __clzll(static_cast<long long>(d))) : 0;
  }
}

// lppm_visitor::visit first-superstep label match (nonunique_ee.hpp:523-537).
// Also writes a 1-bit-per-vertex "matches some template" bitmap: superstep 0
// probes it before gathering Tl (V/8 bytes stay L2-resident, and only a
// minority of scanned entries point at matching vertices on R-MAT).
__global__ void k_label_match(const uint64_t* __restrict__ labels, uint64_t n, PatArgs pa, uint16_t* __restrict__ tl,
                              unsigned long long* __restrict__ tlbits) {
  const uint64_t nwords = (n + kWave - 1) / kWave;
  const int lane = lane_id();
  const uint64_t wave = (blockIdx.x * uint64_t(blockDim.x) + threadIdx.x) / kWave;
  const uint64_t nwaves = uint64_t(gridDim.x) * blockDim.x / kWave;
  for (uint64_t wd = wave; wd < nwords; wd += nwaves) {
    const uint64_t v = wd * kWave + lane;
    uint16_t t = 0;
    if (v < n) {
      const uint64_t lab = labels[v];
      for (int i = 0; i < pa.K; ++i)
        if (pa.plabel[i] == lab) t |= static_cast<uint16_t>(1u << i);
      tl[v] = t;
    }
    const unsigned long long m = __ballot(t != 0);
    if (lane == 0) tlbits[wd] = m;
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
// Survivors get T_pub = T_state, |M[u]| and a slot in slist.
// MODE (ablation only, 0 in the product): bit0 skips the M writes, bit1 the
// bitmap/Tl gathers, bit2 the segmented scans (diagnostic builds, wrong output).
template <int MODE, int KU = kU>
__global__ __launch_bounds__(kBlock) void k_lcc_first(
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ col, const uint16_t* __restrict__ tl,
    const unsigned long long* __restrict__ tlbits, uint64_t n, PatArgs pa, OwnerArgs oa, uint16_t* __restrict__ tst, uint16_t* __restrict__ tpub,
    uint32_t* __restrict__ mcol, uint8_t* __restrict__ mst, uint32_t* __restrict__ mlen,
    uint32_t* __restrict__ malive, unsigned long long* __restrict__ cmask, unsigned long long* __restrict__ part) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  BlockAcc acc;
  __shared__ uint64_t s_rs[kWpb][kWave];
  __shared__ uint64_t s_beg[kWpb][kWave];
  __shared__ uint32_t s_acc[kWpb][kWave];  // TN | (contributing distinct count << 16), carried across strips
  __shared__ uint32_t s_cnt[kWpb][kWave];  // running distinct count (can exceed 16 bits)
  __shared__ uint16_t s_nm[kWpb][kWave];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t nchunks = (n + kWave - 1) / kWave;
  const uint64_t cstride = uint64_t(gridDim.x) * kWpb;
  // Vertex data of the next chunk is loaded one iteration ahead (software
  // pipelining): Tl and the two row offsets come from independent, coalesced
  // loads (off[u+1] via a lane shuffle) so no HBM round trip sits between chunks.
  uint64_t chunk = uint64_t(blockIdx.x) * kWpb + w;
  uint16_t pf_t = 0;
  uint64_t pf_o = 0, pf_o63 = 0;
  auto prefetch = [&](uint64_t c) {
    const uint64_t u = c * kWave + lane;
    pf_t = (c < nchunks && u < n) ? tl[u] : uint16_t(0);
    pf_o = (c < nchunks) ? off[u < n ? u : n] : 0;
    pf_o63 = (c < nchunks && lane == kWave - 1) ? off[(u + 1) < n ? (u + 1) : n] : 0;
  };
  prefetch(chunk);
  for (; chunk < nchunks; chunk += cstride) {
    const uint64_t u = chunk * kWave + lane;
    const uint16_t Tu = pf_t;
    const uint64_t o_next = __shfl_down(pf_o, 1, kWave);
    const uint64_t beg = pf_o;
    const uint64_t deg = Tu ? ((lane == kWave - 1 ? pf_o63 : o_next) - beg) : 0;
    prefetch(chunk + cstride);
    const uint64_t incl = wave_incl_scan(deg);
    const uint64_t total = __shfl(incl, kWave - 1, kWave);
    s_rs[w][lane] = incl - deg;
    s_beg[w][lane] = beg;
    s_nm[w][lane] = nbr_mask(Tu, pa);
    s_acc[w][lane] = 0;
    s_cnt[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    // Strips of kU x 64 entries: every lane issues kU independent adjacency
    // loads, then kU independent Tl gathers, before any reduction (memory-level
    // parallelism; a single 64-entry strip per iteration is latency bound).
    for (uint64_t j0 = 0; j0 < total; j0 += uint64_t(kWave) * KU) {
      int r[KU];
      uint64_t rel[KU], e[KU];
      uint32_t v[KU];
#pragma unroll
      for (int q = 0; q < KU; ++q) {
        const uint64_t j = j0 + uint64_t(q) * kWave + lane;
        r[q] = kWave;  // sentinel row for idle lanes
        rel[q] = 0;
        e[q] = 0;
        v[q] = kNone;
        if (j < total) {
          r[q] = find_row(s_rs[w], j);
          rel[q] = j - s_rs[w][r[q]];
          e[q] = s_beg[w][r[q]] + rel[q];
          v[q] = col[e[q]];
        }
      }
      uint32_t pv0 = kNone;
      if (lane == 0 && r[0] < kWave && rel[0] > 0) pv0 = col[e[0] - 1];
      bool hit[KU];
      uint16_t tv[KU];
      if (MODE & 2) {
#pragma unroll
        for (int q = 0; q < KU; ++q) tv[q] = static_cast<uint16_t>(v[q] & 0x1Fu);
      } else {
#pragma unroll
        for (int q = 0; q < KU; ++q) hit[q] = (r[q] < kWave) && ((tlbits[v[q] >> 6] >> (v[q] & 63)) & 1ull);
#pragma unroll
        for (int q = 0; q < KU; ++q) tv[q] = hit[q] ? tl[v[q]] : uint16_t(0);
      }
#pragma unroll
      for (int q = 0; q < KU; ++q) {
        // predecessor entry j-1 (same row whenever rel > 0): lane-1 of this
        // slice, lane 63 of the previous slice, or loaded before the strip.
        uint32_t pv = __shfl_up(v[q], 1, kWave);
        const uint32_t carry = q ? __shfl(v[q ? q - 1 : 0], kWave - 1, kWave) : pv0;
        if (lane == 0) pv = carry;
        const bool valid = r[q] < kWave;
        uint32_t x = 0;
        if (valid) {
          const bool first = (rel[q] == 0) || (pv != v[q]);
          const bool cm = (tv[q] & s_nm[w][r[q]]) != 0;
          x = (cm ? tv[q] : 0u) | ((cm && first) ? (1u << 16) : 0u);
        }
        const uint32_t inc = (MODE & 4) ? x : seg_scan_orsum(x, r[q]);
        const int rnext = __shfl_down(r[q], 1, kWave);
        if (valid) {
          if ((x >> 16) && !(MODE & 1)) {
            // exclusive position of this distinct contributor inside u's row
            const uint32_t pos = s_cnt[w][r[q]] + (inc >> 16) - 1;
            const uint64_t dst = s_beg[w][r[q]] + pos;
            mcol[dst] = v[q];
            mst[dst] = 1;
          }
          if (lane == kWave - 1 || rnext != r[q]) {
            s_acc[w][r[q]] |= inc & 0xFFFFu;
            s_cnt[w][r[q]] += inc >> 16;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    // finalize row `lane`
    bool survivor = false, removed = false;
    uint32_t cnt = 0;
    if (u < n && Tu) {
      const uint16_t TN = static_cast<uint16_t>(s_acc[w][lane] & 0xFFFFu);
      if (TN) {  // entered the state map
        const uint16_t T = keep_bits(Tu, TN, pa);
        if (T) {
          survivor = true;
          cnt = s_cnt[w][lane];
          tst[u] = T;
          tpub[u] = T;
          mlen[u] = cnt;
          malive[u] = cnt;
        } else {
          removed = true;
        }
      }
    }
    const uint64_t smask = __ballot(survivor);
    if (lane == 0) cmask[chunk] = smask;  // slist is built from these masks (k_slist_write)
    // counts: vertices/edges per rank (owner rule) and traversed entries
    acc.trav += deg;
    acc.match += Tu != 0;
    acc.removed |= removed;
    if (survivor) {
      if (oa.nranks <= 1) {
        acc.vs += 1;
        acc.es += cnt;
      } else {
        acc_owner(s_hist, oa, u, cnt);
      }
    }
  }
  flush_block(acc, oa, s_hist, s_red, part);
}

// Alternative superstep-0 kernel (ablation): one lane per row, serial scan of
// the row with kU-way unrolled independent loads; no LDS, no shuffles.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_lcc_first_lpr(
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ col, const uint16_t* __restrict__ tl,
    const unsigned long long* __restrict__ tlbits, uint64_t n, PatArgs pa, OwnerArgs oa,
    uint16_t* __restrict__ tst, uint16_t* __restrict__ tpub, uint32_t* __restrict__ mcol, uint8_t* __restrict__ mst,
    uint32_t* __restrict__ mlen, uint32_t* __restrict__ malive, unsigned long long* __restrict__ cmask,
    unsigned long long* __restrict__ part) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  BlockAcc acc;
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t nchunks = (n + kWave - 1) / kWave;
  for (uint64_t chunk = uint64_t(blockIdx.x) * kWpb + w; chunk < nchunks; chunk += uint64_t(gridDim.x) * kWpb) {
    const uint64_t u = chunk * kWave + lane;
    uint16_t Tu = 0;
    uint64_t beg = 0, deg = 0;
    if (u < n) {
      Tu = tl[u];
      if (Tu) {
        beg = off[u];
        deg = off[u + 1] - beg;
      }
    }
    const uint16_t NM = nbr_mask(Tu, pa);
    uint32_t TN = 0, cnt = 0, prev = kNone;
    for (uint64_t i0 = 0; i0 < deg; i0 += kU) {
      uint32_t v[kU];
      uint16_t tv[kU];
#pragma unroll
      for (int q = 0; q < kU; ++q) v[q] = (i0 + q < deg) ? col[beg + i0 + q] : kNone;
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        const bool hit = v[q] != kNone && ((tlbits[v[q] >> 6] >> (v[q] & 63)) & 1ull);
        tv[q] = hit ? tl[v[q]] : uint16_t(0);
      }
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        if (v[q] == kNone) break;
        const bool cm = (tv[q] & NM) != 0;
        if (cm) {
          TN |= tv[q];
          if (v[q] != prev) {
            if (!(MODE & 1)) {
              mcol[beg + cnt] = v[q];
              mst[beg + cnt] = 1;
            }
            ++cnt;
          }
        }
        prev = v[q];
      }
    }
    bool survivor = false, removed = false;
    if (Tu && TN) {
      const uint16_t T = keep_bits(Tu, static_cast<uint16_t>(TN), pa);
      if (T) {
        survivor = true;
        tst[u] = T;
        tpub[u] = T;
        mlen[u] = cnt;
        malive[u] = cnt;
      } else {
        removed = true;
      }
    }
    const uint64_t smask = __ballot(survivor);
    if (lane == 0) cmask[chunk] = smask;
    acc.trav += deg;
    acc.match += Tu != 0;
    acc.removed |= removed;
    if (survivor) {
      if (oa.nranks <= 1) {
        acc.vs += 1;
        acc.es += cnt;
      } else {
        acc_owner(s_hist, oa, u, cnt);
      }
    }
  }
  flush_block(acc, oa, s_hist, s_red, part);
}

// slist from the superstep-0 survivor masks: an exclusive scan of the
// per-chunk popcounts (hipcub) gives each chunk's base.
__global__ void k_slist_write(const unsigned long long* __restrict__ cmask, const uint64_t* __restrict__ base,
                              uint64_t nchunks, uint32_t* __restrict__ slist, uint32_t* __restrict__ nS) {
  for (uint64_t c = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; c < nchunks; c += uint64_t(gridDim.x) * blockDim.x) {
    unsigned long long m = cmask[c];
    uint64_t o = base[c];
    while (m) {
      const int b = __ffsll(static_cast<long long>(m)) - 1;
      m &= m - 1;
      slist[o++] = static_cast<uint32_t>(c * kWave + b);
    }
    if (c == nchunks - 1) *nS = static_cast<uint32_t>(o);
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
// symmetry, which is reported through flags[1] (the host then refuses to go on).
__global__ __launch_bounds__(kBlock) void k_lcc_step(
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ slist, const uint32_t* __restrict__ nSp,
    const uint16_t* __restrict__ tcur, uint16_t* __restrict__ tnxt, uint16_t* __restrict__ tst, PatArgs pa,
    OwnerArgs oa, const uint32_t* __restrict__ mcol, uint8_t* __restrict__ mst, const uint32_t* __restrict__ mlen,
    uint32_t* __restrict__ malive, unsigned long long* __restrict__ part) {
  __shared__ unsigned long long s_hist[2 * kMaxRanks];
  __shared__ unsigned long long s_red[kWpb * 6];
  for (int i = threadIdx.x; i < 2 * kMaxRanks; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  BlockAcc acc;
  __shared__ uint64_t s_rs[kWpb][kWave];
  __shared__ uint64_t s_beg[kWpb][kWave];
  __shared__ uint32_t s_acc[kWpb][kWave];
  __shared__ uint32_t s_cnt[kWpb][kWave];
  __shared__ uint16_t s_nm[kWpb][kWave];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const uint32_t nS = *nSp;
  const uint64_t nchunks = (uint64_t(nS) + kWave - 1) / kWave;
  for (uint64_t chunk = uint64_t(blockIdx.x) * kWpb + w; chunk < nchunks; chunk += uint64_t(gridDim.x) * kWpb) {
    const uint64_t i = chunk * kWave + lane;
    uint32_t u = kNone;
    uint16_t Tu = 0;
    uint64_t beg = 0, len = 0;
    uint32_t alive0 = 0;
    if (i < nS) {
      u = slist[i];
      Tu = tcur[u];
      if (Tu) {
        beg = off[u];
        len = mlen[u];
        alive0 = malive[u];
      } else {
        tnxt[u] = 0;
      }
    }
    const uint64_t incl = wave_incl_scan(len);
    const uint64_t total = __shfl(incl, kWave - 1, kWave);
    s_rs[w][lane] = incl - len;
    s_beg[w][lane] = beg;
    s_nm[w][lane] = nbr_mask(Tu, pa);
    s_acc[w][lane] = 0;
    s_cnt[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    bool asym = false;
    for (uint64_t j0 = 0; j0 < total; j0 += uint64_t(kWave) * kU) {
      int r[kU];
      uint64_t e[kU];
      uint8_t st[kU];
      uint32_t v[kU];
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        const uint64_t j = j0 + uint64_t(q) * kWave + lane;
        r[q] = kWave;
        e[q] = 0;
        st[q] = 0;
        v[q] = 0;
        if (j < total) {
          r[q] = find_row(s_rs[w], j);
          e[q] = s_beg[w][r[q]] + (j - s_rs[w][r[q]]);
          st[q] = mst[e[q]];
          v[q] = mcol[e[q]];
        }
      }
      uint16_t tv[kU];
#pragma unroll
      for (int q = 0; q < kU; ++q) tv[q] = (st[q] & 1u) ? tcur[v[q]] : uint16_t(0);
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        uint32_t x = 0;
        if (st[q] & 1u) {
          const bool ok = (tv[q] & s_nm[w][r[q]]) != 0;
          const bool flag = ok || (st[q] & 2u);
          mst[e[q]] = flag ? 1u : 0u;
          if ((st[q] & 2u) && !ok && tv[q]) asym = true;
          x = (ok ? tv[q] : 0u) | (flag ? (1u << 16) : 0u);
        }
        const uint32_t inc = seg_scan_orsum(x, r[q]);
        const int rnext = __shfl_down(r[q], 1, kWave);
        if (r[q] < kWave && (lane == kWave - 1 || rnext != r[q])) {
          s_acc[w][r[q]] |= inc & 0xFFFFu;
          s_cnt[w][r[q]] += inc >> 16;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    bool survivor = false, removed = false;
    uint32_t cnt = 0;
    if (Tu) {
      const uint16_t TN = static_cast<uint16_t>(s_acc[w][lane] & 0xFFFFu);
      const uint16_t T = keep_bits(tst[u], TN, pa);
      if (T) {
        survivor = true;
        cnt = s_cnt[w][lane];
        tst[u] = T;
        tnxt[u] = T;
        malive[u] = cnt;
      } else {
        removed = true;
        tnxt[u] = 0;
        malive[u] = 0;
      }
    }
    acc.trav += alive0;
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
  }
  flush_block(acc, oa, s_hist, s_red, part);
}

// Counts of the current state (after token-passing post-processing).
__global__ __launch_bounds__(kBlock) void k_count_state(const uint32_t* __restrict__ slist,
                                                        const uint32_t* __restrict__ nSp,
                                                        const uint16_t* __restrict__ tpub,
                                                        const uint32_t* __restrict__ malive, OwnerArgs oa,
                                                        unsigned long long* __restrict__ part) {
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
  flush_block(acc, oa, s_hist, s_red, part);
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
  oa.nhubs = static_cast<uint32_t>(c.hubs_host.size());
  oa.nranks = c.nranks;
  return oa;
}

void launch_degree_labels(Ctx& c) {
  hipLaunchKernelGGL(k_degree_labels, dim3(grid_for(c.n, kBlock, 8192)), dim3(kBlock), 0, c.stream, c.d_off, c.n,
                     c.d_labels);
  PM_HIP_CHECK(hipGetLastError());
}

void launch_label_match(Ctx& c) {
  hipLaunchKernelGGL(k_label_match, dim3(grid_for(c.n, kBlock, 8192)), dim3(kBlock), 0, c.stream, c.d_labels, c.n,
                     c.pa, c.d_tl, reinterpret_cast<unsigned long long*>(c.d_tlbits));
  PM_HIP_CHECK(hipGetLastError());
}

uint32_t slot_words(const Ctx& c) { return 2 * (c.nranks <= 1 ? 1 : c.nranks) + 4; }

static void reduce_into(Ctx& c, unsigned grid, uint64_t* d_slot) {
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kBlock), 0, c.stream,
                     reinterpret_cast<const unsigned long long*>(c.d_part), grid, slot_words(c),
                     reinterpret_cast<unsigned long long*>(d_slot));
  PM_HIP_CHECK(hipGetLastError());
}

// variant: 0 = product (strip kernel); 1..7 = strip ablation MODE; 16+ = lane-per-row (MODE = variant-16)
void launch_lcc_first_kernel(Ctx& c, int variant, unsigned grid) {
#define PM_K1_ARGS                                                                                                 \
  dim3(grid), dim3(kBlock), 0, c.stream, c.d_off, c.d_col, c.d_tl,                                                \
      reinterpret_cast<const unsigned long long*>(c.d_tlbits), c.n, c.pa, owner_args(c), c.d_tst, c.d_tpub[c.cur], \
      c.d_mcol, c.d_mst, c.d_mlen, c.d_malive, reinterpret_cast<unsigned long long*>(c.d_cmask),                   \
      reinterpret_cast<unsigned long long*>(c.d_part)
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_lcc_first<0>, PM_K1_ARGS); break;
    case 1: hipLaunchKernelGGL(k_lcc_first<1>, PM_K1_ARGS); break;
    case 2: hipLaunchKernelGGL(k_lcc_first<2>, PM_K1_ARGS); break;
    case 3: hipLaunchKernelGGL(k_lcc_first<3>, PM_K1_ARGS); break;
    case 4: hipLaunchKernelGGL(k_lcc_first<4>, PM_K1_ARGS); break;
    case 7: hipLaunchKernelGGL(k_lcc_first<7>, PM_K1_ARGS); break;
    case 8: hipLaunchKernelGGL((k_lcc_first<0, 4>), PM_K1_ARGS); break;
    case 9: hipLaunchKernelGGL((k_lcc_first<0, 16>), PM_K1_ARGS); break;
    case 16: hipLaunchKernelGGL(k_lcc_first_lpr<0>, PM_K1_ARGS); break;
    case 17: hipLaunchKernelGGL(k_lcc_first_lpr<1>, PM_K1_ARGS); break;
    default: throw std::runtime_error("unknown superstep-0 kernel variant");
  }
#undef PM_K1_ARGS
  PM_HIP_CHECK(hipGetLastError());
}

unsigned lcc_first_grid(const Ctx& c) {
  return grid_for((c.n + kWave - 1) / kWave, kWpb, c.k1_resident_blocks ? c.k1_resident_blocks : kMaxGrid);
}

// Resident 256-thread blocks of the superstep-0 kernel on the whole chip
// (occupancy query minus one block per CU: the API over-reports by one for
// SGPR-heavy 256-thread kernels, MI355X_MICROARCH.md "Residency").
unsigned query_k1_resident_blocks(int device) {
  int per_cu = 0;
  PM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lcc_first<0>, kBlock, 0));
  hipDeviceProp_t prop;
  PM_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  per_cu = std::max(1, per_cu - 1);
  return static_cast<unsigned>(per_cu * prop.multiProcessorCount);
}

void launch_lcc_first(Ctx& c, uint64_t* d_slot) {
  const uint64_t chunks = (c.n + kWave - 1) / kWave;
  const unsigned grid = lcc_first_grid(c);
  launch_lcc_first_kernel(c, 0, grid);
  reduce_into(c, grid, d_slot);
  // slist = survivors in id order
  hipcub::TransformInputIterator<uint64_t, PopcOp, const unsigned long long*> it(
      reinterpret_cast<const unsigned long long*>(c.d_cmask), PopcOp());
  size_t tmp = c.scan_tmp_bytes;
  PM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(c.d_scan_tmp, tmp, it, c.d_cbase, static_cast<int>(chunks), c.stream));
  hipLaunchKernelGGL(k_slist_write, dim3(grid_for(chunks, kBlock, 4096)), dim3(kBlock), 0, c.stream,
                     reinterpret_cast<const unsigned long long*>(c.d_cmask), c.d_cbase, chunks, c.d_slist, c.d_nS);
  PM_HIP_CHECK(hipGetLastError());
}

size_t slist_scan_tmp_bytes(uint64_t n) {
  const uint64_t chunks = (n + kWave - 1) / kWave;
  hipcub::TransformInputIterator<uint64_t, PopcOp, const unsigned long long*> it(nullptr, PopcOp());
  size_t tmp = 0;
  PM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, static_cast<uint64_t*>(nullptr),
                                                static_cast<int>(std::max<uint64_t>(chunks, 1)), hipStream_t(0)));
  return tmp;
}

void launch_lcc_step(Ctx& c, uint64_t* d_slot) {
  const uint64_t chunks = (uint64_t(c.nS_host) + kWave - 1) / kWave;
  const unsigned grid = grid_for(chunks, kWpb, kMaxGrid);
  hipLaunchKernelGGL(k_lcc_step, dim3(grid), dim3(kBlock), 0, c.stream, c.d_off, c.d_slist, c.d_nS,
                     c.d_tpub[c.cur], c.d_tpub[c.cur ^ 1], c.d_tst, c.pa, owner_args(c), c.d_mcol, c.d_mst, c.d_mlen,
                     c.d_malive, reinterpret_cast<unsigned long long*>(c.d_part));
  PM_HIP_CHECK(hipGetLastError());
  reduce_into(c, grid, d_slot);
  c.cur ^= 1;
}

void launch_count_state(Ctx& c, uint64_t* d_slot) {
  const unsigned grid = grid_for(c.nS_host, kBlock, kMaxGrid);
  hipLaunchKernelGGL(k_count_state, dim3(grid), dim3(kBlock), 0, c.stream, c.d_slist, c.d_nS, c.d_tpub[c.cur],
                     c.d_malive, owner_args(c), reinterpret_cast<unsigned long long*>(c.d_part));
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
  for (int k = 0; k < n; ++k) {
    la.I[k] = static_cast<uint16_t>(line.indices[k]);
    const uint64_t t = line.indices[k];
    la.lok[k] = (t < c.pattern.graph.vertex_data.size() && c.pattern.graph.vertex_data[t] == line.labels[k]) ? 1 : 0;
    la.E[k] = k < static_cast<int>(line.enumeration.size()) ? static_cast<uint16_t>(line.enumeration[k]) : 0xFFFF;
  }
  return la;
}

__device__ __forceinline__ bool pos_ok(uint16_t T, int k, const LineArgs& la) {
  return la.lok[k] && ((T >> la.I[k]) & 1u);
}

// Source selection, nem_1.hpp:387-479 / tds_batch_1.hpp:1067-1135 (over S:
// T_pub != 0 only for members of S).  Stream compaction of slist (hipcub).
struct SourcePred {
  const uint16_t* tpub;
  LineArgs la;
  int tds;
  __device__ bool operator()(uint32_t u) const {
    const uint16_t T = tpub[u];
    if (!T || !pos_ok(T, 0, la)) return false;
    if (!tds && !la.VC && !((T >> la.ilast) & 1u)) return false;
    return true;
  }
};

__global__ void k_mark_sources(const uint32_t* __restrict__ sources, const int* __restrict__ nsrc,
                               uint8_t* __restrict__ tsm) {
  const uint64_t n = static_cast<uint64_t>(*nsrc);
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    tsm[sources[i]] = 1;
}

// Number of alive entries of M[u] (excluding `skip`) -> outputs per item.
__global__ void k_row_alive(const uint32_t* __restrict__ items, uint64_t nitems, int stride, int pos,
                            const uint64_t* __restrict__ off, const uint32_t* __restrict__ malive,
                            uint32_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nitems; i += uint64_t(gridDim.x) * blockDim.x)
    out[i] = malive[items[i * stride + pos]];
}

// Level-1 tokens of path/cycle lines: (v, s, parent = s) for v in M[s].
__global__ void k_tp_init(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint64_t* __restrict__ obase,
                          const uint64_t* __restrict__ off, const uint32_t* __restrict__ mcol,
                          const uint8_t* __restrict__ mst, const uint32_t* __restrict__ mlen,
                          uint32_t* __restrict__ tu, uint32_t* __restrict__ ts, uint32_t* __restrict__ tp) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    uint64_t o = obase[i];
    const uint64_t b = off[s], L = mlen[s];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mst[e] & 1u)) continue;
      tu[o] = mcol[e];
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
                                  uint64_t nf, const uint64_t* __restrict__ off, const uint32_t* __restrict__ mcol,
                                  const uint8_t* __restrict__ mst, const uint32_t* __restrict__ mlen,
                                  const uint32_t* __restrict__ malive, uint32_t* __restrict__ cnt,
                                  unsigned long long* __restrict__ trav) {
  uint64_t t = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nf; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = static_cast<uint32_t>(fk[i] & 0xFFFFFFFFull);
    const uint32_t x = fx[i];
    const uint64_t b = off[u], L = mlen[u];
    uint32_t c = 0;
    for (uint64_t e = b; e < b + L; ++e)
      if ((mst[e] & 1u) && mcol[e] != x) ++c;
    cnt[i] = c;
    t += malive[u];
  }
  block_atomic_add(trav, t);
}

__global__ void k_tp_expand_write(const unsigned long long* __restrict__ fk, const uint32_t* __restrict__ fx,
                                  uint64_t nf, const uint64_t* __restrict__ obase, const uint64_t* __restrict__ off,
                                  const uint32_t* __restrict__ mcol, const uint8_t* __restrict__ mst,
                                  const uint32_t* __restrict__ mlen, uint32_t* __restrict__ tu,
                                  uint32_t* __restrict__ ts, uint32_t* __restrict__ tp) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nf; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = static_cast<uint32_t>(fk[i] & 0xFFFFFFFFull);
    const uint32_t s = static_cast<uint32_t>(fk[i] >> 32);
    const uint32_t x = fx[i];
    uint64_t o = obase[i];
    const uint64_t b = off[u], L = mlen[u];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mst[e] & 1u)) continue;
      const uint32_t w = mcol[e];
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
                              const uint16_t* __restrict__ tpub, const uint64_t* __restrict__ off,
                              const uint32_t* __restrict__ mcol, uint8_t* __restrict__ mst,
                              const uint32_t* __restrict__ mlen, uint8_t* __restrict__ tsm) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < ntok; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = tu[i], s = ts[i];
    if (!pos_ok(tpub[u], la.C + 1, la)) continue;
    if (!la.VC) {
      if (u == s) continue;
      if (tpub[s]) tsm[s] = 2;  // ack visitor needs an active source (nem_1.hpp:101, :326-336)
    } else {
      if (u != s) continue;
      tsm[s] = 2;
      // mark M[s][parent] (rows are sorted by neighbour id)
      const uint32_t p = tp[i];
      uint64_t lo = off[s], hi = off[s] + mlen[s];
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (mcol[mid] < p) lo = mid + 1; else hi = mid;
      }
      if (lo < off[s] + mlen[s] && mcol[lo] == p && (mst[lo] & 1u)) mst[lo] = 3;
    }
  }
}

// ---- TDS ----------------------------------------------------------------
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

__global__ void k_tds_init(const uint32_t* __restrict__ sources, uint64_t nsrc, const uint64_t* __restrict__ obase,
                           const uint64_t* __restrict__ off, const uint32_t* __restrict__ mcol,
                           const uint8_t* __restrict__ mst, const uint32_t* __restrict__ mlen, int stride,
                           uint32_t* __restrict__ walks) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nsrc; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = sources[i];
    uint64_t o = obase[i];
    const uint64_t b = off[s], L = mlen[s];
    for (uint64_t e = b; e < b + L; ++e) {
      if (!(mst[e] & 1u)) continue;
      walks[o * stride + 0] = s;
      walks[o * stride + 1] = mcol[e];
      ++o;
    }
  }
}

// Non-terminal position k: receiver checks, then sender-side filter per
// neighbour.  pass 0 counts, pass 1 writes.
template <int PASS>
__global__ void k_tds_expand(const uint32_t* __restrict__ win, uint64_t nw, int k, int stride, LineArgs la,
                             const uint16_t* __restrict__ tpub, const uint64_t* __restrict__ off,
                             const uint32_t* __restrict__ mcol, const uint8_t* __restrict__ mst,
                             const uint32_t* __restrict__ mlen, const uint32_t* __restrict__ malive,
                             uint32_t* __restrict__ cnt, const uint64_t* __restrict__ obase,
                             uint32_t* __restrict__ wout, unsigned long long* __restrict__ trav) {
  uint64_t t = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nw; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t* w = win + i * stride;
    const uint32_t u = w[k];
    uint32_t c = 0;
    if (pos_ok(tpub[u], k, la) && enum_ok(w, k, u, la)) {
      const uint32_t s = w[0];
      const uint64_t b = off[u], L = mlen[u];
      uint64_t o = PASS ? obase[i] : 0;
      for (uint64_t e = b; e < b + L; ++e) {
        if (!(mst[e] & 1u)) continue;
        const uint32_t nb = mcol[e];
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
        if (PASS) {
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

// Post-processing of unacked sources (beta.cpp:964-1000).
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
  hipcub::TransformInputIterator<uint64_t, hipcub::CastOp<uint64_t>, const uint32_t*> it(in, hipcub::CastOp<uint64_t>());
  size_t tmp = 0;
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, it, out + 1, static_cast<int>(n), c.stream));
  void* d_tmp = c.arena.get(tmp);
  PM_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(d_tmp, tmp, it, out + 1, static_cast<int>(n), c.stream));
  PM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(uint64_t), c.stream));
  uint64_t total = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&total, out + n, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  return total;
}

static void ensure_sources(Ctx& c, const LineArgs& la, int tds, unsigned long long* d_nsrc) {
  // previous line's sources are cleared from tsm first
  if (c.d_sources && c.nsources) {
    hipLaunchKernelGGL(k_clear_tsm, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                       c.nsources, c.d_tsm);
  }
  (void)d_nsrc;
  SourcePred pred{c.d_tpub[c.cur], la, tds};
  int* d_ns = arena_alloc<int>(c, 1);
  size_t tmp = 0;
  const int nitems = static_cast<int>(std::max<uint32_t>(c.nS_host, 1));
  PM_HIP_CHECK(hipMemsetAsync(d_ns, 0, sizeof(int), c.stream));
  if (c.nS_host) {
    PM_HIP_CHECK(hipcub::DeviceSelect::If(nullptr, tmp, c.d_slist, c.d_sources, d_ns, nitems, pred, c.stream));
    void* d_tmp = c.arena.get(tmp);
    PM_HIP_CHECK(hipcub::DeviceSelect::If(d_tmp, tmp, c.d_slist, c.d_sources, d_ns, nitems, pred, c.stream));
    hipLaunchKernelGGL(k_mark_sources, dim3(grid_for(c.nS_host, kBlock, 1024)), dim3(kBlock), 0, c.stream,
                       c.d_sources, d_ns, c.d_tsm);
    PM_HIP_CHECK(hipGetLastError());
  }
  int ns = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&ns, d_ns, sizeof(ns), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.nsources = static_cast<uint64_t>(ns);
}

TpResult run_path_line(Ctx& c, const NlcLine& line) {
  TpResult res;
  c.arena.reset();
  const LineArgs la = make_line_args(c, line);
  auto* d_nsrc = arena_alloc<unsigned long long>(c, 2);
  auto* d_trav = d_nsrc + 1;
  PM_HIP_CHECK(hipMemsetAsync(d_nsrc, 0, 2 * sizeof(unsigned long long), c.stream));
  ensure_sources(c, la, 0, d_nsrc);
  res.sources = c.nsources;
  if (c.nsources == 0) return res;
  const uint16_t* tpub = c.d_tpub[c.cur];
  // level 1 tokens
  auto* cnt = arena_alloc<uint32_t>(c, c.nsources);
  auto* obase = arena_alloc<uint64_t>(c, c.nsources + 1);
  hipLaunchKernelGGL(k_row_alive, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, 1, 0, c.d_off, c.d_malive, cnt);
  uint64_t ntok = exclusive_scan_u32_to_u64(c, cnt, obase, c.nsources);
  uint64_t trav_init = ntok;  // sources scan all of M[s]
  auto* tu = arena_alloc<uint32_t>(c, ntok);
  auto* ts = arena_alloc<uint32_t>(c, ntok);
  auto* tp = arena_alloc<uint32_t>(c, ntok);
  hipLaunchKernelGGL(k_tp_init, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, obase, c.d_off, c.d_mcol, c.d_mst, c.d_mlen, tu, ts, tp);
  PM_HIP_CHECK(hipGetLastError());
  res.tokens += ntok;
  SeenSet seen{};
  seen.count = 0;
  const int C = la.C;
  for (int k = 1; k <= C && ntok > 0; ++k) {
    auto* keys = arena_alloc<unsigned long long>(c, ntok);
    hipLaunchKernelGGL(k_tp_filter, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, tu, ts, ntok, k,
                       la, tpub, keys);
    auto* keys_s = arena_alloc<unsigned long long>(c, ntok);
    auto* par_s = arena_alloc<uint32_t>(c, ntok);
    size_t tmp = 0;
    PM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys, keys_s, tp, par_s, static_cast<int>(ntok), 0,
                                                    64, c.stream));
    void* d_tmp = c.arena.get(tmp);
    PM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp, keys, keys_s, tp, par_s, static_cast<int>(ntok), 0,
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
    PM_HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, tmp, keys_s, head, fk, d_nsel, static_cast<int>(ntok), c.stream));
    d_tmp = c.arena.get(tmp);
    PM_HIP_CHECK(hipcub::DeviceSelect::Flagged(d_tmp, tmp, keys_s, head, fk, d_nsel, static_cast<int>(ntok), c.stream));
    PM_HIP_CHECK(hipcub::DeviceSelect::Flagged(d_tmp, tmp, excl, head, fx, d_nsel, static_cast<int>(ntok), c.stream));
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
                       c.d_off, c.d_mcol, c.d_mst, c.d_mlen, c.d_malive, ecnt, d_trav);
    auto* eb = arena_alloc<uint64_t>(c, nf + 1);
    const uint64_t nnext = exclusive_scan_u32_to_u64(c, ecnt, eb, nf);
    tu = arena_alloc<uint32_t>(c, nnext);
    ts = arena_alloc<uint32_t>(c, nnext);
    tp = arena_alloc<uint32_t>(c, nnext);
    hipLaunchKernelGGL(k_tp_expand_write, dim3(grid_for(nf, kBlock, 1024)), dim3(kBlock), 0, c.stream, fk, fx, nf, eb,
                       c.d_off, c.d_mcol, c.d_mst, c.d_mlen, tu, ts, tp);
    PM_HIP_CHECK(hipGetLastError());
    ntok = nnext;
    res.tokens += ntok;
  }
  if (ntok > 0) {
    hipLaunchKernelGGL(k_tp_terminal, dim3(grid_for(ntok, kBlock, 1024)), dim3(kBlock), 0, c.stream, tu, ts, tp, ntok,
                       la, tpub, c.d_off, c.d_mcol, c.d_mst, c.d_mlen, c.d_tsm);
    PM_HIP_CHECK(hipGetLastError());
  }
  unsigned long long trav = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&trav, d_trav, sizeof(trav), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  res.edges = trav + trav_init;
  return res;
}

TpResult run_tds_line(Ctx& c, const NlcLine& line, std::vector<uint32_t>& walks_out, uint32_t& stride_out) {
  TpResult res;
  c.arena.reset();
  const LineArgs la = make_line_args(c, line);
  const int C = la.C;
  const int stride = C + 2;
  stride_out = static_cast<uint32_t>(stride);
  walks_out.clear();
  if (line.enumeration.size() < static_cast<size_t>(stride))
    throw std::runtime_error("pattern_non_local_constraint enumeration shorter than the TDS walk");
  auto* d_nsrc = arena_alloc<unsigned long long>(c, 2);
  auto* d_trav = d_nsrc + 1;
  PM_HIP_CHECK(hipMemsetAsync(d_nsrc, 0, 2 * sizeof(unsigned long long), c.stream));
  ensure_sources(c, la, 1, d_nsrc);
  res.sources = c.nsources;
  if (c.nsources == 0) return res;
  const uint16_t* tpub = c.d_tpub[c.cur];
  auto* cnt = arena_alloc<uint32_t>(c, c.nsources);
  auto* obase = arena_alloc<uint64_t>(c, c.nsources + 1);
  hipLaunchKernelGGL(k_row_alive, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, 1, 0, c.d_off, c.d_malive, cnt);
  uint64_t nw = exclusive_scan_u32_to_u64(c, cnt, obase, c.nsources);
  const uint64_t trav_init = nw;
  auto* walks = arena_alloc<uint32_t>(c, nw * stride);
  hipLaunchKernelGGL(k_tds_init, dim3(grid_for(c.nsources, kBlock, 4096)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, obase, c.d_off, c.d_mcol, c.d_mst, c.d_mlen, stride, walks);
  PM_HIP_CHECK(hipGetLastError());
  res.tokens += nw;
  for (int k = 1; k <= C && nw > 0; ++k) {
    auto* wc = arena_alloc<uint32_t>(c, nw);
    hipLaunchKernelGGL(k_tds_expand<0>, dim3(grid_for(nw, kBlock, 1024)), dim3(kBlock), 0, c.stream, walks, nw, k,
                       stride, la, tpub, c.d_off, c.d_mcol, c.d_mst, c.d_mlen, c.d_malive, wc,
                       static_cast<const uint64_t*>(nullptr), static_cast<uint32_t*>(nullptr), d_trav);
    auto* wb = arena_alloc<uint64_t>(c, nw + 1);
    const uint64_t nnext = exclusive_scan_u32_to_u64(c, wc, wb, nw);
    auto* wn = arena_alloc<uint32_t>(c, nnext * stride);
    if (nnext) {
      hipLaunchKernelGGL(k_tds_expand<1>, dim3(grid_for(nw, kBlock, 1024)), dim3(kBlock), 0, c.stream, walks, nw, k,
                         stride, la, tpub, c.d_off, c.d_mcol, c.d_mst, c.d_mlen, c.d_malive, wc, wb, wn, d_trav);
      PM_HIP_CHECK(hipGetLastError());
    }
    walks = wn;
    nw = nnext;
    res.tokens += nw;
  }
  if (nw > 0) {
    auto* keep = arena_alloc<uint8_t>(c, nw);
    hipLaunchKernelGGL(k_tds_terminal, dim3(grid_for(nw, kBlock, 1024)), dim3(kBlock), 0, c.stream, walks, nw, stride,
                       la, tpub, c.d_tsm, keep);
    PM_HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> all(nw * stride);
    std::vector<uint8_t> kp(nw);
    PM_HIP_CHECK(hipMemcpyAsync(all.data(), walks, nw * stride * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipMemcpyAsync(kp.data(), keep, nw, hipMemcpyDeviceToHost, c.stream));
    PM_HIP_CHECK(hipStreamSynchronize(c.stream));
    for (uint64_t i = 0; i < nw; ++i)
      if (kp[i]) walks_out.insert(walks_out.end(), all.begin() + i * stride, all.begin() + (i + 1) * stride);
  }
  res.walks = walks_out.size() / stride;
  unsigned long long trav = 0;
  PM_HIP_CHECK(hipMemcpyAsync(&trav, d_trav, sizeof(trav), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  res.edges = trav + trav_init;
  return res;
}

uint32_t launch_post_tp(Ctx& c, const NlcLine& line) {
  if (c.nsources == 0) return 0;
  auto* out = arena_alloc<unsigned long long>(c, 2);
  PM_HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_tp_post, dim3(grid_for(c.nsources, kBlock, 1024)), dim3(kBlock), 0, c.stream, c.d_sources,
                     c.nsources, c.d_tsm, c.d_tpub[c.cur], static_cast<int>(line.indices[0]), out);
  PM_HIP_CHECK(hipGetLastError());
  unsigned long long h[2] = {0, 0};
  PM_HIP_CHECK(hipMemcpyAsync(h, out, sizeof(h), hipMemcpyDeviceToHost, c.stream));
  PM_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.last_acked = h[0];
  return h[1] ? 1u : 0u;
}

}  // namespace pm
