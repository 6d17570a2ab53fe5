// R-MAT edge stream, bit-compatible with the reference generator.
//
//   * generate_edge        include/havoqgt/rmat_edge_generator.hpp:218-261
//   * iterator get_next    include/havoqgt/rmat_edge_generator.hpp:127-139
//     (edge e is emitted as (u,v) then (v,u); edges 0..count-1 are emitted)
//   * hash_nbits           include/havoqgt/detail/hash.hpp:65-145
//   * per-rank seed/count  src/generate_rmat.cpp:202-205
//       seed = 5489 + 3*rank, count = 2^S * 16 / P_gen, a,b,c,d = .57,.19,.19,.05
//
// RNG: boost::mt19937 == std::mt19937 (same recurrence and integer seeding);
// boost::uniform_01<mt19937> (Boost 1.57, backward-compatible class) returns
// x * 2^-32 for each 32-bit engine output x.  That uniform_01 mapping is
// restated from Boost's published implementation (Boost is not in the image:
// "parity unpinned" for that one step).
//
// All floating point here must be evaluated without FMA contraction
// (compile with -ffp-contract=off), exactly as x86-64 SSE2 code does.
#pragma once

#include <cstdint>
#include <random>
#include <utility>

namespace pm {

inline uint32_t hash32(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}

inline uint16_t hash16(uint16_t a) {
  // uint16_t arithmetic promotes to int and truncates on assignment.
  a = static_cast<uint16_t>((a + 0x5d16) + (a << 6));
  a = static_cast<uint16_t>((a ^ 0xc23c) ^ (a >> 9));
  a = static_cast<uint16_t>((a + 0x67b1) + (a << 5));
  a = static_cast<uint16_t>((a + 0x646c) ^ (a << 7));
  a = static_cast<uint16_t>((a + 0x46c5) + (a << 3));
  a = static_cast<uint16_t>((a ^ 0x4f09) ^ (a >> 8));
  return a;
}

inline uint64_t shifted_n_hash32(uint64_t input, int n) {
  uint64_t to_hash = (input >> n) & 0xFFFFFFFFull;
  to_hash = hash32(static_cast<uint32_t>(to_hash));
  const uint64_t mask = 0xFFFFFFFFull << n;
  return (input & ~mask) | (to_hash << n);
}

inline uint64_t shifted_n_hash16(uint64_t input, int n) {
  uint64_t to_hash = (input >> n) & 0xFFFFull;
  to_hash = hash16(static_cast<uint16_t>(to_hash));
  const uint64_t mask = 0xFFFFull << n;
  return (input & ~mask) | (to_hash << n);
}

// hash.hpp:115-145.  For n < 16 the reference's assert is compiled out in
// Release builds and the loops do not execute (identity).
inline uint64_t hash_nbits(uint64_t input, int n) {
  if (n == 32) {
    input = hash32(static_cast<uint32_t>(input));
  } else if (n > 32) {
    n -= 32;
    for (int i = 0; i <= n; ++i) input = shifted_n_hash32(input, i);
    for (int i = n; i >= 0; --i) input = shifted_n_hash32(input, i);
  } else {
    n -= 16;
    for (int i = 0; i <= n; ++i) input = shifted_n_hash16(input, i);
    for (int i = n; i >= 0; --i) input = shifted_n_hash16(input, i);
  }
  return input;
}

class RmatStream {
 public:
  RmatStream(uint64_t seed, uint64_t scale, double a = 0.57, double b = 0.19, double c = 0.19,
             double d = 0.05, bool scramble = true)
      : rng_(static_cast<std::mt19937::result_type>(seed)),
        scale_(scale), a_(a), b_(b), c_(c), d_(d), scramble_(scramble) {}

  double u01() { return static_cast<double>(rng_()) * (1.0 / 4294967296.0); }

  // rmat_edge_generator.hpp:218-261 (one undirected edge; the caller emits
  // (u,v) then (v,u) when symmetrizing).
  std::pair<uint64_t, uint64_t> next_edge() {
    double ra = a_, rb = b_, rc = c_, rd = d_;
    uint64_t u = 0, v = 0;
    uint64_t step = (uint64_t(1) << scale_) / 2;
    for (uint64_t j = 0; j < scale_; ++j) {
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
      const double S = ra + rb + rc + rd;
      ra /= S;
      rb /= S;
      rc /= S;
      rd = 1. - ra - rb - rc;
    }
    if (scramble_) {
      u = hash_nbits(u, static_cast<int>(scale_));
      v = hash_nbits(v, static_cast<int>(scale_));
    }
    return {u, v};
  }

 private:
  std::mt19937 rng_;
  uint64_t scale_;
  double a_, b_, c_, d_;
  bool scramble_;
};

// generate_rmat.cpp:202-205
inline uint64_t rmat_seed(uint64_t rank) { return uint64_t(5489) + rank * 3ull; }
inline uint64_t rmat_edges_per_rank(uint64_t scale, uint64_t p_gen) {
  return (uint64_t(1) << scale) * 16 / p_gen;
}

}  // namespace pm
