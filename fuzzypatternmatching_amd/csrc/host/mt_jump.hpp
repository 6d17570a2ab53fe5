// MT19937 jump-ahead over GF(2): the host half of the GPU R-MAT generator.
//
// The reference draws every R-MAT edge of generator rank r from ONE
// sequential boost::mt19937 stream (seed 5489 + 3r, src/generate_rmat.cpp:202-205;
// 5*S draws per edge, rmat_edge_generator.hpp:218-246).  To generate a stream
// on many CUs at once it is cut into substreams whose start states are
// obtained by jumping the engine ahead instead of stepping it.
//
// State.  std::mt19937 keeps the window W_k = (x_k, ..., x_{k+623}) of its
// word sequence x_t (x_0..x_623 = the seeded array); output m is
// temper(x_{624+m}) and x_{t+624} = x_{t+397} ^ twist(x_t upper, x_{t+1} lower).
// The window slide T (one output) is linear over GF(2).  Only 19937 of the
// window's bits matter (the low 31 bits of x_k are never read), and on those
// T acts with the characteristic polynomial phi(x) of degree 19937.  Hence
// W_{k+J} = p(T) W_k on every bit that matters, with p = x^J mod phi, and
//   p(T) W_k = XOR_{i : p_i = 1} W_{k+i},   i.e.   word j = XOR_i p_i x_{k+i+j}.
//
// phi comes from Berlekamp-Massey on 2 * 19937 output bits (the minimal
// polynomial of any nonzero output-bit sequence is phi, which is primitive
// for MT19937); x^J mod phi by square-and-multiply-by-x.  Everything here is
// host C++; the GPU applies p (pm_rmat.hip).
#pragma once

#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace pm {
namespace mtj {

static constexpr int kN = 624, kM = 397;
static constexpr int kDeg = 19937;
static constexpr int kWords = (kDeg + 64) / 64;  // 312 words hold bits 0..19936 (and bit 19937 of phi)

inline uint32_t twist(uint32_t a, uint32_t b) {  // (x_t upper | x_{t+1} lower) A
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

inline uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// W_0: the seeded array of std::mt19937(seed).
inline void seed_window(uint32_t seed, uint32_t* w) {
  w[0] = seed;
  for (int i = 1; i < kN; ++i) w[i] = 1812433253u * (w[i - 1] ^ (w[i - 1] >> 30)) + static_cast<uint32_t>(i);
}

// x_k .. x_{k+len-1} from the window W_k (len >= 624).
inline void extend(const uint32_t* w, uint32_t* seq, size_t len) {
  for (int i = 0; i < kN; ++i) seq[i] = w[i];
  for (size_t t = kN; t < len; ++t) seq[t] = seq[t - (kN - kM)] ^ twist(seq[t - kN], seq[t - kN + 1]);
}

using Poly = std::vector<uint64_t>;  // bit i = coefficient of x^i

inline bool bit(const Poly& p, size_t i) { return i / 64 < p.size() && ((p[i / 64] >> (i % 64)) & 1u); }

inline size_t degree(const Poly& p) {
  for (size_t w = p.size(); w-- > 0;)
    if (p[w]) return w * 64 + 63 - __builtin_clzll(p[w]);
  return 0;
}

// Berlekamp-Massey over GF(2): connection polynomial C (C_0 = 1) of the bits.
inline Poly berlekamp_massey(const std::vector<uint8_t>& s, size_t& L_out) {
  const size_t n = s.size();
  const size_t W = n / 64 + 2;
  Poly C(W, 0), B(W, 0), Tmp;
  C[0] = B[0] = 1;
  size_t L = 0, m = 1;
  // r = s reversed, packed: bit t of r = s[n-1-t]; then sum_{i=1..L} C_i s[k-i]
  // is the parity of C & (r >> (n-1-k)) over bits 1..L.
  Poly r(W + 1, 0);
  for (size_t t = 0; t < n; ++t)
    if (s[n - 1 - t]) r[t / 64] |= 1ull << (t % 64);
  auto r_word = [&](size_t base, size_t k) -> uint64_t {  // 64 bits of r starting at base + 64k
    const size_t b = base + 64 * k, wi = b / 64, off = b % 64;
    uint64_t x = wi < r.size() ? r[wi] >> off : 0;
    if (off && wi + 1 < r.size()) x |= r[wi + 1] << (64 - off);
    return x;
  };
  for (size_t k = 0; k < n; ++k) {
    const size_t base = n - 1 - k;  // bit i of the window = s[k - i]
    uint64_t acc = 0;
    const size_t nw = L / 64 + 1;
    for (size_t w = 0; w < nw; ++w) acc ^= C[w] & r_word(base, w);
    uint32_t d = static_cast<uint32_t>(__builtin_popcountll(acc) & 1);  // includes i = 0: C_0 s[k]
    if (!d) {
      ++m;
      continue;
    }
    // C ^= B << m
    const bool grow = 2 * L <= k;
    if (grow) Tmp = C;
    const size_t ws = m / 64, bs = m % 64;
    for (size_t w = W; w-- > ws;) {
      uint64_t x = B[w - ws] << bs;
      if (bs && w - ws >= 1) x |= B[w - ws - 1] >> (64 - bs);
      C[w] ^= x;
    }
    if (grow) {
      L = k + 1 - L;
      B.swap(Tmp);
      m = 1;
    } else {
      ++m;
    }
  }
  L_out = L;
  return C;
}

// phi(x) = x^L C(1/x): the characteristic polynomial of the window slide.
inline const Poly& char_poly() {
  static Poly phi;
  static std::once_flag once;
  std::call_once(once, [] {
    const size_t nbits = 2 * kDeg + 64;
    std::vector<uint32_t> w(kN), seq(kN + nbits + 1);
    seed_window(5489u, w.data());
    extend(w.data(), seq.data(), seq.size());
    std::vector<uint8_t> s(nbits);
    for (size_t i = 0; i < nbits; ++i) s[i] = temper(seq[kN + i]) & 1u;
    size_t L = 0;
    const Poly C = berlekamp_massey(s, L);
    if (L != static_cast<size_t>(kDeg)) throw std::runtime_error("MT19937 linear complexity is not 19937");
    Poly p(kWords, 0);
    for (size_t i = 0; i <= L; ++i)
      if (bit(C, L - i)) p[i / 64] |= 1ull << (i % 64);
    phi = p;
  });
  return phi;
}

// a mod phi for a of degree < 2 * kDeg (in place).
inline void reduce(Poly& a) {
  const Poly& phi = char_poly();
  for (size_t t = a.size() * 64; t-- > static_cast<size_t>(kDeg);) {
    if (!bit(a, t)) continue;
    const size_t sh = t - kDeg, ws = sh / 64, bs = sh % 64;
    for (size_t w = 0; w < phi.size(); ++w) {
      const uint64_t x = phi[w];
      if (!x) continue;
      if (w + ws < a.size()) a[w + ws] ^= x << bs;
      if (bs && w + ws + 1 < a.size()) a[w + ws + 1] ^= x >> (64 - bs);
    }
  }
  a.resize(kWords);
}

inline Poly square_mod(const Poly& a) {
  Poly s(2 * kWords, 0);
  for (size_t w = 0; w < a.size(); ++w) {
    uint64_t x = a[w];
    uint64_t lo = 0, hi = 0;
    for (int b = 0; b < 32; ++b) {
      lo |= ((x >> b) & 1ull) << (2 * b);
      hi |= ((x >> (b + 32)) & 1ull) << (2 * b);
    }
    s[2 * w] = lo;
    s[2 * w + 1] = hi;
  }
  reduce(s);
  return s;
}

inline Poly times_x_mod(const Poly& a) {
  Poly s(kWords + 1, 0);
  for (size_t w = 0; w < a.size(); ++w) {
    s[w] |= a[w] << 1;
    s[w + 1] |= a[w] >> 63;
  }
  reduce(s);
  return s;
}

// x^J mod phi.
inline Poly jump_poly(uint64_t J) {
  Poly r(kWords, 0);
  r[0] = 1;
  for (int b = 63; b >= 0; --b) {
    r = square_mod(r);
    if ((J >> b) & 1ull) r = times_x_mod(r);
  }
  return r;
}

// Host application of p to W_k (checker and small jumps): W_{k+J}.
inline void apply(const Poly& p, const uint32_t* w, uint32_t* out) {
  std::vector<uint32_t> seq(kDeg + kN);
  extend(w, seq.data(), seq.size());
  for (int j = 0; j < kN; ++j) out[j] = 0;
  for (size_t i = 0; i < static_cast<size_t>(kDeg); ++i)
    if (bit(p, i))
      for (int j = 0; j < kN; ++j) out[j] ^= seq[i + j];
}

}  // namespace mtj
}  // namespace pm
