// Host-side checks of the superstep-0 layout rules (pm_internal.hpp):
// degree classes, the slot -> row divisor, the row-start masks of a tile for
// every 16-B alignment shift, and the 2-bit T_pub code.  Exit 0 on success.
#include <cstdio>
#include <cstdlib>

#include "pm_internal.hpp"

using namespace pm;

static uint32_t tpub_code_ref(uint32_t T, uint32_t tu) {  // restated from the definition
  int n = 0;
  uint32_t b[16];
  for (int t = 0; t < 16; ++t)
    if ((tu >> t) & 1u) b[n++] = 1u << t;
  if (n > 2) return T ? 3u : 0u;
  uint32_t c = 0;
  if (n > 0 && (T & b[0])) c |= 1u;
  if (n > 1 && (T & b[1])) c |= 2u;
  return c;
}

#define CHECK(x)                                             \
  do {                                                       \
    if (!(x)) {                                              \
      std::fprintf(stderr, "FAILED %s (line %d)\n", #x, __LINE__); \
      return 1;                                              \
    }                                                        \
  } while (0)

int main() {
  // classes: monotone, G >= degree, G of the previous class < degree
  uint32_t prev = 0;
  for (uint64_t d = 1; d <= kLightMax; ++d) {
    const uint32_t k = light_kind(d), g = kind_slots(k);
    CHECK(k < static_cast<uint32_t>(kHeavyKind));
    CHECK(k >= prev);
    CHECK(g >= d);
    CHECK(k == 0 || kind_slots(k - 1) < d);
    CHECK(padded_degree(d) == g);
    prev = k;
  }
  CHECK(padded_degree(0) == 0);
  CHECK(padded_degree(kLightMax + 1) == kLightMax + 1);
  CHECK(light_kind(kLightMax) == static_cast<uint32_t>(kHeavyKind) - 1);
  // tiles: rpt * g <= kTileEntries - 4 (room for the alignment shift), exact division
  for (uint32_t k = 0; k < static_cast<uint32_t>(kHeavyKind); ++k) {
    const uint32_t g = kind_slots(k), rpt = (kTileEntries - 4) / g, rdiv = ((1u << 19) + g - 1) / g;
    CHECK(rpt >= 1 && rpt * g <= kTileEntries - 4);
    for (uint32_t sl = 0; sl < kTileEntries; ++sl) CHECK(((sl * rdiv) >> 19) == sl / g);
    // row-start bits for each shift: every row start of the tile lands in the two 16-B loads
    for (uint32_t sh = 0; sh < 4; ++sh) {
      uint32_t starts = 0;
      for (uint32_t sl = 0; sl < rpt * g; sl += g) {
        const uint32_t o = sl + sh;
        CHECK(o / 256 < 2);
        ++starts;
      }
      CHECK(starts == rpt);
    }
  }
  // 2-bit T_pub code against a restatement, every label template set of up to 4 bits and every subset
  for (uint32_t tu = 1; tu < (1u << 8); ++tu)
    for (uint32_t T = 0; T < (1u << 8); ++T) {
      if (T & ~tu) continue;
      CHECK(tpub_code(T, tu) == tpub_code_ref(T, tu));
      CHECK((tpub_code(T, tu) == 0) == (T == 0));
    }
  std::printf("layout checks passed\n");
  return 0;
}
