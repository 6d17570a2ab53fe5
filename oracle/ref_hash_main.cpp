// ORACLE -- TEST INFRASTRUCTURE ONLY.
// Prints hash_nbits golden vectors using the reference's own
// include/havoqgt/detail/hash.hpp (Boost-free), compiled in place by
// `make -C oracle ref`.  Output: "<x> <n> <hash_nbits(x,n)>" per line.
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <havoqgt/detail/hash.hpp>

int main() {
  const int ns[] = {17, 18, 20, 21, 24, 26, 28, 30, 31, 32, 33, 40};
  const uint64_t xs[] = {0, 1, 2, 3, 12345, 65535, 65536, 1000003, 123456789, 2147483647ull, 4294967295ull};
  for (int n : ns)
    for (uint64_t x : xs) {
      uint64_t in = (n < 64) ? (x & ((uint64_t(1) << n) - 1)) : x;
      std::printf("%llu %d %llu\n", (unsigned long long)in, n,
                  (unsigned long long)havoqgt::detail::hash_nbits(in, n));
    }
  return 0;
}
