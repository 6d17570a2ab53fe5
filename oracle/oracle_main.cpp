// ORACLE -- TEST INFRASTRUCTURE ONLY.  Standalone driver of the CPU restatement
// (pm_oracle.cpp, linked in): builds the symmetrized R-MAT graph of
// generate_rmat.cpp with the oracle's own generator and runs one full pattern
// search.  Exists so that the oracle can be built and run under
// -fsanitize=address,undefined (`make -C oracle sanitize`).
//
// usage: oracle_main SCALE P_GEN PATTERN_DIR [THREADS] [LABEL_ALPHABET]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

extern "C" {
struct oracle_stats_c {
  uint64_t iterations, terminated, lcc_edges, nlcc_edges, tds_edges, paths, final_vertices, final_edges;
  double seconds;
  uint64_t lcc_calls, supersteps;
};
int oracle_run_csr_mt(uint64_t n, const uint64_t* off, const uint32_t* col, const uint64_t* labels,
                      const char* pattern_dir, const char* result_dir, uint32_t nranks, uint64_t hub_threshold,
                      uint64_t max_iterations, uint32_t threads, oracle_stats_c* stats);
void oracle_rmat_rank(uint64_t scale, uint64_t p_gen, uint64_t rank, uint64_t count, uint64_t* us, uint64_t* vs);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s SCALE P_GEN PATTERN_DIR [THREADS] [LABEL_ALPHABET]\n", argv[0]);
    return 2;
  }
  const uint64_t scale = std::strtoull(argv[1], nullptr, 10), p_gen = std::strtoull(argv[2], nullptr, 10);
  const uint32_t threads = argc > 4 ? static_cast<uint32_t>(std::atoi(argv[4])) : 1;
  const uint64_t alphabet = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 0;
  const uint64_t n = 1ull << scale, per = (n * 16) / p_gen;
  std::vector<std::pair<uint64_t, uint64_t>> e;
  std::vector<uint64_t> us(per), vs(per);
  for (uint64_t r = 0; r < p_gen; ++r) {
    oracle_rmat_rank(scale, p_gen, r, per, us.data(), vs.data());
    for (uint64_t i = 0; i < per; ++i) {
      e.emplace_back(us[i], vs[i]);
      e.emplace_back(vs[i], us[i]);
    }
  }
  std::sort(e.begin(), e.end());
  std::vector<uint64_t> off(n + 1, 0);
  std::vector<uint32_t> col(e.size());
  for (size_t i = 0; i < e.size(); ++i) {
    ++off[e[i].first + 1];
    col[i] = static_cast<uint32_t>(e[i].second);
  }
  for (uint64_t v = 0; v < n; ++v) off[v + 1] += off[v];
  std::vector<uint64_t> labels;
  if (alphabet) {  // a small explicit alphabet (config C5 style)
    labels.resize(n);
    for (uint64_t v = 0; v < n; ++v) labels[v] = (v * 0x9E3779B97F4A7C15ull >> 40) % alphabet;
  }
  oracle_stats_c st{};
  const int rc = oracle_run_csr_mt(n, off.data(), col.data(), alphabet ? labels.data() : nullptr, argv[3], nullptr, 1,
                                   1048576, 100, threads, &st);
  if (rc) return 1;
  std::printf("iterations %llu lcc %llu nlcc %llu tds %llu paths %llu final |S| %llu |M| %llu\n",
              (unsigned long long)st.iterations, (unsigned long long)st.lcc_edges,
              (unsigned long long)st.nlcc_edges, (unsigned long long)st.tds_edges, (unsigned long long)st.paths,
              (unsigned long long)st.final_vertices, (unsigned long long)st.final_edges);
  return 0;
}
