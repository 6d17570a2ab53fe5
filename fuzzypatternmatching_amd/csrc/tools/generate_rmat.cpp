// generate_rmat -- R-MAT graph builder with the reference CLI
// (src/generate_rmat.cpp:78-150, 196-213): -s scale (17), -d delegate
// threshold (1048576), -o output base (required), -b backup base, -p/-f/-c
// accepted and ignored (Boost.Interprocess partitioning knobs).
// The reference generates one stream per MPI rank (seed 5489+3r, 2^S*16/P
// edges); this single process emulates P generator ranks with -n P (default
// 1) and writes P per-rank files <base>_<r>_of_<P>.
#include <getopt.h>

#include <iostream>
#include <string>

#include "../host/graph_store.hpp"

int main(int argc, char** argv) {
  uint64_t scale = 17, threshold = 1048576, nranks = 1;
  std::string out, backup;
  bool help = false, found = false;
  int c;
  std::cout << "CMD line:";
  for (int i = 0; i < argc; ++i) std::cout << " " << argv[i];
  std::cout << std::endl;
  while ((c = getopt(argc, argv, "s:d:o:b:p:f:c:n:h ")) != -1) {
    switch (c) {
      case 'h': help = true; break;
      case 's': scale = std::atoll(optarg); break;
      case 'd': threshold = std::atoll(optarg); break;
      case 'o': found = true; out = optarg; break;
      case 'b': backup = optarg; break;
      case 'p': case 'f': case 'c': break;
      case 'n': nranks = std::atoll(optarg); break;
      default: std::cerr << "Unrecognized option: " << char(c) << ", ignore." << std::endl; help = true; break;
    }
  }
  if (help || !found || nranks == 0) {
    std::cerr << "Usage: -s <int> -d <int> -o <string> [-b <string>] [-n <generator ranks>]\n";
    return 255;
  }
  try {
    pm::Csr g = pm::build_rmat_csr(scale, nranks);
    uint64_t maxdeg = 0;
    for (uint64_t v = 0; v < g.n; ++v) maxdeg = std::max<uint64_t>(maxdeg, g.off[v + 1] - g.off[v]);
    pm::write_graph_files(out, g, static_cast<uint32_t>(nranks), threshold);
    std::cout << "Graph Ready: " << g.n << " vertices, " << g.off[g.n] << " directed edges, Max Degree = " << maxdeg
              << std::endl;
    if (!backup.empty()) pm::transfer_graph_files(out, backup);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
