// run_pattern_matching_beta -- drop-in CLI for the MI355X pattern-matching path.
//
// Same options and result directory as src/run_pattern_matching_beta.cpp
// (getopt "i:b:v:e:p:o:x:h ", :82-142), one process driving one gfx950 GPU
// through the C-ABI of include/pm_abi.h.  Per-rank result files are written
// for the P the graph files were created with (<base>_<r>_of_<P>).
//
// Kept quirks: -i falls through into -b (beta.cpp:105-110), so `-i X` alone
// also sets the backup base to X -- the transfer is then skipped instead of
// truncating X onto itself; -e and -x are accepted and ignored.
// Extensions (not in the reference): environment PM_MAX_ITERATIONS caps the
// do/while loop (the reference can loop forever, SURVEY.md A.6 hazard 11) and
// PM_DEVICE selects the GPU.
#include <getopt.h>

#include <bitset>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "../../../include/pm_abi.h"
#include "../host/graph_store.hpp"

static void usage() {
  std::cerr << "Usage: -i <string> -p <string> -o <string>\n"
            << " -i <string>   - input graph base filename (required)\n"
            << " -b <string>   - backup graph base filename. If set, \"input\" graph will be deleted if it exists\n"
            << " -v <string>   - vertex metadata base filename (optional, Default is degree based metadata)\n"
            << " -e <string>   - edge metadata base filename (optional)\n"
            << " -p <string>   - pattern base directory (required)\n"
            << " -o <string>   - output base directory (required)\n"
            << " -x <int>      - Token Passing batch size (optional)\n"
            << " -h            - print help and exit\n\n";
}

int main(int argc, char** argv) {
  std::string graph_input, backup_input, vertex_metadata, edge_metadata, pattern_dir, result_dir;
  std::cout << "CMD Line :";
  for (int i = 0; i < argc; ++i) std::cout << " " << argv[i];
  std::cout << std::endl;
  bool help = false;
  std::bitset<3> required;
  int c;
  while ((c = getopt(argc, argv, "i:b:v:e:p:o:x:h ")) != -1) {
    switch (c) {
      case 'h':
        help = true;
        break;
      case 'i':
        graph_input = optarg;
        required.set(0);
        // fall through (beta.cpp:105-110)
      case 'b':
        backup_input = optarg;
        break;
      case 'v':
        vertex_metadata = optarg;
        break;
      case 'e':
        edge_metadata = optarg;
        break;
      case 'p':
        pattern_dir = optarg;
        required.set(1);
        break;
      case 'o':
        result_dir = optarg;
        required.set(2);
        break;
      case 'x':
        (void)std::stoull(optarg);
        break;
      default:
        std::cerr << "Unrecognized Option : " << char(c) << ", Ignore." << std::endl;
        help = true;
        break;
    }
  }
  if (help || !required.all()) {
    usage();
    return 255;  // exit(-1)
  }
  try {
    if (!backup_input.empty()) pm::transfer_graph_files(backup_input, graph_input);
    uint64_t *off = nullptr, n = 0, hub = 0;
    uint32_t *col = nullptr, nranks = 1;
    int symmetric = 1;
    std::cout << "Loading Graph ... " << std::endl;
    if (pm_read_graph(graph_input.c_str(), &off, &col, &n, &symmetric, &nranks, &hub) != 0) {
      std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
      return 1;
    }
    std::cout << "Done Loading Graph. " << n << " vertices, " << off[n] << " directed edges, " << nranks
              << " partition(s)." << std::endl;
    pm_graph_desc d{n, off, col, symmetric, nranks, hub};
    const char* dev = std::getenv("PM_DEVICE");
    pm_ctx* ctx = pm_create(&d, pattern_dir.c_str(), dev ? std::atoi(dev) : 0);
    if (!ctx) {
      std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
      return 1;
    }
    if (!vertex_metadata.empty()) {
      // parsed on the GPU (pm_ingest.hip); PM_HOST_LABELS=1 takes the host loader instead
      if (std::getenv("PM_HOST_LABELS")) {
        std::vector<uint64_t> labels = pm::load_vertex_labels(vertex_metadata, n);
        if (pm_vertex_data_set(ctx, labels.data()) != 0) throw std::runtime_error(pm_last_error(ctx));
      } else if (pm_vertex_data_files(ctx, vertex_metadata.c_str()) != 0) {
        throw std::runtime_error(pm_last_error(ctx));
      }
    }
    const char* mi = std::getenv("PM_MAX_ITERATIONS");
    pm_run_stats st{};
    if (pm_run_beta(ctx, result_dir.c_str(), mi ? std::strtoull(mi, nullptr, 10) : 0, &st) != 0)
      throw std::runtime_error(pm_last_error(ctx));
    std::cout << "Fuzzy Pattern Matching Time | Pattern [0] : " << st.seconds << std::endl;
    std::cout << "Fuzzy Pattern Matching | Pattern [0] | # Iterations : " << st.iterations
              << (st.terminated ? "" : " (stopped by PM_MAX_ITERATIONS)") << std::endl;
    std::cout << "Active vertices " << st.final_vertices << ", active edges " << st.final_edges << ", walks "
              << st.walks << ", edges traversed " << (st.lcc_edges + st.nlcc_edges + st.tds_edges) << std::endl;
    pm_destroy(ctx);
    pm_free_host(off);
    pm_free_host(col);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
