// ingest_edge_list -- text edge lists to graph files, reference CLI
// (src/ingest_edge_list.cpp:82-162): -o output base (required), -b backup,
// -d delegate threshold, -u <0|1> symmetrize, -p/-f/-c ignored, then files.
// Lines are "src dst [weight]" (parallel_edge_list_reader.hpp:242-266); the
// weight is unused on the pattern-matching path.  Blank or unparsable lines
// are skipped (the reference reads uninitialised values there).  Extension:
// -n P writes P per-rank files (the reference: one per MPI rank); -g <device>
// parses the text and builds the CSR on that GPU (pm_ingest_edge_list_gpu,
// same graph as the host path).
#include <getopt.h>

#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../host/graph_store.hpp"
#include "../../../include/pm_abi.h"

int main(int argc, char** argv) {
  std::string out, backup;
  uint64_t threshold = 1048576, nranks = 1;
  bool undirected = false, help = false, found = false;
  int gpu = -1;
  int c;
  while ((c = getopt(argc, argv, "o:d:p:f:c:b:u:n:g:h ")) != -1) {
    switch (c) {
      case 'h': help = true; break;
      case 'd': threshold = std::atoll(optarg); break;
      case 'o': found = true; out = optarg; break;
      case 'b': backup = optarg; break;
      case 'p': case 'f': case 'c': break;
      case 'u': undirected = std::atoi(optarg) != 0; break;
      case 'n': nranks = std::atoll(optarg); break;
      case 'g': gpu = std::atoi(optarg); break;
      default: std::cerr << "Unrecognized option: " << char(c) << ", ignore." << std::endl; help = true; break;
    }
  }
  if (help || !found) {
    std::cerr << "Usage: -o <string> -d <int> [-u 0|1] [-n ranks] [-g device] [file ...]\n";
    return 255;
  }
  try {
    if (gpu >= 0) {
      std::vector<const char*> files;
      for (int i = optind; i < argc; ++i) files.push_back(argv[i]);
      uint64_t *off = nullptr, n = 0;
      uint32_t* col = nullptr;
      int sym = 0;
      if (pm_ingest_edge_list_gpu(files.data(), static_cast<uint32_t>(files.size()), undirected ? 1 : 0, gpu, &off,
                                  &col, &n, &sym) != 0)
        throw std::runtime_error(pm_last_error(nullptr));
      pm::Csr g;
      g.n = n;
      g.off.assign(off, off + n + 1);
      g.col.assign(col, col + g.off[n]);
      g.symmetric = sym != 0;
      pm_free_host(off);
      pm_free_host(col);
      pm::write_graph_files(out, g, static_cast<uint32_t>(nranks), threshold);
      std::cout << "Graph Ready: " << n << " vertices, " << g.off[n] << " directed edges, symmetric="
                << g.symmetric << " (GPU ingest)" << std::endl;
      if (!backup.empty()) pm::transfer_graph_files(out, backup);
      return 0;
    }
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    uint64_t maxv = 0;
    for (int i = optind; i < argc; ++i) {
      std::ifstream f(argv[i]);
      if (!f) {
        std::cerr << "Error opening filename: " << argv[i] << std::endl;
        continue;
      }
      std::string line;
      while (std::getline(f, line)) {
        std::istringstream ss(line);
        uint64_t s, t;
        if (!(ss >> s >> t)) continue;
        if (s > 0xFFFFFFFEull || t > 0xFFFFFFFEull) throw std::runtime_error("vertex id exceeds 32 bits");
        maxv = std::max(maxv, std::max(s, t));
        pairs.emplace_back(static_cast<uint32_t>(s), static_cast<uint32_t>(t));
        if (undirected) pairs.emplace_back(static_cast<uint32_t>(t), static_cast<uint32_t>(s));
      }
    }
    const uint64_t n = pairs.empty() ? 0 : maxv + 1;
    pm::Csr g = pm::build_csr(n, pairs, undirected);
    if (!undirected) {  // detect symmetric input anyway (rows are sorted)
      bool sym = true;
      for (uint64_t v = 0; v < n && sym; ++v)
        for (uint64_t e = g.off[v]; e < g.off[v + 1] && sym; ++e) {
          const uint32_t u = g.col[e];
          const auto b = g.col.begin() + g.off[u], en = g.col.begin() + g.off[u + 1];
          const auto cf = std::count(g.col.begin() + g.off[v], g.col.begin() + g.off[v + 1], u);
          const auto cr = std::count(b, en, static_cast<uint32_t>(v));
          sym = cf == cr;
        }
      g.symmetric = sym;
    }
    pm::write_graph_files(out, g, static_cast<uint32_t>(nranks), threshold);
    std::cout << "Graph Ready: " << n << " vertices, " << g.off[n] << " directed edges, symmetric="
              << g.symmetric << std::endl;
    if (!backup.empty()) pm::transfer_graph_files(out, backup);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
