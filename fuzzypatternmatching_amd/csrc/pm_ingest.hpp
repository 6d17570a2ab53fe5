// GPU text ingest (pm_ingest.hip): edge lists and -v label files parsed in HBM.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "pm_rmat.hpp"

namespace pm {

struct IngestCsr {
  DevCsr fwd;               // out-rows, sorted, with multiplicity (caller frees d_off / d_col)
  DevCsr rev;               // in-rows (only when !symmetric and want_rev)
  bool symmetric = true;    // every (u,v) has a matching (v,u) with equal multiplicity
  uint64_t lines = 0;       // text lines seen
  uint64_t bytes = 0;       // text bytes uploaded
};

// ingest_edge_list.cpp:164-240 over parallel_edge_list_reader.hpp:242-266:
// "src dst [weight]" lines, -u 1 adds (dst, src) for every edge.
IngestCsr ingest_edges_device(const std::vector<std::string>& files, bool undirected, bool want_rev,
                              hipStream_t stream);

// vertex_data_db.hpp:176-185, 197-257: "vid label" lines applied in file order
// (last write wins), vertices not listed keep 0; d_labels holds n entries.
void labels_from_files_device(const std::vector<std::string>& files, uint64_t n, uint64_t* d_labels,
                              hipStream_t stream);

}  // namespace pm
