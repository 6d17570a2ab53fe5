// Host-side CSR construction, the repo's own graph file format and label input.
//
// The reference keeps its graph in per-rank Boost.Interprocess segments
// (include/havoqgt/distributed_db.hpp:191-272, file name <base>_<rank>_of_<P>
// at :353-357) built by delegate_partitioned_graph (impl/delegate_partitioned_
// graph.ipp:818-969).  That layout cannot be read without Boost; this file
// defines the MI355X build's format under the same names: one file per rank,
// each holding the rows of the vertices that rank owns (owner = id % P, hubs
// at sorted-hub-index % P, ipp:346-355), rows sorted by target so duplicate
// entries are adjacent (the device code relies on that).
//
// Semantics kept from the reference:
//   * the CSR holds every directed edge with multiplicity, self loops included
//     (no dedup anywhere in ipp:818-969);
//   * degree(v) = out-degree with multiplicity (ipp:1767-1781);
//   * -b copies backup -> input before opening (distributed_db.hpp:106-182),
//     guarded here against copying a file onto itself (the reference's -i
//     falls through into -b, beta.cpp:105-110, and truncates the input).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <fcntl.h>
#include <fstream>
#include <memory>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <regex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "rmat.hpp"

namespace pm {

struct Csr {
  uint64_t n = 0;              // number of vertex ids (max id + 1)
  std::vector<uint64_t> off;   // n + 1
  std::vector<uint32_t> col;   // targets, sorted within each row
  bool symmetric = false;      // every (u,v) has a matching (v,u) with equal multiplicity
};

inline unsigned hw_threads() {
  unsigned t = std::thread::hardware_concurrency();
  if (t == 0) t = 1;
  if (t > 64) t = 64;
  return t;
}

template <typename F>
inline void parallel_for(uint64_t n, unsigned threads, F&& f) {
  if (threads <= 1 || n < 4096) {
    f(uint64_t(0), n);
    return;
  }
  std::vector<std::thread> pool;
  const uint64_t chunk = (n + threads - 1) / threads;
  for (unsigned t = 0; t < threads; ++t) {
    const uint64_t b = std::min<uint64_t>(n, t * chunk), e = std::min<uint64_t>(n, b + chunk);
    if (b >= e) break;
    pool.emplace_back([&f, b, e] { f(b, e); });
  }
  for (auto& th : pool) th.join();
}

// Builds a row-sorted CSR from a list of directed (src,dst) pairs.
inline Csr build_csr(uint64_t n, const std::vector<std::pair<uint32_t, uint32_t>>& pairs,
                     bool symmetric, unsigned threads = hw_threads()) {
  Csr g;
  g.n = n;
  g.symmetric = symmetric;
  std::vector<std::atomic<uint64_t>> deg(n);
  for (auto& d : deg) d.store(0, std::memory_order_relaxed);
  parallel_for(pairs.size(), threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) deg[pairs[i].first].fetch_add(1, std::memory_order_relaxed);
  });
  g.off.assign(n + 1, 0);
  for (uint64_t v = 0; v < n; ++v) g.off[v + 1] = g.off[v] + deg[v].load(std::memory_order_relaxed);
  g.col.assign(g.off[n], 0);
  for (uint64_t v = 0; v < n; ++v) deg[v].store(g.off[v], std::memory_order_relaxed);
  parallel_for(pairs.size(), threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint64_t pos = deg[pairs[i].first].fetch_add(1, std::memory_order_relaxed);
      g.col[pos] = pairs[i].second;
    }
  });
  parallel_for(n, threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t v = b; v < e; ++v) std::sort(g.col.begin() + g.off[v], g.col.begin() + g.off[v + 1]);
  });
  return g;
}

// The streams of generator ranks `vranks` (of P_gen), symmetrized, in rank
// order: 2 * 2^S * 16 / P_gen directed pairs per rank (generate_rmat.cpp:202-213),
// written through emit(index, u, v).
template <typename Emit>
inline uint64_t rmat_stream_of(uint64_t scale, uint64_t p_gen, const std::vector<uint64_t>& vranks, Emit&& emit,
                               unsigned threads = hw_threads()) {
  if (scale > 32) throw std::runtime_error("scale > 32 not supported (u32 vertex ids)");
  if (p_gen == 0) throw std::runtime_error("P_gen must be positive");
  for (uint64_t r : vranks)
    if (r >= p_gen) throw std::runtime_error("generator rank out of range");
  const uint64_t per_rank = rmat_edges_per_rank(scale, p_gen);
  std::atomic<uint64_t> next(0);
  auto worker = [&] {
    for (;;) {
      const uint64_t i = next.fetch_add(1);
      if (i >= vranks.size()) break;
      RmatStream s(rmat_seed(vranks[i]), scale);
      const uint64_t base = 2 * per_rank * i;
      for (uint64_t e = 0; e < per_rank; ++e) {
        auto uv = s.next_edge();
        emit(base + 2 * e, static_cast<uint32_t>(uv.first), static_cast<uint32_t>(uv.second));
        emit(base + 2 * e + 1, static_cast<uint32_t>(uv.second), static_cast<uint32_t>(uv.first));
      }
    }
  };
  std::vector<std::thread> pool;
  const unsigned nt = std::max<unsigned>(1, std::min<unsigned>(threads, static_cast<unsigned>(vranks.size())));
  for (unsigned t = 0; t < nt; ++t) pool.emplace_back(worker);
  for (auto& th : pool) th.join();
  return 2 * per_rank * vranks.size();
}

inline std::vector<std::pair<uint32_t, uint32_t>> rmat_pairs_of(uint64_t scale, uint64_t p_gen,
                                                                const std::vector<uint64_t>& vranks,
                                                                unsigned threads = hw_threads()) {
  std::vector<std::pair<uint32_t, uint32_t>> pairs(2 * rmat_edges_per_rank(scale, std::max<uint64_t>(p_gen, 1)) *
                                                   vranks.size());
  rmat_stream_of(scale, p_gen, vranks, [&](uint64_t i, uint32_t u, uint32_t v) { pairs[i] = {u, v}; }, threads);
  return pairs;
}

// All P_gen generator ranks' streams, symmetrized: 2 * 2^S * 16 directed pairs.
inline std::vector<std::pair<uint32_t, uint32_t>> rmat_pairs(uint64_t scale, uint64_t p_gen,
                                                             unsigned threads = hw_threads()) {
  std::vector<uint64_t> all(p_gen);
  for (uint64_t r = 0; r < p_gen; ++r) all[r] = r;
  return rmat_pairs_of(scale, p_gen, all, threads);
}

inline Csr build_rmat_csr(uint64_t scale, uint64_t p_gen, unsigned threads = hw_threads()) {
  auto pairs = rmat_pairs(scale, p_gen, threads);
  return build_csr(uint64_t(1) << scale, pairs, /*symmetric=*/true, threads);
}

// ---------------------------------------------------------------------------
// Ownership (delegate partitioning) -- only used to name per-rank output files.
// owner(v) = v % P; hubs (out-degree >= threshold, ipp:508) are numbered in
// sorted id order (ipp:680-681) and controlled by hub_index % P (ipp:346-355).
struct Ownership {
  uint32_t nranks = 1;
  std::vector<uint64_t> hubs;  // sorted hub ids
  uint32_t owner(uint64_t v) const {
    if (!hubs.empty()) {
      auto it = std::lower_bound(hubs.begin(), hubs.end(), v);
      if (it != hubs.end() && *it == v) return static_cast<uint32_t>((it - hubs.begin()) % nranks);
    }
    return static_cast<uint32_t>(v % nranks);
  }
};

inline Ownership make_ownership(const Csr& g, uint32_t nranks, uint64_t hub_threshold) {
  Ownership o;
  o.nranks = nranks == 0 ? 1 : nranks;
  for (uint64_t v = 0; v < g.n; ++v)
    if (g.off[v + 1] - g.off[v] >= hub_threshold) o.hubs.push_back(v);
  return o;
}

// ---------------------------------------------------------------------------
// Graph files: <base>_<rank>_of_<P>.
static constexpr char kGraphMagic[8] = {'P', 'M', 'C', 'S', 'R', '0', '1', '\0'};

struct GraphFileHeader {
  char magic[8];
  uint64_t n;            // global vertex-id count
  uint64_t rank, nranks;
  uint64_t hub_threshold;
  uint64_t symmetric;
  uint64_t nrows;        // rows stored in this file
  uint64_t nnz;          // entries stored in this file
};

inline std::string graph_file_name(const std::string& base, uint64_t rank, uint64_t nranks) {
  return base + "_" + std::to_string(rank) + "_of_" + std::to_string(nranks);
}

inline void write_graph_files(const std::string& base, const Csr& g, uint32_t nranks, uint64_t hub_threshold) {
  const Ownership own = make_ownership(g, nranks, hub_threshold);
  for (uint32_t r = 0; r < own.nranks; ++r) {
    std::vector<uint64_t> rows;
    uint64_t nnz = 0;
    for (uint64_t v = 0; v < g.n; ++v)
      if (own.owner(v) == r) {
        rows.push_back(v);
        nnz += g.off[v + 1] - g.off[v];
      }
    GraphFileHeader h{};
    std::memcpy(h.magic, kGraphMagic, 8);
    h.n = g.n;
    h.rank = r;
    h.nranks = own.nranks;
    h.hub_threshold = hub_threshold;
    h.symmetric = g.symmetric ? 1 : 0;
    h.nrows = rows.size();
    h.nnz = nnz;
    const std::string path = graph_file_name(base, r, own.nranks);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot create graph file " + path);
    std::fwrite(&h, sizeof(h), 1, f);
    std::fwrite(rows.data(), sizeof(uint64_t), rows.size(), f);
    std::vector<uint64_t> deg(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) deg[i] = g.off[rows[i] + 1] - g.off[rows[i]];
    std::fwrite(deg.data(), sizeof(uint64_t), deg.size(), f);
    for (size_t i = 0; i < rows.size(); ++i)
      std::fwrite(g.col.data() + g.off[rows[i]], sizeof(uint32_t), deg[i], f);
    std::fclose(f);
  }
}

inline bool file_exists(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f) return false;
  std::fclose(f);
  return true;
}

// distributed_db::transfer(backup, input), distributed_db.hpp:106-182: copy
// every <backup>_<r>_of_<P> over <input>_<r>_of_<P>.
inline void transfer_graph_files(const std::string& from, const std::string& to) {
  if (from == to) return;  // guard: the reference would truncate its own input here
  for (uint64_t nranks = 1; nranks <= 4096; ++nranks) {
    if (!file_exists(graph_file_name(from, 0, nranks))) continue;
    for (uint64_t r = 0; r < nranks; ++r) {
      const std::string src = graph_file_name(from, r, nranks), dst = graph_file_name(to, r, nranks);
      std::ifstream in(src, std::ios::binary);
      if (!in) throw std::runtime_error("missing backup graph file " + src);
      std::ofstream out(dst, std::ios::binary | std::ios::trunc);
      if (!out) throw std::runtime_error("cannot write graph file " + dst);
      out << in.rdbuf();
    }
    return;
  }
  throw std::runtime_error("no backup graph files found for base " + from);
}

// A graph file mapped read-only (the reference maps its per-rank segments,
// distributed_db.hpp:191-272): header, row ids, degrees and the rows' entries
// are read in place, with no staging copy of the file.
class MappedGraphFile {
 public:
  explicit MappedGraphFile(const std::string& path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("missing graph file " + path);
    struct stat st{};
    if (::fstat(fd_, &st) != 0 || st.st_size < static_cast<off_t>(sizeof(GraphFileHeader))) {
      ::close(fd_);
      throw std::runtime_error("not a graph file: " + path);
    }
    size_ = static_cast<size_t>(st.st_size);
    void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) {
      ::close(fd_);
      throw std::runtime_error("cannot map graph file " + path);
    }
    ::madvise(p, size_, MADV_SEQUENTIAL);
    base_ = static_cast<const char*>(p);
    std::memcpy(&h_, base_, sizeof(h_));
    const uint64_t need = sizeof(h_) + 16 * h_.nrows + 4 * h_.nnz;
    if (std::memcmp(h_.magic, kGraphMagic, 8) != 0) {
      unmap();
      throw std::runtime_error("not a graph file: " + path);
    }
    if (size_ < need) {
      unmap();
      throw std::runtime_error("truncated graph file " + path);
    }
  }
  ~MappedGraphFile() { unmap(); }
  MappedGraphFile(const MappedGraphFile&) = delete;
  MappedGraphFile& operator=(const MappedGraphFile&) = delete;
  const GraphFileHeader& header() const { return h_; }
  // unaligned-safe element reads (the sections follow a 64-B header: aligned in practice)
  const uint64_t* rows() const { return reinterpret_cast<const uint64_t*>(base_ + sizeof(h_)); }
  const uint64_t* degrees() const { return rows() + h_.nrows; }
  const uint32_t* cols() const { return reinterpret_cast<const uint32_t*>(degrees() + h_.nrows); }

 private:
  void unmap() {
    if (base_) ::munmap(const_cast<char*>(base_), size_);
    if (fd_ >= 0) ::close(fd_);
    base_ = nullptr;
    fd_ = -1;
  }
  int fd_ = -1;
  size_t size_ = 0;
  const char* base_ = nullptr;
  GraphFileHeader h_{};
};

// Reads every <base>_<r>_of_<P> file (mapped) and assembles the global CSR.
inline Csr read_graph_files(const std::string& base, uint32_t* nranks_out = nullptr,
                            uint64_t* hub_threshold_out = nullptr) {
  uint64_t nranks = 0;
  for (uint64_t p = 1; p <= 4096; ++p)
    if (file_exists(graph_file_name(base, 0, p))) {
      nranks = p;
      break;
    }
  if (nranks == 0) throw std::runtime_error("no graph files found for base " + base);
  Csr g;
  std::vector<std::unique_ptr<MappedGraphFile>> files;
  uint64_t hub_threshold = 0;
  for (uint64_t r = 0; r < nranks; ++r) {
    files.emplace_back(new MappedGraphFile(graph_file_name(base, r, nranks)));
    const GraphFileHeader& h = files.back()->header();
    if (r == 0) {
      g.n = h.n;
      g.symmetric = h.symmetric != 0;
      hub_threshold = h.hub_threshold;
    } else if (h.n != g.n || h.nranks != nranks) {
      throw std::runtime_error("graph file " + graph_file_name(base, r, nranks) + " belongs to another graph");
    }
  }
  std::vector<uint64_t> deg(g.n, 0);
  for (const auto& f : files) {
    const GraphFileHeader& h = f->header();
    const uint64_t* rows = f->rows();
    const uint64_t* d = f->degrees();
    for (uint64_t i = 0; i < h.nrows; ++i) {
      if (rows[i] >= g.n) throw std::runtime_error("graph file row id out of range");
      deg[rows[i]] = d[i];
    }
  }
  g.off.assign(g.n + 1, 0);
  for (uint64_t v = 0; v < g.n; ++v) g.off[v + 1] = g.off[v] + deg[v];
  g.col.resize(g.off[g.n]);
  for (const auto& f : files) {  // each row straight from the mapping to its CSR slot
    const GraphFileHeader& h = f->header();
    const uint64_t* rows = f->rows();
    const uint64_t* d = f->degrees();
    const uint32_t* c = f->cols();
    uint64_t pos = 0;
    for (uint64_t i = 0; i < h.nrows; ++i) {
      if (pos + d[i] > h.nnz) throw std::runtime_error("truncated graph file");
      std::memcpy(g.col.data() + g.off[rows[i]], c + pos, d[i] * sizeof(uint32_t));
      pos += d[i];
    }
  }
  if (nranks_out) *nranks_out = static_cast<uint32_t>(nranks);
  if (hub_threshold_out) *hub_threshold_out = hub_threshold;
  return g;
}

// P of the graph files of `base` (the first <base>_0_of_<P> found), 0 when there are none.
inline uint32_t graph_file_partitions(const std::string& base) {
  for (uint64_t p = 1; p <= 4096; ++p)
    if (file_exists(graph_file_name(base, 0, p))) return static_cast<uint32_t>(p);
  return 0;
}

// The header of <base>_0_of_<P> (vertex count, P, hub threshold, symmetric flag).
inline GraphFileHeader graph_file_header(const std::string& base) {
  const uint32_t P = graph_file_partitions(base);
  if (P == 0) throw std::runtime_error("no graph files found for base " + base);
  MappedGraphFile f(graph_file_name(base, 0, P));
  return f.header();
}

// One shard of a sharded search, read from the graph files.  The reference's rank r opens only
// <base>_<r>_of_<P> (distributed_db.hpp:353-357, beta.cpp:209-223) because its files ARE the partition; the
// search's partition here is owner = id % nshards with a delegate's row (global degree >= the hub threshold)
// split by target owner (delegate_partitioned_graph.ipp:1402-1648), which the files (a delegate's whole row at
// its controller) do not hold as such.  So every file's row index and degrees are read (16 B per row: the
// global degrees every shard needs for labels and the delegate rule), and only the entries this shard holds
// are copied out of the mappings: owned rows whole, delegate rows filtered by target.  nshards may differ
// from the files' P.
struct ShardCsr {
  uint64_t n = 0;
  std::vector<uint64_t> off;     // n + 1 by id: the rows held here, every other row empty
  std::vector<uint32_t> col;     // their entries, sorted within each row (>= 1 element)
  std::vector<uint32_t> degree;  // n global degrees
  bool symmetric = false;
  uint32_t nranks = 1;           // P of the files (result-file attribution)
  uint64_t hub_threshold = 0;
};

inline ShardCsr read_graph_shard(const std::string& base, uint32_t nshards, uint32_t shard,
                                 unsigned threads = hw_threads()) {
  if (nshards == 0 || shard >= nshards) throw std::runtime_error("read_graph_shard: bad shard index");
  const uint32_t P = graph_file_partitions(base);
  if (P == 0) throw std::runtime_error("no graph files found for base " + base);
  ShardCsr s;
  s.nranks = P;
  std::vector<std::unique_ptr<MappedGraphFile>> files;
  for (uint32_t r = 0; r < P; ++r) {
    files.emplace_back(new MappedGraphFile(graph_file_name(base, r, P)));
    const GraphFileHeader& h = files.back()->header();
    if (r == 0) {
      s.n = h.n;
      s.symmetric = h.symmetric != 0;
      s.hub_threshold = h.hub_threshold;
    } else if (h.n != s.n || h.nranks != P) {
      throw std::runtime_error("graph file " + graph_file_name(base, r, P) + " belongs to another graph");
    }
  }
  const uint64_t n = s.n;
  // global degrees and, for every row this shard may hold, where its entries lie: file << 48 | entry index
  s.degree.assign(n, 0);
  std::vector<uint64_t> loc(n, ~uint64_t(0));
  for (uint32_t r = 0; r < P; ++r) {
    const GraphFileHeader& h = files[r]->header();
    const uint64_t* rows = files[r]->rows();
    const uint64_t* d = files[r]->degrees();
    uint64_t pos = 0;
    for (uint64_t i = 0; i < h.nrows; ++i) {
      const uint64_t v = rows[i];
      if (v >= n) throw std::runtime_error("graph file row id out of range");
      if (d[i] > 0xFFFFFFFFull) throw std::runtime_error("degree above 2^32");
      if (pos + d[i] > h.nnz) throw std::runtime_error("truncated graph file");
      s.degree[v] = static_cast<uint32_t>(d[i]);
      loc[v] = (uint64_t(r) << 48) | pos;
      pos += d[i];
    }
  }
  const bool split = nshards > 1;
  auto is_hub = [&](uint64_t v) { return split && s.degree[v] >= s.hub_threshold; };
  auto row = [&](uint64_t v) { return files[loc[v] >> 48]->cols() + (loc[v] & ((uint64_t(1) << 48) - 1)); };
  // entries held per row: an owned row whole, a delegate row's entries whose target this shard owns
  std::vector<uint64_t> held(n, 0);
  parallel_for(n, threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t v = b; v < e; ++v) {
      if (!s.degree[v]) continue;
      if (is_hub(v)) {
        const uint32_t* c = row(v);
        uint64_t k = 0;
        for (uint64_t j = 0; j < s.degree[v]; ++j) k += c[j] % nshards == shard;
        held[v] = k;
      } else if (v % nshards == shard) {
        held[v] = s.degree[v];
      }
    }
  });
  s.off.assign(n + 1, 0);
  for (uint64_t v = 0; v < n; ++v) s.off[v + 1] = s.off[v] + held[v];
  held.clear();
  held.shrink_to_fit();
  s.col.resize(std::max<uint64_t>(s.off[n], 1));
  if (!s.off[n]) s.col[0] = 0;
  parallel_for(n, threads, [&](uint64_t b, uint64_t e) {
    for (uint64_t v = b; v < e; ++v) {
      if (s.off[v + 1] == s.off[v]) continue;
      const uint32_t* c = row(v);
      uint32_t* out = s.col.data() + s.off[v];
      if (is_hub(v)) {
        for (uint64_t j = 0; j < s.degree[v]; ++j)
          if (c[j] % nshards == shard) *out++ = c[j];
      } else {
        std::memcpy(out, c, uint64_t(s.degree[v]) * sizeof(uint32_t));
      }
    }
  });
  return s;
}

// ---------------------------------------------------------------------------
// Labels.
// Default: label = ceil(log2(degree + 1)) (vertex_data_db_degree.hpp:109),
// which equals bit_width(degree) for every degree < 2^52.
inline uint64_t degree_label(uint64_t degree) {
  uint64_t w = 0;
  while (degree) {
    ++w;
    degree >>= 1;
  }
  return w;
}

// -v <prefix>: every regular file in dirname(prefix) whose name matches
// basename(prefix).* (vertex_data_db.hpp:137-165, 197-257); lines "vid label";
// vertices not listed keep 0.  A line that fails to parse yields the entry
// (0, 0), exactly like the reference's `iss >> v >> d` on zero-initialised
// values (vertex_data_db.hpp:176-185).  Files are applied in sorted name order.
inline std::vector<std::string> vertex_label_files(const std::string& prefix) {
  std::string dir = ".", wildcard = prefix;
  const size_t slash = prefix.find_last_of('/');
  if (slash != std::string::npos) {
    dir = prefix.substr(0, slash);
    if (dir.empty()) dir = "/";
    wildcard = prefix.substr(slash + 1);
  }
  std::vector<std::string> files;
  const std::regex filter(wildcard + ".*");
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* ent = readdir(d)) {
      const std::string name = ent->d_name;
      if (name == "." || name == "..") continue;
      const std::string full = dir + "/" + name;
      std::ifstream probe(full);
      if (!probe.good()) continue;
      if (ent->d_type == DT_DIR) continue;
      if (std::regex_match(name, filter)) files.push_back(full);
    }
    closedir(d);
  }
  if (files.empty()) throw std::runtime_error("no vertex label files match " + prefix);
  std::sort(files.begin(), files.end());
  return files;
}

// Host loader (tests and host-only tools; the product CLI parses on the GPU,
// pm_vertex_data_files / pm_ingest.hip).
inline std::vector<uint64_t> load_vertex_labels(const std::string& prefix, uint64_t n) {
  const std::vector<std::string> files = vertex_label_files(prefix);
  std::vector<uint64_t> labels(n, 0);
  for (const auto& path : files) {
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream iss(line);
      uint64_t v = 0, d = 0;
      iss >> v >> d;
      if (v < n) labels[v] = d;
    }
  }
  return labels;
}

}  // namespace pm
