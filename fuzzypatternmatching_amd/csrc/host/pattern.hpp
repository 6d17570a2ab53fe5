// Pattern-directory loaders for the label-constrained pattern-matching path.
//
// Reads <dir>/0/pattern_{edge,vertex_data,stat,nlc,non_local_constraint} with
// the same parse rules as the reference loaders:
//   * ::graph 5-arg ctor           include/havoqgt/graph.hpp:73-110
//     read_edge_list               include/havoqgt/graph.hpp:195-207
//     generate_vertex_list         include/havoqgt/graph.hpp:224-270
//     read_vertex_data_list        include/havoqgt/graph.hpp:181-193
//     read_stat                    include/havoqgt/graph.hpp:337-358
//   * pattern_util (nlc + enumeration)
//     read_pattern_list            include/havoqgt/pattern_util.hpp:172-210
//     read_pattern_enumeration_list_2  include/havoqgt/pattern_util.hpp:254-278
//     split<T>                     include/havoqgt/util.hpp:18-28
// Errors are thrown as std::runtime_error (the reference asserts or hits UB
// on the same malformed inputs).
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace pm {

static constexpr int kMaxTemplateVertices = 16;  // beta.cpp:270 max_bit_vector_size

inline std::string trim_copy(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

inline bool iequals(const std::string& a, const std::string& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
      return false;
  return true;
}

inline std::vector<std::string> split_str(const std::string& line, char delim) {
  std::vector<std::string> out;
  std::string tok;
  std::istringstream iss(line);
  while (std::getline(iss, tok, delim)) out.push_back(tok);
  return out;
}

// util.hpp:18-28: every token goes through std::stoull; an empty token (two
// consecutive delimiters) throws, exactly as in the reference.
inline std::vector<uint64_t> split_u64(const std::string& line, char delim) {
  std::vector<uint64_t> out;
  for (const auto& t : split_str(line, delim)) {
    size_t pos = 0;
    out.push_back(std::stoull(t, &pos));
  }
  return out;
}

struct PatternGraph {
  uint64_t vertex_count = 0;
  uint64_t edge_count = 0;
  uint64_t diameter = 0;
  std::vector<uint64_t> vertices;     // CSR offsets, vertex_count + 1
  std::vector<uint64_t> edges;        // CSR targets
  std::vector<uint64_t> vertex_data;  // template labels (one per line of pattern_vertex_data)
  uint16_t adj[kMaxTemplateVertices] = {0};  // adj[t] = bitmask of template neighbours of t
};

struct NlcLine {
  std::vector<uint64_t> labels;    // L[0..C+1]
  std::vector<uint64_t> indices;   // I[0..C+1]
  uint64_t cycle_length = 0;       // C
  bool valid_cycle = false;        // VC
  bool interleave_lp = false;      // IL
  bool selected_vertices = false;  // SV
  std::vector<uint64_t> enumeration;  // E[0..C+1] (pattern_non_local_constraint)
  std::vector<uint8_t> aggregation;
};

struct Pattern {
  PatternGraph graph;
  std::vector<NlcLine> lines;
};

inline std::ifstream open_or_throw(const std::string& path) {
  std::ifstream f(path, std::ifstream::in);
  if (!f.is_open()) throw std::runtime_error("cannot open pattern file: " + path);
  return f;
}

// graph.hpp:195-207 + 224-270 (+ the 5-arg ctor order at :73-110).
inline PatternGraph load_pattern_graph(const std::string& base) {
  PatternGraph g;
  std::vector<std::pair<uint64_t, uint64_t>> edge_list;
  {
    auto f = open_or_throw(base + "_edge");
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream iss(line);
      uint64_t s = 0, t = 0;
      iss >> s >> t;
      g.edges.push_back(t);
      edge_list.emplace_back(s, t);
    }
  }
  g.edge_count = g.edges.size();
  if (edge_list.empty()) throw std::runtime_error("pattern_edge is empty");
  // generate_vertex_list: walks the (source-sorted) edge list; an index past the
  // end of the list never matches the current vertex (the reference reads past
  // the end there, which is undefined; this is the only defined reading).
  {
    const uint64_t max_vertex = edge_list.back().first;
    uint64_t vertex_count = 0, l = 0, degree = 0, current = 0;
    std::vector<uint64_t> vertex_degree;
    do {
      const bool in_range = l < edge_list.size();
      if (in_range && edge_list[l].first == current) {
        ++degree;
        ++l;
      } else {
        g.vertices.push_back(g.vertices.empty() ? 0 : vertex_degree.back() + g.vertices.back());
        vertex_degree.push_back(degree);
        degree = 0;
        ++vertex_count;
        current = vertex_count;
      }
    } while (current <= max_vertex);
    g.vertices.push_back(g.vertices.empty() ? 0 : vertex_degree.back() + g.vertices.back());
    g.vertex_count = vertex_count;
  }
  {
    auto f = open_or_throw(base + "_vertex_data");
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream iss(line);
      uint64_t v = 0, d = 0;
      iss >> v >> d;
      g.vertex_data.push_back(d);
    }
  }
  {
    auto f = open_or_throw(base + "_stat");
    std::string line;
    while (std::getline(f, line)) {
      auto toks = split_str(line, ':');
      if (toks.size() < 2) continue;
      if (iequals(trim_copy(toks[0]), "diameter")) g.diameter = std::stoull(trim_copy(toks[1]));
    }
  }
  if (g.vertex_data.size() > static_cast<size_t>(kMaxTemplateVertices))
    throw std::runtime_error("pattern has more than 16 template vertices");
  if (g.vertex_data.size() > g.vertex_count)
    throw std::runtime_error("pattern_vertex_data lists more vertices than pattern_edge defines");
  for (uint64_t t = 0; t < g.vertex_data.size(); ++t) {
    uint16_t m = 0;
    for (uint64_t e = g.vertices[t]; e < g.vertices[t + 1]; ++e) {
      if (g.edges[e] >= static_cast<uint64_t>(kMaxTemplateVertices))
        throw std::runtime_error("pattern edge target >= 16");
      m |= static_cast<uint16_t>(1u << g.edges[e]);
    }
    g.adj[t] = m;
  }
  return g;
}

// pattern_util.hpp:172-210 and :254-278.
inline std::vector<NlcLine> load_nlc(const std::string& nlc_path, const std::string& enum_path) {
  std::vector<NlcLine> lines;
  {
    auto f = open_or_throw(nlc_path);
    std::string line;
    while (std::getline(f, line)) {
      auto toks = split_str(line, ':');
      if (toks.size() < 6) throw std::runtime_error("pattern_nlc line needs 6 ':' fields: '" + line + "'");
      for (int i = 0; i < 6; ++i) toks[i] = trim_copy(toks[i]);
      NlcLine l;
      l.labels = split_u64(toks[0], ' ');
      l.indices = split_u64(toks[1], ' ');
      l.cycle_length = std::stoull(toks[2]);
      l.valid_cycle = std::stoull(toks[3]) != 0;
      l.interleave_lp = std::stoull(toks[4]) != 0;
      l.selected_vertices = std::stoull(toks[5]) != 0;
      lines.push_back(std::move(l));
    }
  }
  {
    auto f = open_or_throw(enum_path);
    std::string line;
    size_t i = 0;
    while (std::getline(f, line)) {
      line = trim_copy(line);
      auto toks = split_str(line, ':');
      if (toks.size() < 3) throw std::runtime_error("pattern_non_local_constraint line needs 3 fields");
      if (i < lines.size()) {
        lines[i].enumeration = split_u64(trim_copy(toks[1]), ' ');
        for (auto x : split_u64(trim_copy(toks[2]), ' ')) lines[i].aggregation.push_back(static_cast<uint8_t>(x));
      }
      ++i;
    }
  }
  for (auto& l : lines) {
    const size_t n = l.cycle_length + 2;
    if (l.labels.size() < n || l.indices.size() < n)
      throw std::runtime_error("pattern_nlc line shorter than cycle_length + 2");
    for (size_t k = 0; k < n; ++k)
      if (l.indices[k] >= static_cast<uint64_t>(kMaxTemplateVertices))
        throw std::runtime_error("pattern_nlc template index >= 16");
    if (n > 16) throw std::runtime_error("walks longer than 16 positions are not supported (tds_batch_1.hpp:964)");
  }
  return lines;
}

inline Pattern load_pattern_dir(const std::string& dir) {
  // beta.cpp:433-475: only pattern set element 0 is read.
  const std::string base = dir + "/0/pattern";
  Pattern p;
  p.graph = load_pattern_graph(base);
  p.lines = load_nlc(base + "_nlc", base + "_non_local_constraint");
  return p;
}

}  // namespace pm
