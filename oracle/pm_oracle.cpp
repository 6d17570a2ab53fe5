// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of HavoqGT's run_pattern_matching_beta hot path, used by
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
// checker.  Nothing in the product (fuzzypatternmatching_amd/) links, loads
// or calls this file.
//
// It mirrors the reference's data structures and control flow for ONE MPI
// rank owning every vertex (the reference results are partition independent,
// SURVEY.md Appendix A.5; per-rank result files are then re-split by the
// reference owner rule).  Citations are file:line under the reference tree:
//   driver loop            src/run_pattern_matching_beta.cpp:544-1351
//   LCC superstep          include/havoqgt/label_propagation_pattern_matching_nonunique_ee.hpp
//                            lppm_visitor::pre_visit 149-459, ::visit 468-636,
//                            member verify_and_update_vertex_state 647-816,
//                            global verify_and_update_vertex_state 829-1027,
//                            label_propagation_pattern_matching_bsp 1033-1153
//   NLCC path/cycle        include/havoqgt/token_passing_pattern_matching_nonunique_nem_1.hpp
//                            pre_visit 99-303, visit 312-861, driver 913-939
//   NLCC TDS               include/havoqgt/token_passing_pattern_matching_nonunique_tds_batch_1.hpp
//                            pre_visit 123-335, visit 348-919, driver 976-1324
//   init traversal order   include/havoqgt/visitor_queue.hpp:221-251, queue_visitor 395-411
//   pattern files          include/havoqgt/graph.hpp:73-385, pattern_util.hpp:172-278, util.hpp:18-28
//   R-MAT                  include/havoqgt/rmat_edge_generator.hpp:127-139, 218-261;
//                          include/havoqgt/detail/hash.hpp:65-145; src/generate_rmat.cpp:202-205
//
// Parity status: pinned by (a) hash_nbits golden vectors generated from the
// reference's own detail/hash.hpp (oracle/_ref), (b) the std::mt19937
// known answer, (c) hand-built known-answer graphs (tests/golden), and
// (d) the reference's grid-graph CSR fixture.  LCC/NLCC outputs have no
// reference-produced fixture (examples/results/** are empty placeholders):
// that part is "parity unpinned" by reference outputs, see DESIGN.md.
//
// Build: make -C oracle   (g++ -O2 -ffp-contract=off -shared -fPIC)

#include <algorithm>
#include <bitset>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------
// MT19937 written out from its published definition (so the oracle does not
// share the product's std::mt19937 usage).  Known answer: the 10000th output
// of the default-seeded (5489) engine is 4123659995.
class Mt19937 {
 public:
  explicit Mt19937(uint32_t seed) {
    mt_[0] = seed;
    for (int i = 1; i < 624; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + static_cast<uint32_t>(i);
    idx_ = 624;
  }
  uint32_t next() {
    if (idx_ >= 624) twist();
    uint32_t y = mt_[idx_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

 private:
  void twist() {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (mt_[i] & 0x80000000u) | (mt_[(i + 1) % 624] & 0x7fffffffu);
      uint32_t v = mt_[(i + 397) % 624] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908b0dfu;
      mt_[i] = v;
    }
    idx_ = 0;
  }
  uint32_t mt_[624];
  int idx_;
};

static uint32_t h32(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}
static uint16_t h16(uint16_t a) {
  a = (uint16_t)((a + 0x5d16) + (a << 6));
  a = (uint16_t)((a ^ 0xc23c) ^ (a >> 9));
  a = (uint16_t)((a + 0x67b1) + (a << 5));
  a = (uint16_t)((a + 0x646c) ^ (a << 7));
  a = (uint16_t)((a + 0x46c5) + (a << 3));
  a = (uint16_t)((a ^ 0x4f09) ^ (a >> 8));
  return a;
}
static uint64_t hash_nbits(uint64_t x, int n) {
  auto s32 = [](uint64_t in, int k) {
    uint64_t t = h32((uint32_t)((in >> k) & 0xFFFFFFFFull));
    uint64_t m = 0xFFFFFFFFull << k;
    return (in & ~m) | (t << k);
  };
  auto s16 = [](uint64_t in, int k) {
    uint64_t t = h16((uint16_t)((in >> k) & 0xFFFFull));
    uint64_t m = 0xFFFFull << k;
    return (in & ~m) | (t << k);
  };
  if (n == 32) return h32((uint32_t)x);
  if (n > 32) {
    n -= 32;
    for (int i = 0; i <= n; ++i) x = s32(x, i);
    for (int i = n; i >= 0; --i) x = s32(x, i);
    return x;
  }
  n -= 16;
  for (int i = 0; i <= n; ++i) x = s16(x, i);
  for (int i = n; i >= 0; --i) x = s16(x, i);
  return x;
}

// rmat_edge_generator.hpp:218-261 with boost::uniform_01<mt19937> = x / 2^32.
static void rmat_edges(uint64_t scale, uint64_t seed, uint64_t count, uint64_t* us, uint64_t* vs) {
  Mt19937 rng((uint32_t)seed);
  auto g = [&rng]() { return (double)rng.next() / 4294967296.0; };
  for (uint64_t e = 0; e < count; ++e) {
    double a = 0.57, b = 0.19, c = 0.19, d = 0.05;
    uint64_t u = 0, v = 0, step = (uint64_t(1) << scale) / 2;
    for (uint64_t j = 0; j < scale; ++j) {
      double p = g();
      if (p < a) {
      } else if (p >= a && p < a + b) {
        v += step;
      } else if (p >= a + b && p < a + b + c) {
        u += step;
      } else {
        u += step;
        v += step;
      }
      step /= 2;
      a *= 0.9 + 0.2 * g();
      b *= 0.9 + 0.2 * g();
      c *= 0.9 + 0.2 * g();
      d *= 0.9 + 0.2 * g();
      double S = a + b + c + d;
      a /= S;
      b /= S;
      c /= S;
      d = 1. - a - b - c;
    }
    us[e] = hash_nbits(u, (int)scale);
    vs[e] = hash_nbits(v, (int)scale);
  }
}

// ---------------------------------------------------------------------------
// Pattern files (graph.hpp / pattern_util.hpp restatement).
static std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && isspace((unsigned char)s[b])) ++b;
  while (e > b && isspace((unsigned char)s[e - 1])) --e;
  return s.substr(b, e - b);
}
static std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> out;
  std::string t;
  std::istringstream iss(s);
  while (std::getline(iss, t, d)) out.push_back(t);
  return out;
}
static std::vector<uint64_t> split_u64(const std::string& s, char d) {
  std::vector<uint64_t> out;
  for (auto& t : split(s, d)) out.push_back(std::stoull(t));
  return out;
}

struct Nlc {
  std::vector<uint64_t> L, I, E;
  uint64_t C = 0;
  bool VC = false, IL = false, SV = false;
};

struct Pattern {
  std::vector<uint64_t> vertices, edges, vdata;
  uint64_t vertex_count = 0, edge_count = 0, diameter = 0;
  std::vector<Nlc> nlc;
  uint16_t adj(size_t t) const {
    uint16_t m = 0;
    for (uint64_t e = vertices[t]; e < vertices[t + 1]; ++e) m |= (uint16_t)(1u << edges[e]);
    return m;
  }
};

static Pattern load_pattern(const std::string& dir) {
  Pattern p;
  const std::string base = dir + "/0/pattern";
  std::vector<std::pair<uint64_t, uint64_t>> el;
  {
    std::ifstream f(base + "_edge");
    if (!f) throw std::runtime_error("missing " + base + "_edge");
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream iss(line);
      uint64_t s = 0, t = 0;
      iss >> s >> t;
      p.edges.push_back(t);
      el.push_back({s, t});
    }
  }
  p.edge_count = p.edges.size();
  {  // graph.hpp:224-270
    uint64_t maxv = el.back().first, cnt = 0, l = 0, deg = 0, cur = 0;
    std::vector<uint64_t> vd;
    do {
      if (l < el.size() && el[l].first == cur) {
        ++deg;
        ++l;
      } else {
        p.vertices.push_back(p.vertices.empty() ? 0 : vd.back() + p.vertices.back());
        vd.push_back(deg);
        deg = 0;
        ++cnt;
        cur = cnt;
      }
    } while (cur <= maxv);
    p.vertices.push_back(p.vertices.empty() ? 0 : vd.back() + p.vertices.back());
    p.vertex_count = cnt;
  }
  {
    std::ifstream f(base + "_vertex_data");
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream iss(line);
      uint64_t v = 0, d = 0;
      iss >> v >> d;
      p.vdata.push_back(d);
    }
  }
  {
    std::ifstream f(base + "_stat");
    std::string line;
    while (std::getline(f, line)) {
      auto t = split(line, ':');
      if (t.size() < 2) continue;
      std::string k = trim(t[0]);
      for (auto& ch : k) ch = (char)tolower((unsigned char)ch);
      if (k == "diameter") p.diameter = std::stoull(trim(t[1]));
    }
  }
  {
    std::ifstream f(base + "_nlc");
    std::string line;
    while (std::getline(f, line)) {
      auto t = split(line, ':');
      if (t.size() < 6) throw std::runtime_error("bad nlc line");
      Nlc n;
      n.L = split_u64(trim(t[0]), ' ');
      n.I = split_u64(trim(t[1]), ' ');
      n.C = std::stoull(trim(t[2]));
      n.VC = std::stoull(trim(t[3])) != 0;
      n.IL = std::stoull(trim(t[4])) != 0;
      n.SV = std::stoull(trim(t[5])) != 0;
      p.nlc.push_back(n);
    }
  }
  {
    std::ifstream f(base + "_non_local_constraint");
    std::string line;
    size_t i = 0;
    while (std::getline(f, line)) {
      line = trim(line);
      auto t = split(line, ':');
      if (t.size() < 3) throw std::runtime_error("bad non_local_constraint line");
      if (i < p.nlc.size()) p.nlc[i].E = split_u64(trim(t[1]), ' ');
      ++i;
    }
  }
  if (p.vdata.size() > 16 || p.vdata.size() > p.vertex_count) throw std::runtime_error("bad pattern vertex data");
  return p;
}

// ---------------------------------------------------------------------------
struct Stats {
  uint64_t iterations;
  uint64_t terminated;
  uint64_t lcc_edges;     // adjacency entries scanned by LCC senders
  uint64_t nlcc_edges;    // adjacency entries scanned by NLCC (path/cycle) token initiators/relays
  uint64_t tds_edges;     // adjacency entries scanned by TDS initiators/relays
  uint64_t paths;         // complete TDS walks in the final iteration
  uint64_t final_vertices;
  uint64_t final_edges;
  double seconds;
  uint64_t lcc_calls;
  uint64_t supersteps;
};

typedef std::bitset<16> BitSet;

struct VState {
  BitSet tstate;  // vertex_state_generic::template_vertices
  BitSet tn;      // vertex_state_generic::template_neighbors
};

class Engine {
 public:
  Engine(uint64_t n, const uint64_t* off, const uint32_t* col, const uint64_t* labels, const Pattern& p,
         uint32_t nranks, uint64_t hub_threshold, unsigned threads = 1)
      : n_(n), off_(off), col_(col), p_(p), nranks_(nranks ? nranks : 1) {
    T_ = threads ? threads : 1;
    blk_ = std::max<uint64_t>(1, (n + T_ - 1) / T_);
    S_.resize(T_);
    label_.resize(n);
    for (uint64_t v = 0; v < n; ++v) {
      if (labels) {
        label_[v] = labels[v];
      } else {
        // vertex_data_db_degree.hpp:109
        label_[v] = (uint64_t)std::ceil(std::log2((double)(off[v + 1] - off[v]) + 1));
      }
      if (off[v + 1] - off[v] >= hub_threshold) hubs_.push_back(v);
    }
    active_.assign(n, 1);
    tpub_.assign(n, 0);
    M_.resize(n);
    seen_.resize(n);
  }

  uint32_t owner(uint64_t v) const {
    if (!hubs_.empty()) {
      auto it = std::lower_bound(hubs_.begin(), hubs_.end(), v);
      if (it != hubs_.end() && *it == v) return (uint32_t)((it - hubs_.begin()) % nranks_);
    }
    return (uint32_t)(v % nranks_);
  }

  BitSet label_match(uint64_t v) const {
    BitSet b;
    for (size_t t = 0; t < p_.vdata.size(); ++t)
      if (p_.vdata[t] == label_[v]) b.set(t);
    return b;
  }

  // lppm_visitor::verify_and_update_vertex_state valid-parent test (:673-726)
  bool valid_parent(const BitSet& tdst, const BitSet& tsrc) const {
    for (size_t t = 0; t < 16; ++t) {
      if (!tdst.test(t)) continue;
      for (size_t i = 0; i < 16; ++i) {
        if (!tsrc.test(i)) continue;
        for (uint64_t e = p_.vertices[t]; e < p_.vertices[t + 1]; ++e)
          if (p_.edges[e] == i) return true;
      }
    }
    return false;
  }

  // ---- one LCC call (label_propagation_pattern_matching_bsp :1033-1153)
  //
  // Run by T_ worker threads, each the "rank" of a contiguous block of
  // vertex ids (the reference's MPI ranks own id % P; LCC results do not
  // depend on the partition).  A superstep is the BSP of the
  // reference: senders fill per-(sender, receiver) mailboxes, receivers drain
  // the boxes addressed to them, then every rank verifies its own state map.
  // Each vertex's state (active_, tpub_, M_, its S_ entry) is touched only by
  // its owner thread.  T_ = 1 is the original sequential order exactly.
  struct Msg {
    uint64_t dst, src;
    BitSet t;
  };

  void lcc(bool init_step, bool& not_finished, uint64_t itr) {
    stats_.lcc_calls++;
    const unsigned T = T_;
    for (uint64_t ss = 0; ss < p_.diameter; ++ss) {
      stats_.supersteps++;
      const bool first = (ss == 0 && init_step);
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::vector<std::vector<Msg>>> box(T, std::vector<std::vector<Msg>>(T));
      std::vector<uint64_t> trav(T, 0);
      // senders: lppm_visitor::visit (:468-636), one visit per vertex
      parallel([&](unsigned r) {
        auto& out = box[r];
        for (uint64_t v = lo(r); v < lo(r + 1); ++v) {
          if (!active_[v]) continue;
          if (first) {
            BitSet tl = label_match(v);
            if (tl.none()) {
              active_[v] = 0;
              continue;
            }
            tpub_[v] = (uint16_t)tl.to_ulong();
            for (uint64_t e = off_[v]; e < off_[v + 1]; ++e) out[tid_of(col_[e])].push_back({col_[e], v, tl});
            trav[r] += off_[v + 1] - off_[v];
          } else {
            if (S_[r].find(v) == S_[r].end()) continue;
            BitSet tv(tpub_[v]);
            if (tv.none()) continue;
            for (auto& it : M_[v]) out[tid_of(it.first)].push_back({it.first, v, tv});
            trav[r] += M_[v].size();
          }
        }
      });
      uint64_t nmsgs = 0;
      for (unsigned r = 0; r < T; ++r) {
        stats_.lcc_edges += trav[r];
        for (unsigned q = 0; q < T; ++q) nmsgs += box[r][q].size();
      }
      // receivers: lppm_visitor::pre_visit (:149-459)
      parallel([&](unsigned r) {
        auto& Sr = S_[r];
        for (unsigned q = 0; q < T; ++q) {
          for (const auto& m : box[q][r]) {
            const uint64_t u = m.dst;
            if (!active_[u]) continue;
            BitSet tu;
            if (first) {
              tu = label_match(u);
              if (tu.none()) {
                active_[u] = 0;
                continue;
              }
              if (m.t.none()) continue;
              tpub_[u] = (uint16_t)tu.to_ulong();
            } else {
              auto f = Sr.find(u);
              if (f == Sr.end()) continue;
              if (m.t.none()) continue;
              tu = BitSet(tpub_[u]);
              if (tu.none()) continue;
            }
            // member verify_and_update_vertex_state (:647-816)
            if (!valid_parent(tu, m.t)) continue;
            auto f = Sr.find(u);
            if (f == Sr.end()) {
              f = Sr.insert({u, VState()}).first;
              f->second.tstate = tu;
            }
            f->second.tn |= m.t;
            auto fe = M_[u].find(m.src);
            if (fe == M_[u].end()) {
              if (first) M_[u].insert({m.src, 1});
              // else: "did not find the expected item" -- TN already updated (:775 vs :801)
            } else {
              fe->second = 1;
            }
          }
          std::vector<Msg>().swap(box[q][r]);  // drained
        }
      });
      // global verify_and_update_vertex_state (:829-1027)
      std::vector<uint8_t> any_removed(T, 0);
      parallel([&](unsigned r) {
        auto& Sr = S_[r];
        if (first) {
          for (uint64_t v = lo(r); v < lo(r + 1); ++v)
            if (active_[v] && Sr.find(v) == Sr.end()) {
              active_[v] = 0;
              M_[v].clear();
            }
        }
        std::vector<uint64_t> removed;
        for (auto& kv : Sr) {
          const uint64_t v = kv.first;
          VState& st = kv.second;
          for (size_t t = 0; t < 16; ++t) {
            if (!st.tstate.test(t)) continue;
            BitSet pe(p_.adj(t));
            BitSet x = pe & st.tn;
            if (!(pe == x && !x.none())) st.tstate.reset(t);
          }
          if (st.tstate.none()) {
            removed.push_back(v);
            active_[v] = 0;
            M_[v].clear();
          } else {
            tpub_[v] = (uint16_t)st.tstate.to_ulong();
            st.tn.reset();
            for (auto it = M_[v].begin(); it != M_[v].end();) {
              if (!it->second) {
                it = M_[v].erase(it);
              } else {
                it->second = 0;
                ++it;
              }
            }
          }
        }
        if (!removed.empty()) any_removed[r] = 1;
        for (auto v : removed) Sr.erase(v);
      });
      for (unsigned r = 0; r < T; ++r)
        if (any_removed[r]) not_finished = true;
      double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      // outputs (:1103-1145)
      superstep_lines_.push_back(std::to_string(itr) + ", LP, " + std::to_string(ss) + ", " + fmt(secs));
      emit_counts(itr, "LP", ss, nmsgs);
    }
  }

  // worker threads of the LCC: contiguous id blocks
  uint64_t lo(unsigned r) const { return std::min<uint64_t>(n_, uint64_t(r) * blk_); }
  unsigned tid_of(uint64_t v) const { return static_cast<unsigned>(v / blk_); }
  template <typename F>
  void parallel(F&& f) {
    if (T_ == 1) {
      f(0u);
      return;
    }
    std::vector<std::thread> pool;
    for (unsigned r = 0; r < T_; ++r) pool.emplace_back([&f, r] { f(r); });
    for (auto& th : pool) th.join();
  }
  VState* s_find(uint64_t v) {
    auto& Sr = S_[tid_of(v)];
    auto f = Sr.find(v);
    return f == Sr.end() ? nullptr : &f->second;
  }
  template <typename F>
  void s_for_each(F&& f) {
    for (auto& Sr : S_)
      for (auto& kv : Sr) f(kv);
  }
  uint64_t s_size() const {
    uint64_t k = 0;
    for (auto& Sr : S_) k += Sr.size();
    return k;
  }

  void emit_counts(uint64_t itr, const char* tag, uint64_t idx, uint64_t msgs) {
    std::vector<uint64_t> vc(nranks_, 0), ec(nranks_, 0);
    s_for_each([&](const std::pair<const uint64_t, VState>& kv) {
      uint32_t r = owner(kv.first);
      vc[r]++;
      ec[r] += M_[kv.first].size();
    });
    for (uint32_t r = 0; r < nranks_; ++r) {
      std::string pre = std::to_string(itr) + ", " + tag + ", " + std::to_string(idx) + ", ";
      vcount_[r].push_back(pre + std::to_string(vc[r]));
      ecount_[r].push_back(pre + std::to_string(ec[r]));
      // message counts are partition dependent and excluded from parity;
      // rank 0 carries the total.
      mcount_[r].push_back(pre + std::to_string(r == 0 ? msgs : 0));
    }
  }

  // ---- NLCC path / cycle (nem_1)
  struct Tok {
    uint64_t vertex, parent, target;
    uint64_t itr;
    uint64_t ppi;  // parent_pattern_index
    bool ack;
  };

  bool tp_pre_visit(const Nlc& l, const Tok& t, uint64_t& msgcount) {
    msgcount++;
    if (!active_[t.vertex]) return false;
    if (t.ack) return true;
    const uint64_t C = l.C;
    // enable_vertex_token_source: dedup on (vertex, source) for non-terminal arrivals (:131-139)
    if (C > t.itr && seen_[t.vertex].count(t.target)) return false;
    if (C > t.itr && t.vertex == t.target) return false;  // target cannot relay (:174-177)
    const uint64_t k = t.itr + 1;
    if (label_[t.vertex] != l.L[k]) return false;
    BitSet tv(tpub_[t.vertex]);
    if (tv.none() || !tv.test(l.I[k])) return false;
    if (t.ppi != l.I[k - 1]) return false;
    if (C > t.itr) seen_[t.vertex].insert(t.target);
    return true;
  }

  void tp_visit(const Nlc& l, const Tok& t, std::deque<Tok>& q, std::unordered_map<uint64_t, uint8_t>& tsm,
                uint64_t& msgcount) {
    if (!active_[t.vertex]) return;
    if (t.ack) {
      auto f = tsm.find(t.vertex);
      if (f != tsm.end()) f->second = 1;
      return;
    }
    const uint64_t C = l.C, k = t.itr + 1;
    if (C > t.itr && t.vertex == t.target) return;
    if (label_[t.vertex] != l.L[k]) return;
    BitSet tv(tpub_[t.vertex]);
    if (tv.none() || !tv.test(l.I[k])) return;
    const bool parent_ok = (t.ppi == l.I[k - 1]);
    if (C > t.itr) {
      if (!parent_ok) return;
      stats_.nlcc_edges += M_[t.vertex].size();
      for (auto& it : M_[t.vertex]) {
        if (it.first == t.parent) continue;
        Tok nt{it.first, t.vertex, t.target, k, l.I[k], false};
        if (tp_pre_visit(l, nt, msgcount)) q.push_back(nt);
      }
    } else {  // terminal (:661-791)
      if (!parent_ok) return;
      if (!l.VC) {
        if (t.vertex == t.target) return;
        if (l.SV) {  // pattern_selected_vertices (:697-719): the source must be in Seen[vertex]
          if (!seen_[t.vertex].count(t.target)) return;
          auto f = tsm.find(t.vertex);
          if (f != tsm.end()) f->second = 1;  // else "did not find the expected item"
          return;
        }
        Tok ack{t.target, t.vertex, t.target, t.itr, 0, true};
        if (tp_pre_visit(l, ack, msgcount)) q.push_back(ack);
      } else if (t.vertex == t.target) {
        auto f = tsm.find(t.vertex);
        if (f == tsm.end()) return;  // "did not find the expected item" (:749-754)
        f->second = 1;
        auto fe = M_[t.vertex].find(t.parent);
        if (fe != M_[t.vertex].end()) fe->second = 1;  // mark the cycle-closing edge (:764-770)
      }
    }
  }

  void nlcc_path(const Nlc& l, std::unordered_map<uint64_t, uint8_t>& tsm, uint64_t& msgcount) {
    for (uint64_t v = 0; v < n_; ++v) {  // init visits (:387-528)
      if (!active_[v]) continue;
      if (l.SV) {  // pattern_selected_vertices (:409-436): last-label vertices are the ones verified
        if (label_[v] != l.L[0] && label_[v] != l.L.back()) continue;
        if (label_[v] == l.L.back()) {
          if (!tsm.count(v)) tsm.insert({v, 0});
          continue;
        }
      } else if (label_[v] != l.L[0]) {
        continue;
      }
      BitSet tv(tpub_[v]);
      if (tv.none() || !tv.test(l.I[0])) continue;
      if (!l.VC && !l.SV && !tv.test(l.I.back())) continue;  // pattern_indices[size()-1] (nem_1.hpp:447-454)
      if (!l.SV && !tsm.count(v)) tsm.insert({v, 0});
      std::deque<Tok> q;
      stats_.nlcc_edges += M_[v].size();
      for (auto& it : M_[v]) {
        Tok t{it.first, v, v, 0, l.I[0], false};
        if (tp_pre_visit(l, t, msgcount)) q.push_back(t);
      }
      while (!q.empty()) {  // tppm_queue is FIFO (:14-50)
        Tok t = q.front();
        q.pop_front();
        tp_visit(l, t, q, tsm, msgcount);
      }
    }
  }

  // ---- TDS (tds_batch_1)
  struct Walk {
    uint64_t vertex, parent, target, itr, ppi;
    bool ack;
    uint64_t visited[16];
  };

  bool tds_enum_ok(const Nlc& l, uint64_t pos, uint64_t v, const uint64_t* visited) const {
    // pattern_enumeration check (:284-302, :622-639)
    if (l.E[pos] == pos) {
      for (uint64_t i = 0; i < pos; ++i)
        if (visited[i] == v) return false;
      return true;
    } else if (l.E[pos] < pos) {
      return visited[l.E[pos]] == v;
    }
    return false;
  }

  bool tds_pre_visit(const Nlc& l, const Walk& w, uint64_t& msgcount) {
    msgcount++;
    if (!active_[w.vertex]) return false;
    if (w.ack) return true;
    const uint64_t k = w.itr + 1;
    if (label_[w.vertex] != l.L[k]) return false;
    BitSet tv(tpub_[w.vertex]);
    if (tv.none() || !tv.test(l.I[k])) return false;
    if (w.ppi != l.I[k - 1]) return false;
    if (l.C > w.itr && !tds_enum_ok(l, k, w.vertex, w.visited)) return false;
    return true;
  }

  void tds_visit(const Nlc& l, const Walk& w, std::deque<Walk>& q, std::unordered_map<uint64_t, uint8_t>& tsm,
                 uint64_t& msgcount, std::vector<std::vector<std::string>>& paths) {
    if (!active_[w.vertex]) return;
    if (w.ack) {
      auto f = tsm.find(w.vertex);
      if (f != tsm.end()) f->second = 1;
      return;
    }
    const uint64_t C = l.C, k = w.itr + 1;
    if (label_[w.vertex] != l.L[k]) return;
    BitSet tv(tpub_[w.vertex]);
    if (tv.none() || !tv.test(l.I[k])) return;
    const bool parent_ok = (w.ppi == l.I[k - 1]);
    if (C > w.itr) {
      if (!parent_ok) return;
      if (!tds_enum_ok(l, k, w.vertex, w.visited)) return;
      stats_.tds_edges += M_[w.vertex].size();
      for (auto& it : M_[w.vertex]) {
        const uint64_t nb = it.first;
        if (C == k) {  // penultimate hop (:808-845)
          if (l.VC && nb != w.target) continue;
          if (!l.VC && nb == w.target) continue;
          if (!l.VC && !tds_enum_ok(l, k + 1, nb, w.visited)) continue;
        } else {
          if (!tds_enum_ok(l, k + 1, nb, w.visited)) continue;
        }
        Walk nw;
        nw.vertex = nb;
        nw.parent = w.vertex;
        nw.target = w.target;
        nw.itr = k;
        nw.ppi = l.I[k];
        nw.ack = false;
        std::memcpy(nw.visited, w.visited, sizeof(nw.visited));
        nw.visited[k + 1] = nb;
        if (tds_pre_visit(l, nw, msgcount)) q.push_back(nw);
      }
    } else {  // terminal (:641-758)
      if (!parent_ok) return;
      bool write = false;
      if (!l.VC) {
        if (w.vertex == w.target) return;
        Walk ack = w;
        ack.vertex = w.target;
        ack.ack = true;
        if (tds_pre_visit(l, ack, msgcount)) q.push_back(ack);
        write = true;
      } else if (w.vertex == w.target && w.vertex == w.visited[0]) {
        auto f = tsm.find(w.vertex);
        if (f != tsm.end()) f->second = 1;
        write = true;
      }
      if (write) {
        std::string s = "[" + std::to_string(owner(w.vertex)) + "], ";
        for (uint64_t i = 0; i <= k; ++i) s += std::to_string(w.visited[i]) + ", ";
        s += "[" + std::to_string(w.vertex) + "]";
        paths[owner(w.vertex)].push_back(s);
        stats_.paths++;
      }
    }
  }

  void tds(const Nlc& l, std::unordered_map<uint64_t, uint8_t>& tsm, uint64_t& msgcount,
           std::vector<std::vector<std::string>>& paths) {
    if (l.E.size() < l.C + 2) throw std::runtime_error("enumeration line shorter than walk");
    stats_.paths = 0;
    std::unordered_set<uint64_t> sources;  // :1064-1135
    for (uint64_t v = 0; v < n_; ++v) {
      if (!active_[v] || label_[v] != l.L[0]) continue;
      BitSet tv(tpub_[v]);
      if (tv.none() || !tv.test(l.I[0])) continue;
      sources.insert(v);
    }
    for (auto v : sources) tsm.insert({v, 0});
    for (uint64_t v = 0; v < n_; ++v) {  // init visits (:425-512)
      if (!active_[v] || !tsm.count(v)) continue;
      if (label_[v] != l.L[0]) continue;
      BitSet tv(tpub_[v]);
      if (tv.none() || !tv.test(l.I[0])) continue;
      std::deque<Walk> q;
      Walk base{};
      base.visited[0] = v;
      stats_.tds_edges += M_[v].size();
      for (auto& it : M_[v]) {
        Walk w = base;
        w.vertex = it.first;
        w.parent = v;
        w.target = v;
        w.itr = 0;
        w.ppi = l.I[0];
        w.ack = false;
        w.visited[1] = it.first;
        if (tds_pre_visit(l, w, msgcount)) q.push_back(w);
      }
      while (!q.empty()) {
        Walk w = q.front();
        q.pop_front();
        tds_visit(l, w, q, tsm, msgcount, paths);
      }
    }
  }

  // ---- driver (run_pattern_matching_beta.cpp:544-1351)
  void run(const std::string& out, uint64_t max_iterations) {
    auto t_start = std::chrono::steady_clock::now();
    vcount_.assign(nranks_, {});
    ecount_.assign(nranks_, {});
    mcount_.assign(nranks_, {});
    std::vector<std::vector<std::vector<std::string>>> subgraphs(p_.nlc.size(),
                                                                 std::vector<std::vector<std::string>>(nranks_));
    bool init_step = true, nf = false;
    uint64_t itr = 0;
    bool terminated = true;
    do {
      if (max_iterations && itr >= max_iterations) {  // 0 = unlimited (the reference has no cap)
        terminated = false;
        break;
      }
      nf = false;
      auto it0 = std::chrono::steady_clock::now();
      auto lp0 = std::chrono::steady_clock::now();
      lcc(init_step, nf, itr);
      step_lines_.push_back(std::to_string(itr) + ", LP, " + fmt(since(lp0)));
      init_step = false;
      if (itr == 0) nf = true;
      if (nf) {
        nf = false;
        for (size_t pl = 0; pl < p_.nlc.size(); ++pl) {
          const Nlc& l = p_.nlc[pl];
          if (l.SV && (pl >= 4 || l.VC))
            throw std::runtime_error("pattern_selected_vertices=1 is supported on path lines (index < 4, valid_cycle 0)");
          for (auto& r : subgraphs[pl]) r.clear();  // file reopened with truncation (:713-717)
          std::unordered_map<uint64_t, uint8_t> tsm;
          if (!l.SV) {
            for (auto& s : seen_) s.clear();  // beta.cpp:791-793
          } else {  // keep the sets of active vertices with the line's last label (beta.cpp:823-850)
            for (uint64_t v = 0; v < n_; ++v)
              if (!(active_[v] && label_[v] == l.L.back())) seen_[v].clear();
          }
          uint64_t msgcount = 0;
          auto tp0 = std::chrono::steady_clock::now();
          if (pl >= 4) {  // :762-767
            tds(l, tsm, msgcount, subgraphs[pl]);
          } else {
            nlcc_path(l, tsm, msgcount);
          }
          // post-processing (:956-1071)
          bool deleted = false;
          const uint64_t ibit = l.SV ? l.I.back() : l.I[0];  // token_source_pattern_ndices_tp_index (:959-962)
          for (auto& s : tsm) {
            if (s.second) continue;
            BitSet tv(tpub_[s.first]);
            if (tv.none()) continue;
            if (tv.test(ibit)) {
              tv.reset(ibit);
              tpub_[s.first] = (uint16_t)tv.to_ulong();
            }
            if (tv.none()) active_[s.first] = 0;
            nf = true;
            deleted = true;
          }
          for (auto& s : tsm)
            if (!active_[s.first]) S_[tid_of(s.first)].erase(s.first);
          superstep_lines_.push_back(std::to_string(itr) + ", TP, " + std::to_string(pl) + ", " + fmt(since(tp0)));
          emit_counts(itr, "TP", pl, msgcount);
          if (deleted && l.IL) {
            auto lpi = std::chrono::steady_clock::now();
            lcc(false, nf, itr);
            step_lines_.push_back(std::to_string(itr) + ", LP, " + fmt(since(lpi)));
          }
        }
      } else {
        nf = false;
      }
      iteration_lines_.push_back(std::to_string(itr) + ", " + fmt(since(it0)));
      ++itr;
    } while (nf);
    const double secs = since(t_start);
    stats_.iterations = itr;
    stats_.terminated = terminated ? 1 : 0;
    stats_.seconds = secs;
    stats_.final_vertices = s_size();
    uint64_t fe = 0;
    s_for_each([&](const std::pair<const uint64_t, VState>& kv) { fe += M_[kv.first].size(); });
    stats_.final_edges = fe;
    if (!out.empty()) write_results(out, itr, secs, subgraphs);
  }

  void write_results(const std::string& out, uint64_t itr, double secs,
                     const std::vector<std::vector<std::vector<std::string>>>& subgraphs) {
    const std::string d = out + "/0";
    auto wr = [](const std::string& path, const std::vector<std::string>& lines) {
      std::ofstream f(path);
      if (!f) throw std::runtime_error("cannot write " + path);
      for (auto& l : lines) f << l << "\n";
    };
    wr(out + "/result_pattern_set",
       {"0, " + std::to_string(nranks_) + ", " + std::to_string(itr) + ", " + fmt(secs) + ", " +
        std::to_string(p_.edge_count) + ", " + std::to_string(p_.vertex_count) + ", " +
        std::to_string(p_.nlc.size())});
    wr(d + "/result_iteration", iteration_lines_);
    wr(d + "/result_step", step_lines_);
    wr(d + "/result_superstep", superstep_lines_);
    std::vector<std::vector<std::string>> av(nranks_), ae(nranks_);
    std::vector<uint64_t> members;
    s_for_each([&](const std::pair<const uint64_t, VState>& kv) { members.push_back(kv.first); });
    for (const uint64_t v : members) {
      const uint32_t r = owner(v);
      av[r].push_back(std::to_string(r) + ", " + std::to_string(v) + ", 0, " + std::to_string(label_[v]) + ", " +
                      BitSet(tpub_[v]).to_string());
      for (auto& nb : M_[v]) ae[r].push_back(std::to_string(r) + ", " + std::to_string(v) + ", " + std::to_string(nb.first));
    }
    for (uint32_t r = 0; r < nranks_; ++r) {
      const std::string rs = std::to_string(r);
      wr(d + "/all_ranks_active_vertices_count/active_vertices_" + rs, vcount_[r]);
      wr(d + "/all_ranks_active_edges_count/active_edges_" + rs, ecount_[r]);
      wr(d + "/all_ranks_messages/messages_" + rs, mcount_[r]);
      wr(d + "/all_ranks_active_vertices/active_vertices_" + rs, av[r]);
      wr(d + "/all_ranks_active_edges/active_edges_" + rs, ae[r]);
      for (size_t pl = 0; pl < subgraphs.size(); ++pl)
        wr(d + "/all_ranks_subgraphs/subgraphs_" + std::to_string(pl) + "_" + rs, subgraphs[pl][r]);
    }
  }

  static std::string fmt(double x) {
    std::ostringstream o;
    o << x;
    return o.str();
  }
  static double since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
  }

  Stats stats_{};

 private:
  uint64_t n_;
  const uint64_t* off_;
  const uint32_t* col_;
  const Pattern& p_;
  uint32_t nranks_;
  std::vector<uint64_t> hubs_;
  std::vector<uint64_t> label_;
  std::vector<uint8_t> active_;
  std::vector<uint16_t> tpub_;
  unsigned T_ = 1;  // LCC worker threads
  uint64_t blk_ = 1;
  std::vector<std::unordered_map<uint64_t, VState>> S_;  // state map, one per worker (owner of the ids)
  std::vector<std::unordered_map<uint64_t, uint8_t>> M_;
  std::vector<std::unordered_set<uint64_t>> seen_;
  std::vector<std::vector<std::string>> vcount_, ecount_, mcount_;
  std::vector<std::string> superstep_lines_, step_lines_, iteration_lines_;
};

}  // namespace oracle

extern "C" {

typedef oracle::Stats oracle_stats_t;

// Runs the whole driver loop on a CSR (rows may be in any order within a row).
// labels == NULL selects degree labels.  result_dir == NULL or "" skips files.
// Returns 0 on success, -1 on error (message on stderr).
// threads: LCC worker threads (rank-partitioned BSP, identical results for any count).
int oracle_run_csr_mt(uint64_t n, const uint64_t* off, const uint32_t* col, const uint64_t* labels,
                      const char* pattern_dir, const char* result_dir, uint32_t nranks, uint64_t hub_threshold,
                      uint64_t max_iterations, uint32_t threads, oracle_stats_t* stats) {
  try {
    oracle::Pattern p = oracle::load_pattern(pattern_dir);
    oracle::Engine eng(n, off, col, labels, p, nranks, hub_threshold, threads);
    eng.run(result_dir ? result_dir : "", max_iterations);
    if (stats) *stats = eng.stats_;
    return 0;
  } catch (const std::exception& e) {
    std::cerr << "oracle error: " << e.what() << std::endl;
    return -1;
  }
}

int oracle_run_csr(uint64_t n, const uint64_t* off, const uint32_t* col, const uint64_t* labels,
                   const char* pattern_dir, const char* result_dir, uint32_t nranks, uint64_t hub_threshold,
                   uint64_t max_iterations, oracle_stats_t* stats) {
  return oracle_run_csr_mt(n, off, col, labels, pattern_dir, result_dir, nranks, hub_threshold, max_iterations, 1,
                           stats);
}

uint64_t oracle_hash_nbits(uint64_t x, int n) { return oracle::hash_nbits(x, n); }

// One generator rank's undirected edges (before symmetrization).
void oracle_rmat_rank(uint64_t scale, uint64_t p_gen, uint64_t rank, uint64_t count, uint64_t* us, uint64_t* vs) {
  (void)p_gen;
  oracle::rmat_edges(scale, 5489 + 3 * rank, count, us, vs);
}

uint32_t oracle_mt19937_nth(uint32_t seed, uint64_t n) {
  oracle::Mt19937 m(seed);
  uint32_t x = 0;
  for (uint64_t i = 0; i < n; ++i) x = m.next();
  return x;
}

}  // extern "C"
