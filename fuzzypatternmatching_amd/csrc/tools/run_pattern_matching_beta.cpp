// run_pattern_matching_beta -- drop-in CLI for the MI355X pattern-matching path.
//
// Same options and result directory as src/run_pattern_matching_beta.cpp
// (getopt "i:b:v:e:p:o:x:h ", :82-142), driving gfx950 GPUs through the C-ABI of
// include/pm_abi.h.  Per-rank result files are written for the P the graph
// files were created with (<base>_<r>_of_<P>).
//
// How the search is placed (the reference runs one MPI rank per core or GPU,
// `srun --ntasks-per-node=4 ./src/run_pattern_matching_beta ...`, README.md:30,
// each rank opening <base>_<rank>_of_<P>, beta.cpp:209-223 /
// distributed_db.hpp:353-357):
//   * launched as several processes (srun, mpirun, torchrun, or PM_RANK /
//     PM_WORLD_SIZE by hand): one shard per process, read from the graph files
//     by that process alone (pm_read_graph_shard); the processes meet at
//     PM_MASTER_ADDR:PM_MASTER_PORT (default MASTER_ADDR, MASTER_PORT + 1) and
//     exchange over RCCL when each has a GPU of its own (device = local rank),
//     else through the group's host collectives (pm_host_comm over TCP);
//   * one process, a P-partition graph (P > 1) and at least P GPUs: P shards,
//     one thread and one GPU each, one RCCL communicator (xGMI);
//   * one process, P > 1 and fewer GPUs than P: the P shards in-process on
//     device 0 (pm_run_beta_local_shards2);
//   * P = 1, or a directed graph (the sharded search takes symmetric graphs): one context holds the whole graph
//     (launched: on rank 0).
// PM_SHARDS=<k> overrides the shard count of a one-process run (any k: the
// shards are read from the files whatever their P); PM_TRANSPORT=rccl|host
// forces a launched run's transport.  Results are identical in every mode.
//
// Kept quirks: -i falls through into -b (beta.cpp:105-110), so `-i X` alone
// also sets the backup base to X -- the transfer is then skipped instead of
// truncating X onto itself; -e and -x are accepted and ignored.
// Extensions (not in the reference): environment PM_MAX_ITERATIONS caps the
// do/while loop (the reference can loop forever, SURVEY.md A.6 hazard 11) and
// PM_DEVICE selects the GPU of a one-context run.
#include <getopt.h>
#include <unistd.h>

#include <bitset>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/pm_abi.h"
#include "../host/graph_store.hpp"
#include "../host/tcp_group.hpp"

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

namespace {

struct Options {
  std::string graph_input, backup_input, vertex_metadata, pattern_dir, result_dir;
  uint64_t max_iterations = 0;
};

const char* transport_name(int t) {
  switch (t) {
    case PM_TRANSPORT_RCCL: return "RCCL";
    case PM_TRANSPORT_HOST: return "host collectives";
    case PM_TRANSPORT_THREADS: return "in-process exchange";
    default: return "none";
  }
}

void report(const pm_run_stats& st, uint32_t nshards, const std::string& placement) {
  std::cout << "Fuzzy Pattern Matching Time | Pattern [0] : " << st.seconds << std::endl;
  std::cout << "Fuzzy Pattern Matching | Pattern [0] | # Iterations : " << st.iterations
            << (st.terminated ? "" : " (stopped by PM_MAX_ITERATIONS)") << std::endl;
  std::cout << "Active vertices " << st.final_vertices << ", active edges " << st.final_edges << ", walks "
            << st.walks << ", edges traversed " << (st.lcc_edges + st.nlcc_edges + st.tds_edges) << std::endl;
  if (nshards > 1)
    std::cout << "Shards " << nshards << " (" << placement << "), collectives " << st.comm_calls << ", replica rows "
              << st.replica_rows << std::endl;
}

// A shard of the graph files on the host (pm_read_graph_shard), freed with the object.
struct HostShard {
  uint64_t* off = nullptr;
  uint32_t* col = nullptr;
  uint32_t* deg = nullptr;
  uint64_t n = 0, hub = 0;
  int symmetric = 1;
  uint32_t nranks = 1;
  std::string err;
  ~HostShard() {
    pm_free_host(off);
    pm_free_host(col);
    pm_free_host(deg);
  }
  bool read(const std::string& base, uint32_t nshards, uint32_t shard) {
    if (pm_read_graph_shard(base.c_str(), nshards, shard, &off, &col, &deg, &n, &symmetric, &nranks, &hub) != 0) {
      err = pm_last_error(nullptr);
      return false;
    }
    return true;
  }
  pm_shard_desc desc(uint32_t nshards, uint32_t shard) const {
    return pm_shard_desc{n, off, col, deg, symmetric, nranks, hub, nshards, shard};
  }
};

// Success agreement of the threads of one process between the phases of a sharded run (a shard that failed
// must not leave the others in a collective it never makes).
class ThreadAgree {
 public:
  explicit ThreadAgree(int n) : n_(n) {}
  bool operator()(bool ok) {
    std::unique_lock<std::mutex> lk(m_);
    const uint64_t g = gen_;
    all_ok_ = all_ok_ && ok;
    if (++arrived_ == n_) {
      result_ = all_ok_;
      all_ok_ = true;
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
      return result_;
    }
    cv_.wait(lk, [&] { return gen_ != g; });
    return result_;
  }

 private:
  int n_, arrived_ = 0;
  uint64_t gen_ = 0;
  bool all_ok_ = true, result_ = true;
  std::mutex m_;
  std::condition_variable cv_;
};

// One context over the whole graph (P = 1).
int run_one_context(const Options& o) {
  uint64_t *off = nullptr, n = 0, hub = 0;
  uint32_t *col = nullptr, nranks = 1;
  int symmetric = 1;
  std::cout << "Loading Graph ... " << std::endl;
  if (pm_read_graph(o.graph_input.c_str(), &off, &col, &n, &symmetric, &nranks, &hub) != 0) {
    std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  std::cout << "Done Loading Graph. " << n << " vertices, " << off[n] << " directed edges, " << nranks
            << " partition(s)." << std::endl;
  pm_graph_desc d{n, off, col, symmetric, nranks, hub};
  const char* dev = std::getenv("PM_DEVICE");
  pm_ctx* ctx = pm_create(&d, o.pattern_dir.c_str(), dev ? std::atoi(dev) : 0);
  int rc = 0;
  try {
    if (!ctx) throw std::runtime_error(pm_last_error(nullptr));
    if (!o.vertex_metadata.empty()) {
      // parsed on the GPU (pm_ingest.hip); PM_HOST_LABELS=1 takes the host loader instead
      if (std::getenv("PM_HOST_LABELS")) {
        std::vector<uint64_t> labels = pm::load_vertex_labels(o.vertex_metadata, n);
        if (pm_vertex_data_set(ctx, labels.data()) != 0) throw std::runtime_error(pm_last_error(ctx));
      } else if (pm_vertex_data_files(ctx, o.vertex_metadata.c_str()) != 0) {
        throw std::runtime_error(pm_last_error(ctx));
      }
    }
    pm_run_stats st{};
    if (pm_run_beta(ctx, o.result_dir.c_str(), o.max_iterations, &st) != 0) throw std::runtime_error(pm_last_error(ctx));
    report(st, 1, "");
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    rc = 1;
  }
  if (ctx) pm_destroy(ctx);
  pm_free_host(off);
  pm_free_host(col);
  return rc;
}

// One process, nshards shards on fewer GPUs than shards: the shards in-process on device 0.
int run_local_shards(const Options& o, uint32_t nshards) {
  uint64_t *off = nullptr, n = 0, hub = 0;
  uint32_t *col = nullptr, nranks = 1;
  int symmetric = 1;
  std::cout << "Loading Graph ... " << std::endl;
  if (pm_read_graph(o.graph_input.c_str(), &off, &col, &n, &symmetric, &nranks, &hub) != 0) {
    std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  std::cout << "Done Loading Graph. " << n << " vertices, " << off[n] << " directed edges, " << nranks
            << " partition(s)." << std::endl;
  pm_graph_desc d{n, off, col, symmetric, nranks, hub};
  std::vector<pm_run_stats> st(nshards);
  const char* dev = std::getenv("PM_DEVICE");
  const int rc = pm_run_beta_local_shards2(&d, o.pattern_dir.c_str(), dev ? std::atoi(dev) : 0, nshards, nullptr,
                                           o.vertex_metadata.empty() ? nullptr : o.vertex_metadata.c_str(),
                                           o.result_dir.c_str(), o.max_iterations, 1, st.data());
  pm_free_host(off);
  pm_free_host(col);
  if (rc != 0) {
    std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  report(st[0], nshards, "in-process on one GPU");
  return 0;
}

// One shard's run after its context exists: labels, the search; every phase agreed over the shards.
template <typename Agree>
bool shard_search(pm_ctx* ctx, const Options& o, Agree& agree, pm_run_stats& st, std::string& err) {
  bool ok = true;
  if (!o.vertex_metadata.empty() && pm_vertex_data_files(ctx, o.vertex_metadata.c_str()) != 0) {
    err = pm_last_error(ctx);
    ok = false;
  }
  if (!agree(ok)) {
    if (ok) err = "another shard failed";
    return false;
  }
  if (pm_run_beta(ctx, o.result_dir.c_str(), o.max_iterations, &st) != 0) {
    err = pm_last_error(ctx);
    return false;
  }
  return true;
}

// One process, nshards <= GPUs: one thread and one GPU per shard, RCCL between them.
int run_gpu_threads(const Options& o, uint32_t nshards) {
  std::vector<HostShard> shards(nshards);
  std::vector<pm_run_stats> st(nshards);
  std::vector<std::string> errs(nshards);
  std::vector<uint8_t> uid(256);
  const int k = pm_comm_unique_id(uid.data(), uid.size());
  if (k < 0) {
    std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  uid.resize(k);
  std::cout << "Loading Graph ... (" << nshards << " shards, one GPU each)" << std::endl;
  ThreadAgree agree(static_cast<int>(nshards));
  auto work = [&](uint32_t q) {
    const bool read = shards[q].read(o.graph_input, nshards, q);
    if (!read) errs[q] = shards[q].err;
    if (!agree(read)) {
      if (read) errs[q] = "another shard failed";
      return;
    }
    const pm_shard_desc d = shards[q].desc(nshards, q);
    pm_ctx* ctx = pm_create_shard(&d, o.pattern_dir.c_str(), static_cast<int>(q), uid.data());
    if (!ctx) {
      errs[q] = pm_last_error(nullptr);
      return;  // (construction is collective and fails on every shard alike)
    }
    // the host copy of the rows is no longer needed (the context holds its own)
    pm_free_host(shards[q].off);
    pm_free_host(shards[q].col);
    shards[q].off = nullptr;
    shards[q].col = nullptr;
    shard_search(ctx, o, agree, st[q], errs[q]);
    pm_destroy(ctx);
  };
  std::vector<std::thread> pool;
  for (uint32_t q = 0; q < nshards; ++q) pool.emplace_back(work, q);
  for (auto& t : pool) t.join();
  for (uint32_t q = 0; q < nshards; ++q)
    if (!errs[q].empty() && errs[q] != "another shard failed") {
      std::cerr << "Error: shard " << q << ": " << errs[q] << std::endl;
      return 1;
    }
  for (uint32_t q = 0; q < nshards; ++q)
    if (!errs[q].empty()) {
      std::cerr << "Error: shard " << q << ": " << errs[q] << std::endl;
      return 1;
    }
  std::cout << "Done. " << shards[0].n << " vertices, " << shards[0].nranks << " partition(s)." << std::endl;
  report(st[0], nshards, std::to_string(nshards) + " GPUs, RCCL");
  return 0;
}

// Launched as one process per rank.
int run_launched(const Options& o, const pm::LaunchEnv& env) {
  const char* a = pm::env_of("PM_MASTER_ADDR");
  if (!a) a = pm::env_of("MASTER_ADDR");
  const std::string addr = a ? a : "127.0.0.1";
  int port = 29577;
  if (const char* p = pm::env_of("PM_MASTER_PORT")) port = std::atoi(p);
  else if (const char* p2 = pm::env_of("MASTER_PORT")) port = std::atoi(p2) + 1;  // (the launcher's store has it)
  const char* to = pm::env_of("PM_BOOTSTRAP_TIMEOUT");
  pm::TcpGroup grp(env.rank, env.size, addr, port, to ? std::atof(to) : 300.0);
  const uint32_t G = static_cast<uint32_t>(env.size), me = static_cast<uint32_t>(env.rank);
  // -b: rank 0 copies every file (the reference's ranks copy their own, distributed_db.hpp:106-182) and the
  // others wait for it
  std::string copy_err;
  if (me == 0 && !o.backup_input.empty()) {
    try {
      pm::transfer_graph_files(o.backup_input, o.graph_input);
    } catch (const std::exception& e) {
      copy_err = e.what();
    }
  }
  if (!grp.agree(copy_err.empty())) {
    std::cerr << "Error: rank " << me << ": " << (copy_err.empty() ? "rank 0 failed to copy the backup graph" : copy_err)
              << std::endl;
    return 1;
  }
  // the transport: RCCL iff every rank has a GPU of its own (host name, device) -- decided from every rank's view
  const int ndev = pm_device_count();
  const int device = ndev > 0 ? env.local_rank % ndev : 0;
  struct Seat {
    char host[64];
    int32_t device, ndev;
  } seat{};
  gethostname(seat.host, sizeof(seat.host) - 1);
  seat.device = device;
  seat.ndev = ndev;
  std::vector<Seat> seats(G);
  grp.allgather(&seat, seats.data(), sizeof(Seat));
  bool own_gpu = true;
  for (uint32_t g = 0; g < G && own_gpu; ++g)
    for (uint32_t h = g + 1; h < G; ++h)
      if (std::strncmp(seats[g].host, seats[h].host, 64) == 0 && seats[g].device == seats[h].device) own_gpu = false;
  bool rccl = own_gpu;
  if (const char* t = pm::env_of("PM_TRANSPORT")) rccl = std::string(t) == "rccl";
  // rank 0 creates the RCCL id (its only use of the device before the context)
  std::vector<uint8_t> uid(256, 0);
  uint32_t uid_len = 0;
  if (me == 0 && rccl) {
    const int k = pm_comm_unique_id(uid.data(), uid.size());
    uid_len = k > 0 ? static_cast<uint32_t>(k) : 0;
  }
  grp.bcast(&uid_len, sizeof(uid_len));
  if (rccl && uid_len == 0) {
    if (me == 0) std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  grp.bcast(uid.data(), uid.size());
  // a directed graph (ingest_edge_list -u 0): the sharded search takes symmetric graphs, so rank 0 runs the
  // search on one context and the other ranks only wait for it
  bool directed = false;
  try {
    directed = !pm::graph_file_header(o.graph_input).symmetric;
  } catch (const std::exception&) {
    // (a missing file is reported by the shard read below, on every rank)
  }
  if (directed) {
    int rc = 0;
    if (me == 0) {
      std::cout << "Directed input graph: one context on rank 0 (the sharded search takes symmetric graphs)"
                << std::endl;
      rc = run_one_context(o);
    }
    return grp.agree(rc == 0) ? 0 : 1;
  }
  if (me == 0)
    std::cout << "Loading Graph ... (" << G << " ranks launched by " << env.launcher << ", "
              << (rccl ? "RCCL" : "host collectives over TCP") << ")" << std::endl;
  HostShard shard;
  const bool read = shard.read(o.graph_input, G, me);
  if (!grp.agree(read)) {
    std::cerr << "Error: rank " << me << ": " << (read ? "another rank failed to read its shard" : shard.err)
              << std::endl;
    return 1;
  }
  const pm_shard_desc d = shard.desc(G, me);
  pm_host_comm hc = grp.host_comm();
  pm_ctx* ctx = rccl ? pm_create_shard(&d, o.pattern_dir.c_str(), device, uid.data())
                     : pm_create_shard_host_comm(&d, o.pattern_dir.c_str(), device, &hc);
  if (!ctx) {
    std::cerr << "Error: rank " << me << ": " << pm_last_error(nullptr) << std::endl;
    return 1;
  }
  pm_free_host(shard.off);
  pm_free_host(shard.col);
  shard.off = nullptr;
  shard.col = nullptr;
  auto agree = [&](bool ok) { return grp.agree(ok); };
  pm_run_stats st{};
  std::string err;
  const bool ok = shard_search(ctx, o, agree, st, err);
  int32_t ranks = 0, transport = 0;
  pm_comm_info(ctx, nullptr, nullptr, &ranks, &transport);
  pm_destroy(ctx);
  if (!ok) {
    std::cerr << "Error: rank " << me << ": " << err << std::endl;
    return 1;
  }
  if (me == 0) {
    std::cout << "Done. " << shard.n << " vertices, " << shard.nranks << " partition(s)." << std::endl;
    report(st, G, std::to_string(G) + " processes, " + transport_name(transport) + " of " + std::to_string(ranks) +
                      " ranks");
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
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
        o.graph_input = optarg;
        required.set(0);
        // fall through (beta.cpp:105-110)
      case 'b':
        o.backup_input = optarg;
        break;
      case 'v':
        o.vertex_metadata = optarg;
        break;
      case 'e':
        break;
      case 'p':
        o.pattern_dir = optarg;
        required.set(1);
        break;
      case 'o':
        o.result_dir = optarg;
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
    if (const char* mi = std::getenv("PM_MAX_ITERATIONS")) o.max_iterations = std::strtoull(mi, nullptr, 10);
    const pm::LaunchEnv env = pm::launch_env();
    if (env.launched) return run_launched(o, env);
    if (!o.backup_input.empty()) pm::transfer_graph_files(o.backup_input, o.graph_input);
    const int P = pm_graph_partitions(o.graph_input.c_str());
    if (P < 0) {
      std::cerr << "Error: " << pm_last_error(nullptr) << std::endl;
      return 1;
    }
    // a directed graph (ingest_edge_list -u 0) runs on one context: the sharded search takes symmetric graphs
    if (!pm::graph_file_header(o.graph_input).symmetric) return run_one_context(o);
    uint32_t nshards = static_cast<uint32_t>(P);
    if (const char* s = std::getenv("PM_SHARDS")) nshards = static_cast<uint32_t>(std::strtoul(s, nullptr, 10));
    if (nshards == 0 || nshards > 64) {
      std::cerr << "Error: PM_SHARDS must be 1..64" << std::endl;
      return 1;
    }
    if (nshards == 1 && !std::getenv("PM_SHARDS")) return run_one_context(o);
    const int ndev = pm_device_count();
    if (ndev >= static_cast<int>(nshards)) return run_gpu_threads(o, nshards);
    return run_local_shards(o, nshards);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
}
