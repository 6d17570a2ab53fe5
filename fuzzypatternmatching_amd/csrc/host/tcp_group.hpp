// Process group of a launched run_pattern_matching_beta: one process per rank, started by a launcher
// (srun / mpirun / torchrun / by hand), meeting over TCP.
//
// The reference is an MPI program (havoqgt_init, environment.hpp:136-228; launched as `srun
// --ntasks-per-node=4 ./src/run_pattern_matching_beta ...`, README.md:30) whose every exchange goes through
// the MPI mailbox (new_mailbox.hpp:289-713) and MPI_Allreduce (impl/vertex_data.hpp:114-126).  This image
// has no MPI, and the search's exchanges belong on RCCL anyway; the group below only
//   * reads rank / size / local rank from whichever launcher started the process (launch_env),
//   * meets at rank 0 (TCP, PM_MASTER_ADDR:PM_MASTER_PORT) and there decides the transport: RCCL when every
//     rank has a GPU of its own (the xGMI path), otherwise the group's own host collectives,
//   * hands out the RCCL communicator id, and agrees on success between the run's phases (a rank that fails
//     to read its shard must not leave the others inside a collective),
//   * carries the search's collectives itself (pm_host_comm) when ranks share a device: a star through rank 0,
//     the transport of last resort (every call is staged through host memory; the reference's mailbox is
//     host-staged too).
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/pm_abi.h"

namespace pm {

struct LaunchEnv {
  bool launched = false;  // some launcher set a world size above 1
  int rank = 0, size = 1, local_rank = 0, local_size = 1;
  std::string launcher;   // which variables were read
};

inline const char* env_of(const char* k) {
  const char* v = std::getenv(k);
  return v && *v ? v : nullptr;
}

// Rank / size / local rank of this process: PM_* first, then Open MPI, MPICH / Intel MPI (PMI), Slurm and
// torch.distributed.run.  A local rank that the launcher does not give defaults to rank % local size (or rank).
inline LaunchEnv launch_env() {
  struct Scheme {
    const char *name, *rank, *size, *lrank, *lsize;
  };
  static const Scheme schemes[] = {
      {"PM", "PM_RANK", "PM_WORLD_SIZE", "PM_LOCAL_RANK", "PM_LOCAL_SIZE"},
      {"Open MPI", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK",
       "OMPI_COMM_WORLD_LOCAL_SIZE"},
      {"PMI", "PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "MPI_LOCALNRANKS"},
      {"Slurm", "SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID", "SLURM_NTASKS_PER_NODE"},
      {"torch.distributed.run", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"},
  };
  LaunchEnv e;
  for (const Scheme& s : schemes) {
    const char* r = env_of(s.rank);
    const char* n = env_of(s.size);
    if (!r || !n) continue;
    e.size = std::atoi(n);
    if (e.size <= 1) continue;
    e.rank = std::atoi(r);
    if (e.rank < 0 || e.rank >= e.size)
      throw std::runtime_error(std::string(s.name) + " rank " + r + " outside world size " + n);
    e.launched = true;
    e.launcher = s.name;
    const char* ls = env_of(s.lsize);
    e.local_size = ls ? std::max(1, std::atoi(ls)) : e.size;  // (Slurm's "4(x2)" form reads as 4)
    const char* lr = env_of(s.lrank);
    e.local_rank = lr ? std::atoi(lr) : e.rank % e.local_size;
    return e;
  }
  return e;
}

class TcpGroup {
 public:
  static constexpr uint32_t kMagic = 0x504D5447u;  // "PMTG"

  // Collective over the `size` processes: rank 0 listens, the others connect (retrying until the timeout).
  TcpGroup(int rank, int size, const std::string& addr, int port, double timeout_s) : rank_(rank), size_(size) {
    if (size < 1 || rank < 0 || rank >= size) throw std::runtime_error("TcpGroup: bad rank / size");
    if (size == 1) return;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    if (rank == 0) {
      const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
      if (ls < 0) throw std::runtime_error("TcpGroup: socket: " + std::string(std::strerror(errno)));
      int one = 1;
      ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_addr.s_addr = htonl(INADDR_ANY);
      a.sin_port = htons(static_cast<uint16_t>(port));
      if (::bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(ls, size) != 0) {
        const std::string err = std::strerror(errno);
        ::close(ls);
        throw std::runtime_error("TcpGroup: rank 0 cannot listen on port " + std::to_string(port) + ": " + err);
      }
      peers_.assign(size, -1);
      for (int k = 1; k < size; ++k) {
        pollfd p{ls, POLLIN, 0};
        const int ms = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(
                                            deadline - std::chrono::steady_clock::now()).count());
        if (ms <= 0 || ::poll(&p, 1, ms) <= 0) {
          ::close(ls);
          throw std::runtime_error("TcpGroup: rank 0 timed out waiting for " + std::to_string(size - k) +
                                   " rank(s) to connect");
        }
        const int s = ::accept(ls, nullptr, nullptr);
        if (s < 0) continue;
        nodelay(s);
        uint32_t hello[3];
        recv_all(s, hello, sizeof(hello));
        if (hello[0] != kMagic || hello[2] != static_cast<uint32_t>(size) || hello[1] == 0 ||
            hello[1] >= static_cast<uint32_t>(size) || peers_[hello[1]] != -1) {
          ::close(s);
          ::close(ls);
          throw std::runtime_error("TcpGroup: a process of another launch (or a repeated rank) connected");
        }
        peers_[hello[1]] = s;
      }
      ::close(ls);
    } else {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (::getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
        throw std::runtime_error("TcpGroup: cannot resolve " + addr);
      int s = -1;
      for (;;) {
        s = ::socket(AF_INET, SOCK_STREAM, 0);
        if (s >= 0 && ::connect(s, res->ai_addr, res->ai_addrlen) == 0) break;
        if (s >= 0) ::close(s);
        s = -1;
        if (std::chrono::steady_clock::now() > deadline) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      }
      ::freeaddrinfo(res);
      if (s < 0) throw std::runtime_error("TcpGroup: rank " + std::to_string(rank) + " cannot reach " + addr + ":" +
                                          std::to_string(port));
      nodelay(s);
      const uint32_t hello[3] = {kMagic, static_cast<uint32_t>(rank), static_cast<uint32_t>(size)};
      send_all(s, hello, sizeof(hello));
      peers_.assign(1, s);
    }
  }
  ~TcpGroup() {
    for (int s : peers_)
      if (s >= 0) ::close(s);
  }
  TcpGroup(const TcpGroup&) = delete;
  TcpGroup& operator=(const TcpGroup&) = delete;

  int rank() const { return rank_; }
  int size() const { return size_; }

  // recv: size blocks of `bytes`, block g from rank g
  void allgather(const void* send, void* recv, uint64_t bytes) {
    char* r = static_cast<char*>(recv);
    std::memmove(r + uint64_t(rank_) * bytes, send, bytes);
    if (size_ == 1) return;
    if (rank_ == 0) {
      for (int g = 1; g < size_; ++g) recv_all(peers_[g], r + uint64_t(g) * bytes, bytes);
      for (int g = 1; g < size_; ++g) send_all(peers_[g], r, bytes * size_);
    } else {
      send_all(up(), send, bytes);
      recv_all(up(), r, bytes * size_);
    }
  }
  template <typename T>
  void allreduce_sum(T* buf, uint64_t count) {
    if (size_ == 1) return;
    if (rank_ == 0) {
      std::vector<T> tmp(count);
      for (int g = 1; g < size_; ++g) {
        recv_all(peers_[g], tmp.data(), count * sizeof(T));
        for (uint64_t i = 0; i < count; ++i) buf[i] += tmp[i];  // (unsigned: wraps like the device sum)
      }
      for (int g = 1; g < size_; ++g) send_all(peers_[g], buf, count * sizeof(T));
    } else {
      send_all(up(), buf, count * sizeof(T));
      recv_all(up(), buf, count * sizeof(T));
    }
  }
  // block g of send (sbytes[g]) to rank g; recv: the blocks from ranks 0..size-1 (rbytes[g] from rank g)
  void alltoallv(const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes) {
    const int G = size_;
    std::vector<uint64_t> soff(G + 1, 0), roff(G + 1, 0);
    for (int g = 0; g < G; ++g) {
      soff[g + 1] = soff[g] + sbytes[g];
      roff[g + 1] = roff[g] + rbytes[g];
    }
    const char* s = static_cast<const char*>(send);
    char* r = static_cast<char*>(recv);
    if (G == 1) {
      if (sbytes[0] != rbytes[0]) throw std::runtime_error("TcpGroup alltoallv: size mismatch");
      std::memmove(r, s, sbytes[0]);
      return;
    }
    if (rank_ == 0) {
      // every rank's size row and send buffer, then each destination's blocks in source order
      std::vector<std::vector<uint64_t>> sz(G, std::vector<uint64_t>(G));
      std::vector<std::vector<char>> data(G);
      sz[0].assign(sbytes, sbytes + G);
      for (int g = 1; g < G; ++g) {
        recv_all(peers_[g], sz[g].data(), G * sizeof(uint64_t));
        uint64_t tot = 0;
        for (int k = 0; k < G; ++k) tot += sz[g][k];
        data[g].resize(tot);
        recv_all(peers_[g], data[g].data(), tot);
      }
      auto block = [&](int src, int dst) -> const char* {
        const char* base = src == 0 ? s : data[src].data();
        uint64_t o = 0;
        for (int k = 0; k < dst; ++k) o += sz[src][k];
        return base + o;
      };
      for (int src = 0; src < G; ++src) {
        if (sz[src][0] != rbytes[src]) throw std::runtime_error("TcpGroup alltoallv: receive size mismatch");
        std::memcpy(r + roff[src], block(src, 0), sz[src][0]);
      }
      for (int dst = 1; dst < G; ++dst)
        for (int src = 0; src < G; ++src) send_all(peers_[dst], block(src, dst), sz[src][dst]);
    } else {
      send_all(up(), sbytes, G * sizeof(uint64_t));
      send_all(up(), s, soff[G]);
      recv_all(up(), r, roff[G]);
    }
  }
  // every rank's ok flag -> true iff all are ok (a failed rank still calls this)
  bool agree(bool ok) {
    std::vector<uint32_t> all(size_);
    const uint32_t mine = ok ? 1u : 0u;
    allgather(&mine, all.data(), sizeof(uint32_t));
    for (uint32_t x : all)
      if (!x) return false;
    return true;
  }
  void bcast(void* buf, uint64_t bytes) {
    if (size_ == 1) return;
    if (rank_ == 0)
      for (int g = 1; g < size_; ++g) send_all(peers_[g], buf, bytes);
    else
      recv_all(up(), buf, bytes);
  }

  // pm_host_comm over this group (the search's collectives on host buffers)
  pm_host_comm host_comm() {
    pm_host_comm h{};
    h.user = this;
    h.nshards = static_cast<uint32_t>(size_);
    h.shard = static_cast<uint32_t>(rank_);
    h.allgather = [](void* u, const void* s, void* r, uint64_t b) {
      return guarded([&] { static_cast<TcpGroup*>(u)->allgather(s, r, b); });
    };
    h.allreduce_sum_u64 = [](void* u, uint64_t* b, uint64_t n) {
      return guarded([&] { static_cast<TcpGroup*>(u)->allreduce_sum(b, n); });
    };
    h.allreduce_sum_u32 = [](void* u, uint32_t* b, uint64_t n) {
      return guarded([&] { static_cast<TcpGroup*>(u)->allreduce_sum(b, n); });
    };
    h.alltoallv = [](void* u, const void* s, const uint64_t* sb, void* r, const uint64_t* rb) {
      return guarded([&] { static_cast<TcpGroup*>(u)->alltoallv(s, sb, r, rb); });
    };
    return h;
  }

 private:
  template <typename F>
  static int guarded(F&& f) {
    try {
      f();
      return 0;
    } catch (const std::exception&) {
      return 1;
    }
  }
  int up() const { return peers_[0]; }
  static void nodelay(int s) {
    int one = 1;
    ::setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  static void send_all(int s, const void* p, uint64_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
      const ssize_t k = ::send(s, c, n, MSG_NOSIGNAL);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) throw std::runtime_error("TcpGroup: send failed (a peer exited?)");
      c += k;
      n -= static_cast<uint64_t>(k);
    }
  }
  static void recv_all(int s, void* p, uint64_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
      const ssize_t k = ::recv(s, c, n, 0);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) throw std::runtime_error("TcpGroup: receive failed (a peer exited?)");
      c += k;
      n -= static_cast<uint64_t>(k);
    }
  }
  int rank_, size_;
  std::vector<int> peers_;  // rank 0: socket per rank (index 0 unused); others: [0] = rank 0
};

}  // namespace pm
