// Host checks of the launched CLI's process group (csrc/host/tcp_group.hpp): `size` forked processes meet
// over TCP at 127.0.0.1:<port>, run every collective the search's pm_host_comm needs with known answers,
// the success agreement with one failing rank, and the pm_host_comm callbacks.  Exit 0 on success.
//   tcp_group_check <port> <size>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host/tcp_group.hpp"

#define CHECK(x)                                                                         \
  do {                                                                                   \
    if (!(x)) {                                                                          \
      std::fprintf(stderr, "rank %d: FAILED %s (line %d)\n", rank, #x, __LINE__);        \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

static int member(int rank, int size, int port) {
  pm::TcpGroup g(rank, size, "127.0.0.1", port, 60.0);
  CHECK(g.rank() == rank && g.size() == size);
  // allgather of ragged content
  std::vector<uint64_t> mine(3), all(3 * size);
  for (int i = 0; i < 3; ++i) mine[i] = uint64_t(rank) * 1000 + i;
  g.allgather(mine.data(), all.data(), 3 * sizeof(uint64_t));
  for (int r = 0; r < size; ++r)
    for (int i = 0; i < 3; ++i) CHECK(all[3 * r + i] == uint64_t(r) * 1000 + i);
  // sums, u32 wrapping like the device's
  std::vector<uint32_t> w(5);
  for (int i = 0; i < 5; ++i) w[i] = 0xFFFFFFF0u + uint32_t(rank) + i;
  g.allreduce_sum(w.data(), w.size());
  for (int i = 0; i < 5; ++i) {
    uint32_t want = 0;
    for (int r = 0; r < size; ++r) want += 0xFFFFFFF0u + uint32_t(r) + i;
    CHECK(w[i] == want);
  }
  std::vector<uint64_t> s64(4, uint64_t(rank + 1) << 40);
  g.allreduce_sum(s64.data(), s64.size());
  for (uint64_t x : s64) CHECK(x == (uint64_t(size) * (size + 1) / 2) << 40);
  // all-to-all-v: rank r sends (r + d) % 3 bytes of value 16 r + d to rank d (some blocks empty)
  std::vector<uint64_t> sb(size), rb(size);
  std::vector<char> send;
  for (int d = 0; d < size; ++d) {
    sb[d] = (rank + d) % 3;
    for (uint64_t k = 0; k < sb[d]; ++k) send.push_back(static_cast<char>(16 * rank + d));
    rb[d] = (d + rank) % 3;
  }
  uint64_t rt = 0;
  for (uint64_t x : rb) rt += x;
  std::vector<char> recv(rt + 1, 0);
  g.alltoallv(send.data(), sb.data(), recv.data(), rb.data());
  uint64_t at = 0;
  for (int s = 0; s < size; ++s)
    for (uint64_t k = 0; k < rb[s]; ++k) CHECK(recv[at++] == static_cast<char>(16 * s + rank));
  // agreement: all ok, then the last rank failing
  CHECK(g.agree(true));
  CHECK(!g.agree(rank != size - 1));
  // broadcast
  uint32_t b = rank == 0 ? 0xC0FFEEu : 0;
  g.bcast(&b, sizeof(b));
  CHECK(b == 0xC0FFEEu);
  // through the pm_host_comm callbacks the library calls
  pm_host_comm h = g.host_comm();
  CHECK(h.nshards == uint32_t(size) && h.shard == uint32_t(rank));
  uint64_t one = rank;
  std::vector<uint64_t> got(size);
  CHECK(h.allgather(h.user, &one, got.data(), sizeof(one)) == 0);
  for (int r = 0; r < size; ++r) CHECK(got[r] == uint64_t(r));
  uint32_t c32 = 1;
  CHECK(h.allreduce_sum_u32(h.user, &c32, 1) == 0 && c32 == uint32_t(size));
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int port = std::atoi(argv[1]), size = std::atoi(argv[2]);
  int rank = -1;
  // launch_env reads a launcher's variables
  setenv("SLURM_PROCID", "2", 1);
  setenv("SLURM_NTASKS", "4", 1);
  setenv("SLURM_LOCALID", "0", 1);
  pm::LaunchEnv e = pm::launch_env();
  CHECK(e.launched && e.rank == 2 && e.size == 4 && e.local_rank == 0 && e.launcher == "Slurm");
  setenv("PM_RANK", "1", 1);
  setenv("PM_WORLD_SIZE", "3", 1);
  e = pm::launch_env();
  CHECK(e.launched && e.rank == 1 && e.size == 3 && e.local_rank == 1 && e.launcher == "PM");
  unsetenv("PM_RANK");
  unsetenv("PM_WORLD_SIZE");
  unsetenv("SLURM_PROCID");
  unsetenv("SLURM_NTASKS");
  unsetenv("SLURM_LOCALID");
  setenv("WORLD_SIZE", "1", 1);
  CHECK(!pm::launch_env().launched);
  std::vector<pid_t> kids;
  for (int r = 1; r < size; ++r) {
    const pid_t p = fork();
    if (p == 0) {
      int rc = 1;
      try {
        rc = member(r, size, port);
      } catch (const std::exception& ex) {
        std::fprintf(stderr, "rank %d: %s\n", r, ex.what());
      }
      _exit(rc);
    }
    kids.push_back(p);
  }
  rank = 0;
  int rc = 1;
  try {
    rc = member(0, size, port);
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "rank 0: %s\n", ex.what());
  }
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  if (rc == 0) std::printf("tcp group OK (%d processes)\n", size);
  return rc;
}
