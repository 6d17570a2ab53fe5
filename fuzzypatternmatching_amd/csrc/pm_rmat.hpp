// GPU R-MAT generator / CSR builder (pm_rmat.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace pm {

struct RmatPlan {
  uint64_t scale = 0;
  uint64_t per_rank = 0;  // undirected edges per generator rank (2^S * 16 / P_gen)
  uint32_t K = 1;         // substreams per rank (power of two)
  uint64_t esub = 0;      // edges per substream (the last one may be shorter or empty)
  uint32_t levels = 0;    // log2 K (jump-tree levels)
};

// Device CSR (row-sorted, with multiplicity); the caller owns d_off / d_col.
struct DevCsr {
  uint64_t n = 0, nnz = 0;
  uint64_t* d_off = nullptr;  // n + 1
  uint32_t* d_col = nullptr;  // nnz
};

RmatPlan rmat_plan(uint64_t scale, uint64_t p_gen);
// 2 * per_rank keys (src << S | dst) per generator rank of vranks, rank after rank.
void rmat_keys_device(const RmatPlan& p, const std::vector<uint64_t>& vranks, uint64_t* d_keys, hipStream_t stream);
// The whole symmetrized graph of P_gen generator ranks on the current device.
DevCsr rmat_csr_device(uint64_t scale, uint64_t p_gen, hipStream_t stream);

struct Comm;
// One shard of a sharded search over the R-MAT graph, built on the current device: this shard
// generates the streams of generator ranks r = shard (mod nshards); every directed entry (u, v)
// travels to its owner -- u % nshards, or v % nshards when u is a delegate (global degree >=
// hub_threshold) -- in one all-to-all; the received entries are radix-sorted into the shard's
// row-sorted CSR (rows it does not hold are empty).  gdeg receives the global degrees (host).
DevCsr rmat_shard_device(uint64_t scale, uint64_t p_gen, uint64_t hub_threshold, Comm& comm, uint32_t nshards,
                         uint32_t shard, std::vector<uint32_t>& gdeg, hipStream_t stream);

}  // namespace pm
