/*
 * C-ABI of the MI355X-native label-constrained pattern-matching path.
 *
 * The reference exposes this path as C++ templates called from one driver
 * (no FFI exists upstream).  Each entry point below replaces one of those
 * in-process interfaces; a caller that used them binds these instead
 * (INTEGRATION.md shows the ctypes and C++ bindings).
 *
 *   pm_create / pm_destroy        graph open + per-pattern containers:
 *                                 src/run_pattern_matching_beta.cpp:209-223, 307-328, 436-492
 *   pm_vertex_data_degree         vertex_data_db_degree(graph, labels):
 *                                 include/havoqgt/vertex_data_db_degree.hpp:133-151 (formula :109)
 *   pm_vertex_data_set            vertex_data_db(graph, labels, prefix, 10000) (-v):
 *                                 include/havoqgt/vertex_data_db.hpp:197-257
 *   pm_lcc_bsp                    label_propagation_pattern_matching_bsp(...):
 *                                 include/havoqgt/label_propagation_pattern_matching_nonunique_ee.hpp:1029-1153
 *   pm_token_passing              token_passing_pattern_matching(...) -- nem_1 for pl < 4,
 *                                 tds_batch_1 for pl >= 4 (switch at beta.cpp:762-767):
 *                                 include/havoqgt/token_passing_pattern_matching_nonunique_nem_1.hpp:908-939,
 *                                 include/havoqgt/token_passing_pattern_matching_nonunique_tds_batch_1.hpp:967-1324
 *   pm_post_token_passing         unacked-source invalidation + state-map erase:
 *                                 src/run_pattern_matching_beta.cpp:956-1071
 *   pm_run_beta                   the whole do { LCC; NLCC lines } while loop and every
 *                                 result file: src/run_pattern_matching_beta.cpp:539-1425
 *   pm_export_state               vertex_state_map / template_vertices / vertex_active_edges_map
 *                                 read-out used by the result writers (beta.cpp:1386-1425)
 *   pm_create_shard               one rank of the delegate-partitioned graph (owner = id % P,
 *                                 include/havoqgt/delegate_partitioned_graph.ipp:1679-1696) with the
 *                                 mailbox exchange (include/havoqgt/new_mailbox.hpp:289-713) and the
 *                                 delegate reductions (impl/vertex_data.hpp:114-126) replaced by RCCL
 *                                 collectives between supersteps
 *   pm_comm_unique_id             the RCCL communicator id rank 0 hands to every rank (the role of
 *                                 MPI_COMM_WORLD set up by havoqgt_init, environment.hpp:136-228)
 *   pm_rmat_edges                 the edge stream of some generator ranks of generate_rmat
 *                                 (src/generate_rmat.cpp:202-213, rmat_edge_generator.hpp:218-261)
 *   pm_rmat_csr_gpu               generate_rmat's graph construction (generate_rmat.cpp:196-213 ->
 *                                 delegate_partitioned_graph ctor, ipp:70-167, CSR fill ipp:818-969)
 *                                 built on the GPU: MT19937 jump-ahead substreams + radix-sorted CSR
 *   pm_create_rmat                generate_rmat + graph open (beta.cpp:209-223) in one step with the
 *                                 adjacency never leaving HBM (north_star scale-28 configuration)
 *   pm_ingest_edge_list_gpu       ingest_edge_list's text parse + graph construction
 *                                 (src/ingest_edge_list.cpp:164-240, parallel_edge_list_reader.hpp:242-266,
 *                                 delegate_partitioned_graph ctor ipp:70-167) parsed and sorted on the GPU
 *   pm_create_edge_list           ingest_edge_list + graph open (beta.cpp:209-223) with the adjacency
 *                                 never leaving HBM (config C5)
 *   pm_vertex_data_files          vertex_data_db(graph, labels, prefix, 10000) (-v) parsed on the GPU:
 *                                 include/havoqgt/vertex_data_db.hpp:137-257
 *   pm_create_shard_host_comm     pm_create_shard with the exchanges through caller-supplied host
 *                                 collectives (pm_host_comm): the reference's own MPI transport
 *                                 (new_mailbox.hpp:358-405, impl/vertex_data.hpp:114-126) or a gloo group
 *   pm_run_rmat_local_shards2     the N-rank delegate partition of generate_rmat's graph
 *                                 (delegate_partitioned_graph.ipp:1402-1648, 346-355) run as N shards on
 *                                 one device, with every shard's statistics (balance / N-GPU projection)
 *
 * Conventions: plain C types; int status (0 = OK, negative = error with
 * pm_last_error()); device memory is owned by the context; host buffers are
 * owned by the caller; one host thread per context.  There is NO CPU
 * fallback: pm_create fails when no gfx950 device / HIP kernel image is
 * available.
 */
#ifndef PM_ABI_H_
#define PM_ABI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pm_ctx pm_ctx;

typedef struct pm_graph_desc {
  uint64_t n;            /* number of vertex ids (max id + 1)                     */
  const uint64_t* off;   /* n + 1 CSR row offsets (host memory)                   */
  const uint32_t* col;   /* off[n] targets, sorted within each row (host memory)  */
  int32_t symmetric;     /* 1: every (u,v) has a matching (v,u)                    */
  uint32_t nranks;       /* P used to name per-rank result files (owner rule)      */
  uint64_t hub_threshold;/* delegate threshold (-d) used by the owner rule         */
} pm_graph_desc;

typedef struct pm_lcc_stats {
  uint64_t supersteps;
  uint64_t edges_traversed;     /* adjacency entries scanned by senders            */
  uint64_t active_vertices;     /* |S| after the last superstep                     */
  uint64_t active_edges;        /* sum |M[v]| over S after the last superstep       */
  uint32_t not_finished;        /* some vertex was removed from S in a verify        */
  uint32_t reserved;
} pm_lcc_stats;

typedef struct pm_tp_stats {
  uint64_t sources;
  uint64_t acked_sources;
  uint64_t edges_traversed;     /* adjacency entries scanned by initiators/relays  */
  uint64_t tokens;              /* tokens / partial walks created                   */
  uint64_t walks;               /* complete TDS walks (0 for path/cycle lines)      */
} pm_tp_stats;

typedef struct pm_run_stats {
  uint64_t iterations;
  uint32_t terminated;          /* 0 when max_iterations stopped the loop           */
  uint32_t hubs;                /* delegates: vertices of degree >= hub_threshold    */
  uint64_t lcc_edges;
  uint64_t nlcc_edges;
  uint64_t tds_edges;
  uint64_t walks;               /* complete walks of the last TDS line run          */
  uint64_t final_vertices;
  uint64_t final_edges;
  double seconds;               /* pattern_time_start -> pattern_time_end           */
  double device_seconds;        /* sum of device-event time inside the loop         */
  double lcc_first_kernel_ms;   /* duration of the fused superstep-0 scan kernel    */
  uint64_t lcc_first_bytes;     /* algorithmic bytes of that kernel                 */
  uint64_t tds_chunks;          /* chunk launches of exact-path TDS enumerations (0: every TDS line ran in
                                   the fused kernel; see run_tds_line, PM_TDS_CAP)    */
  double nlcc_seconds;          /* NLC lines of the search: device time of the fused line launches (first
                                   block start to the last line's end) + host time of exact-path lines */
  uint64_t split_lines;         /* NLC lines run split: sharded, by owner (sources over the shards); one
                                   context, in local parts after the fused kernel's table or walk storage
                                   overflowed                                            */
  uint64_t line_overflows;      /* fused NLC launches that overflowed a capacity (the line reran with a grown
                                   table, or on the exact path)                                          */
  uint64_t exact_lines;         /* NLC lines run on the exact per-position path                          */
  /* This context's share of the work (a shard's own rows; the whole graph on one context):             */
  uint64_t shard_entries;       /* adjacency entries held: owned rows + delegate shares                  */
  uint64_t shard_rows;          /* nonempty rows held                                                     */
  uint64_t shard_hub_entries;   /* entries of the delegate shares held                                   */
  uint64_t shard_hubs_controlled; /* delegates whose state this shard holds (hub ordinal % nshards)      */
  uint64_t shard_ss0_entries;   /* adjacency entries of label-matching rows superstep 0 scanned here     */
  uint64_t shard_ss0_survivors; /* superstep-0 survivors of this shard's rows                            */
  double shard_sharded_ms;      /* device time of the sharded part of the search (its start to the replica
                                   hand-off) less the collectives' host time; 0 on one context            */
  uint64_t comm_calls;          /* collectives the search issued                                          */
  uint64_t comm_bytes;          /* bytes this shard contributed to them                                   */
  uint64_t replica_rows;        /* rows / M entries of the replica at the hand-off                       */
  uint64_t replica_entries;
  double comm_seconds;          /* host time inside the collectives of the search                        */
  uint64_t path_batches;        /* initiator batches of the exact-path path / cycle lines (one per line unless
                                   a line's tokens did not fit the device scratch arena at once)          */
} pm_run_stats;

/* One shard (rank) of a sharded search: the rows of ids v % nshards == shard. */
typedef struct pm_shard_desc {
  uint64_t n;               /* global number of vertex ids                                   */
  const uint64_t* off;      /* n + 1 offsets by id: the owned rows, every other row empty    */
  const uint32_t* col;      /* off[n] targets of the owned rows, sorted within each row      */
  const uint32_t* degree;   /* n global degrees (degree labels, label-major order)           */
  int32_t symmetric;
  uint32_t nranks;          /* P used to name per-rank result files (owner rule)              */
  uint64_t hub_threshold;
  uint32_t nshards;         /* shards of the search (one per GPU / process)                  */
  uint32_t shard;
} pm_shard_desc;

/* Context: uploads the CSR to device `device`, loads <pattern_dir>/0/pattern_*.
 * Returns NULL on failure (message via pm_last_error(NULL)). */
pm_ctx* pm_create(const pm_graph_desc* graph, const char* pattern_dir, int device);
void pm_destroy(pm_ctx* ctx);
const char* pm_last_error(const pm_ctx* ctx);

/* Labels. */
int pm_vertex_data_degree(pm_ctx* ctx);
int pm_vertex_data_set(pm_ctx* ctx, const uint64_t* labels /* n entries, host */);

/* -v <prefix>: every file basename(prefix).* in dirname(prefix), in name order, lines "vid label"
 * parsed on the device (last line wins, unlisted vertices keep 0; vertex_data_db.hpp:176-257). */
int pm_vertex_data_files(pm_ctx* ctx, const char* prefix);

/* Per-pattern reset: every vertex active, empty state map (beta.cpp:484-492). */
int pm_reset(pm_ctx* ctx);

/* One LCC call: exactly `diameter` supersteps (nonunique_ee.hpp:1069). */
int pm_lcc_bsp(pm_ctx* ctx, int init_step, uint64_t itr, pm_lcc_stats* out);

/* One NLC line (index pl): path/cycle walk for pl < 4, TDS for pl >= 4. */
int pm_token_passing(pm_ctx* ctx, uint32_t pl, pm_tp_stats* out);

/* One TDS line (pl >= 4) with its kept walks handed to `sink` instead of a subgraph
 * file: the reference writes each walk as "[rank], v0, ..., vk, [vk]" into its open
 * stream (token_passing_pattern_matching_nonunique_tds_batch_1.hpp:739-743, the
 * stream opened by run_pattern_matching_beta.cpp:713-717); here the sink gets that
 * rank (owner of the last vertex), the vertex ids v0..vk and k + 1.  The walk array
 * is valid during the call only.  Single-GPU contexts. */
typedef void (*pm_path_sink)(void* user, uint32_t rank, const uint32_t* vertices, uint32_t length);
int pm_tds(pm_ctx* ctx, uint32_t pl, pm_path_sink sink, void* user, pm_tp_stats* out);

/* Post-processing of the last pm_token_passing call; *deleted = any source invalidated. */
int pm_post_token_passing(pm_ctx* ctx, uint32_t pl, uint32_t* deleted);

/* Whole driver loop + result files under result_dir (must exist; "" = no files).
 * max_iterations caps the do/while loop (0 = unlimited, as in the reference). */
int pm_run_beta(pm_ctx* ctx, const char* result_dir, uint64_t max_iterations, pm_run_stats* out);

/* State read-out: tpub[n] (0 = not in S), moff/mlen per vertex and the alive
 * neighbour ids.  Any pointer may be NULL.  *n_edges receives sum |M[v]| over S;
 * nbrs must hold that many entries, written row by row in vertex order. */
int pm_export_state(pm_ctx* ctx, uint16_t* tpub, uint32_t* mdeg, uint32_t* nbrs, uint64_t* n_edges);

/* Sharded search, one process per GPU: rank 0 creates the id (>= 128 bytes, returns its
 * length), every rank receives it and calls pm_create_shard collectively; pm_run_beta,
 * pm_lcc_bsp, pm_vertex_data_* and pm_export_state are then collective over the shards.
 * Result files and pm_run_stats cover the whole graph (shard 0 writes the files). */
int pm_comm_unique_id(uint8_t* out, uint64_t len);
pm_ctx* pm_create_shard(const pm_shard_desc* shard, const char* pattern_dir, int device, const uint8_t* unique_id);

/* Host-staged collectives supplied by the caller, for sharded searches whose processes exchange through
 * the host instead of RCCL: an MPI communicator (the reference's transport, new_mailbox.hpp:358-405 and the
 * delegate reductions of impl/vertex_data.hpp:114-126), a torch.distributed gloo group, or several processes
 * sharing one device.  Every function is collective over the nshards processes, is called by every shard in
 * the same order, gets host buffers and returns 0 on success:
 *   allgather: recv receives nshards consecutive blocks of `bytes` (block g = shard g's send);
 *   allreduce_sum_u64 / _u32: element-wise sum in place (wrapping);
 *   alltoallv: block g of send (sbytes[g] bytes, blocks consecutive) goes to shard g; recv holds the blocks
 *              from shards 0..nshards-1 consecutively (rbytes[g] bytes from shard g). */
typedef struct pm_host_comm {
  void* user;
  uint32_t nshards;
  uint32_t shard;
  int (*allgather)(void* user, const void* send, void* recv, uint64_t bytes);
  int (*allreduce_sum_u64)(void* user, uint64_t* buf, uint64_t count);
  int (*allreduce_sum_u32)(void* user, uint32_t* buf, uint64_t count);
  int (*alltoallv)(void* user, const void* send, const uint64_t* sbytes, void* recv, const uint64_t* rbytes);
} pm_host_comm;

/* pm_create_shard with the exchanges through `comm` (copied; its functions and user pointer must stay valid
 * for the context's lifetime).  comm->nshards / comm->shard must equal shard->nshards / shard->shard. */
pm_ctx* pm_create_shard_host_comm(const pm_shard_desc* shard, const char* pattern_dir, int device,
                                  const pm_host_comm* comm);

/* nshards shards of one search run by threads of this process on one device (the
 * partitioning of pm_create_shard with an in-process exchange): parity of the sharded
 * path on a single GPU.  labels may be NULL (degree labels). */
int pm_run_beta_local_shards(const pm_graph_desc* graph, const char* pattern_dir, int device, uint32_t nshards,
                             const uint64_t* labels, const char* result_dir, uint64_t max_iterations,
                             pm_run_stats* out);

/* One shard of a sharded search over the R-MAT graph of generate_rmat, built on the device
 * (collective over the nshards processes): shard q generates the edge streams of generator ranks
 * r = q (mod nshards) (src/generate_rmat.cpp:202-213), every directed entry travels to its owner in
 * one RCCL all-to-all -- the source's owner id % nshards, or for a delegate (global degree >=
 * hub_threshold) the target's owner (delegate_partitioned_graph.ipp:818-969, 1402-1648) -- and
 * the received entries are sorted into the shard's rows.  Same input as pm_create_rmat for every
 * nshards.  gen_seconds (may be NULL): generation + exchange + row build. */
pm_ctx* pm_create_rmat_shard(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nranks,
                             uint64_t hub_threshold, uint32_t nshards, uint32_t shard, const uint8_t* unique_id,
                             double* gen_seconds);
/* The same with nshards shards driven by threads of this process on one device (in-process exchange):
 * the whole sharded path -- generation, all-to-all, delegates, replica -- on a one-GPU box. */
int pm_run_rmat_local_shards(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nshards,
                             uint32_t nranks, uint64_t hub_threshold, const char* result_dir, uint64_t max_iterations,
                             pm_run_stats* out);
/* The same with labels (NULL: degree labels), the search run `repeats` times (>= 1; result files from the
 * first run, statistics from the last) and every shard's statistics: per_shard[q] for q < nshards (the
 * partition balance and per-shard device times of the N-GPU layout, measured with the shards on one device). */
int pm_run_rmat_local_shards2(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nshards,
                              uint32_t nranks, uint64_t hub_threshold, const uint64_t* labels, const char* result_dir,
                              uint64_t max_iterations, uint32_t repeats, pm_run_stats* per_shard);

/* The same with every shard's statistics (per_shard[q], q < nshards; may be NULL), the search run `repeats`
 * times (result files from the first run) and -v label files: label_prefix (NULL: `labels`, or degree labels
 * when both are NULL) is parsed on the device once and shared by the shards (vertex_data_db.hpp:137-257).
 * The drop-in executable's mode for a P-partition graph on fewer GPUs than P (run_pattern_matching_beta). */
int pm_run_beta_local_shards2(const pm_graph_desc* graph, const char* pattern_dir, int device, uint32_t nshards,
                              const uint64_t* labels, const char* label_prefix, const char* result_dir,
                              uint64_t max_iterations, uint32_t repeats, pm_run_stats* per_shard);

/* Graph files of a sharded run.  pm_graph_partitions: P of <base>_<r>_of_<P> (-1: none found).
 * pm_read_graph_shard: shard `shard` of `nshards` read straight from the files, as pm_create_shard takes it --
 * the rows of ids v % nshards == shard whole, of a delegate (degree >= the files' hub threshold, nshards > 1)
 * the entries whose target that shard owns (delegate_partitioned_graph.ipp:1402-1648), every other row empty
 * -- plus the n global degrees.  Each rank of a launch reads its own shard (distributed_db.hpp:353-357 opens
 * <base>_<rank>_of_<P>; here every file's row index is read for the global degrees, and only the held entries
 * are copied).  off (n + 1), col (>= 1 element), degree (n) are malloc'ed (pm_free_host). */
int pm_graph_partitions(const char* base);
int pm_read_graph_shard(const char* base, uint32_t nshards, uint32_t shard, uint64_t** off, uint32_t** col,
                        uint32_t** degree, uint64_t* n, int* symmetric, uint32_t* nranks, uint64_t* hub_threshold);

/* HIP devices visible to this process (0 without a GPU; no context is created). */
int pm_device_count(void);

/* A context's place in its search: shard count, its shard, the ranks of its communicator as the transport
 * reports them (RCCL: ncclCommCount; 0 on a one-context search) and the transport. */
#define PM_TRANSPORT_NONE 0    /* one context, no exchange                                      */
#define PM_TRANSPORT_RCCL 1    /* RCCL over xGMI, one rank per GPU                               */
#define PM_TRANSPORT_HOST 2    /* caller's host collectives (pm_host_comm: MPI, gloo, TCP)      */
#define PM_TRANSPORT_THREADS 3 /* in-process shards on one device                                */
int pm_comm_info(const pm_ctx* ctx, uint32_t* nshards, uint32_t* shard, int32_t* comm_ranks, int32_t* transport);

/* Host-side input builders (no device needed). */
/* Directed pairs (u,v),(v,u) of generator ranks first, first + stride, ... < p_gen. */
int pm_rmat_edges(uint64_t scale, uint64_t p_gen, uint64_t first, uint64_t stride, uint32_t** src, uint32_t** dst,
                  uint64_t* m);
int pm_rmat_csr(uint64_t scale, uint64_t p_gen, uint64_t** off, uint32_t** col, uint64_t* n);
void pm_free_host(void* p);

/* GPU generator: bit-identical to pm_rmat_csr (same stream, same sorted CSR), built on `device`. */
int pm_rmat_csr_gpu(uint64_t scale, uint64_t p_gen, int device, uint64_t** off, uint32_t** col, uint64_t* n);
/* Context over a GPU-generated R-MAT graph (degree labels, no host copy of the adjacency).
 * gen_seconds (may be NULL) receives the generation + CSR build wall time. */
pm_ctx* pm_create_rmat(uint64_t scale, uint64_t p_gen, const char* pattern_dir, int device, uint32_t nranks,
                       uint64_t hub_threshold, double* gen_seconds);
/* GPU text ingest: files of "src dst [weight]" lines (lines that do not start with two numbers are
 * skipped; ids above 2^32 - 2 are an error), undirected != 0 adds (dst, src) for every edge.  Returns
 * the row-sorted CSR with multiplicity (malloc'ed, pm_free_host) and whether it is symmetric. */
int pm_ingest_edge_list_gpu(const char* const* files, uint32_t nfiles, int undirected, int device, uint64_t** off,
                            uint32_t** col, uint64_t* n, int* symmetric);
/* Context over a GPU-ingested text graph (degree labels; no host copy of the adjacency).
 * ingest_seconds (may be NULL) receives the parse + CSR build wall time. */
pm_ctx* pm_create_edge_list(const char* const* files, uint32_t nfiles, int undirected, const char* pattern_dir,
                            int device, uint32_t nranks, uint64_t hub_threshold, double* ingest_seconds);
/* Size of the graph a context holds (vertex ids, directed entries, symmetric flag); any pointer may be NULL. */
int pm_graph_size(const pm_ctx* ctx, uint64_t* n, uint64_t* nnz, int* symmetric);
/* Host check of the MT19937 jump-ahead (no device): outputs skip .. skip+count-1 of mt19937(seed). */
int pm_mt19937_jump_outputs(uint32_t seed, uint64_t skip, uint32_t* out, uint64_t count);
int pm_write_graph(const char* base, uint64_t n, const uint64_t* off, const uint32_t* col, int symmetric,
                   uint32_t nranks, uint64_t hub_threshold);
int pm_read_graph(const char* base, uint64_t** off, uint32_t** col, uint64_t* n, int* symmetric,
                  uint32_t* nranks, uint64_t* hub_threshold);

/* Test-input writers (config C5 at size: a text edge list and -v label files too large for Python).
 * pm_write_rmat_text: the undirected R-MAT edge stream of every generator rank r < p_gen, generated on
 * `device` and written as "u v" lines to <base>.<r> (formatted on host threads); bytes_out: text bytes.
 * pm_write_label_text: "v labels[v]" lines for v < n, split into nfiles files <prefix>.<i>. */
int pm_write_rmat_text(uint64_t scale, uint64_t p_gen, int device, const char* base, uint64_t* bytes_out);
int pm_write_label_text(const uint64_t* labels, uint64_t n, const char* prefix, uint32_t nfiles, uint64_t* bytes_out);

/* Parsed pattern directory as JSON text (host only; loader check). */
int pm_pattern_summary(const char* pattern_dir, char* buf, uint64_t buflen);

/* Diagnostics: average time of `reps` launches of superstep-0 kernel variant
 * (0 = product kernel; others are ablation builds used by tools/ubench.py). */
int pm_debug_time_lcc_first(pm_ctx* ctx, int variant, int reps, float* ms_out);
/* Diagnostics: a one-rank RCCL collective of `bytes` (op 0 ncclAllGather, 1 ncclAllReduce u64 sum),
   result checked: 0 = right, 1 = wrong, -1 = error (pm_last_error). */
int pm_debug_rccl_selftest(int device, uint64_t bytes, int op);
/* Diagnostics: HBM copy bandwidth of a 16-B nontemporal copy kernel over two `bytes` buffers (read + write
   bytes per second / 1e9), the measured ceiling beside the datasheet peak. */
int pm_debug_copy_gbs(int device, uint64_t bytes, int reps, double* gbs);
/* Diagnostics: the floor of the first later superstep's neighbour-T_pub gathers: superstep 0
   runs, its light survivors' alive M entries are collected as code indices in record order, and gather-only
   kernels are timed over them (variant 0 record order, 1 index stream only, 2 XCD-sliced buckets, 3 the buckets
   spread over every XCD, 4 uniformly random, 5 sorted, 6 distinct-line misses of a 4 GiB buffer (FETCH_SIZE calibration),
   7 the bucketing pass).  info[0] entries, [1] checksum of the gathered codes, [2] code array bytes. */
int pm_debug_gather_floor(pm_ctx* ctx, int variant, int reps, float* ms_out, uint64_t* info);
/* Diagnostics: superstep-0 tiling statistics (real entries, loaded slots, rows, tiles, ranges, heavy rows). */
int pm_debug_layout_stats(pm_ctx* ctx, uint64_t* out, uint64_t n);

/* Diagnostics: T_pub census (both ping-pong buffers) -- out[0], out[1]: nonzero entries of buffer 0 / 1,
   out[2]: positions with a nonzero entry in either buffer that are not in the current slist (the invariant
   the search-start clear relies on: 0).  deferred_reset != 0 first runs the search start's reset as a search
   does (deferred, then flushed in one launch), so out[0..2] must all be 0 afterwards. */
int pm_debug_tpub_census(pm_ctx* ctx, int deferred_reset, uint64_t* out);

/* Build info: returns the offload arch the kernels were compiled for ("gfx950"). */
const char* pm_build_arch(void);

#ifdef __cplusplus
}
#endif

#endif /* PM_ABI_H_ */
