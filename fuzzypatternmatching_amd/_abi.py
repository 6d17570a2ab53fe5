"""ctypes binding of the C-ABI declared in include/pm_abi.h.

The shared library lib/libpm.so (HIP kernels for gfx950 + host driver) is the
product; this module only declares signatures.  It fails loudly when the
library is missing: there is no Python or CPU fallback for the hot path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PM_LIB") or os.path.join(_HERE, "lib", "libpm.so")  # PM_LIB: diagnostic builds

c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_i32 = ctypes.c_int32
c_vp = ctypes.c_void_p
c_char_p = ctypes.c_char_p


class GraphDesc(ctypes.Structure):
    _fields_ = [
        ("n", c_u64),
        ("off", c_vp),
        ("col", c_vp),
        ("symmetric", c_i32),
        ("nranks", c_u32),
        ("hub_threshold", c_u64),
    ]


class ShardDesc(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("off", ctypes.c_void_p),
        ("col", ctypes.c_void_p),
        ("degree", ctypes.c_void_p),
        ("symmetric", ctypes.c_int32),
        ("nranks", ctypes.c_uint32),
        ("hub_threshold", ctypes.c_uint64),
        ("nshards", ctypes.c_uint32),
        ("shard", ctypes.c_uint32),
    ]


# pm_host_comm callbacks (include/pm_abi.h): host buffers, 0 on success
HostAllgather = ctypes.CFUNCTYPE(ctypes.c_int, c_vp, c_vp, c_vp, c_u64)
HostAllreduce64 = ctypes.CFUNCTYPE(ctypes.c_int, c_vp, c_vp, c_u64)
HostAllreduce32 = ctypes.CFUNCTYPE(ctypes.c_int, c_vp, c_vp, c_u64)
HostAlltoallv = ctypes.CFUNCTYPE(ctypes.c_int, c_vp, c_vp, c_vp, c_vp, c_vp)


class HostComm(ctypes.Structure):
    _fields_ = [
        ("user", c_vp),
        ("nshards", c_u32),
        ("shard", c_u32),
        ("allgather", HostAllgather),
        ("allreduce_sum_u64", HostAllreduce64),
        ("allreduce_sum_u32", HostAllreduce32),
        ("alltoallv", HostAlltoallv),
    ]


class LccStats(ctypes.Structure):
    _fields_ = [
        ("supersteps", c_u64),
        ("edges_traversed", c_u64),
        ("active_vertices", c_u64),
        ("active_edges", c_u64),
        ("not_finished", c_u32),
        ("reserved", c_u32),
    ]


# void (*)(void* user, uint32_t rank, const uint32_t* vertices, uint32_t length)
PathSink = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32)


class TpStats(ctypes.Structure):
    _fields_ = [
        ("sources", c_u64),
        ("acked_sources", c_u64),
        ("edges_traversed", c_u64),
        ("tokens", c_u64),
        ("walks", c_u64),
    ]


class RunStats(ctypes.Structure):
    _fields_ = [
        ("iterations", c_u64),
        ("terminated", c_u32),
        ("hubs", c_u32),
        ("lcc_edges", c_u64),
        ("nlcc_edges", c_u64),
        ("tds_edges", c_u64),
        ("walks", c_u64),
        ("final_vertices", c_u64),
        ("final_edges", c_u64),
        ("seconds", ctypes.c_double),
        ("device_seconds", ctypes.c_double),
        ("lcc_first_kernel_ms", ctypes.c_double),
        ("lcc_first_bytes", c_u64),
        ("tds_chunks", c_u64),
        ("nlcc_seconds", ctypes.c_double),
        ("split_lines", c_u64),
        ("line_overflows", c_u64),
        ("exact_lines", c_u64),
        ("shard_entries", c_u64),
        ("shard_rows", c_u64),
        ("shard_hub_entries", c_u64),
        ("shard_hubs_controlled", c_u64),
        ("shard_ss0_entries", c_u64),
        ("shard_ss0_survivors", c_u64),
        ("shard_sharded_ms", ctypes.c_double),
        ("comm_calls", c_u64),
        ("comm_bytes", c_u64),
        ("replica_rows", c_u64),
        ("replica_entries", c_u64),
        ("comm_seconds", ctypes.c_double),
        ("path_batches", c_u64),
    ]

    def as_dict(self):
        return {f[0]: getattr(self, f[0]) for f in self._fields_ if f[0] != "reserved"}


# (name, restype, argtypes) -- every symbol include/pm_abi.h declares.
SIGNATURES = [
    ("pm_create", c_vp, [ctypes.POINTER(GraphDesc), c_char_p, ctypes.c_int]),
    ("pm_destroy", None, [c_vp]),
    ("pm_last_error", c_char_p, [c_vp]),
    ("pm_vertex_data_degree", ctypes.c_int, [c_vp]),
    ("pm_vertex_data_set", ctypes.c_int, [c_vp, c_vp]),
    ("pm_reset", ctypes.c_int, [c_vp]),
    ("pm_lcc_bsp", ctypes.c_int, [c_vp, ctypes.c_int, c_u64, ctypes.POINTER(LccStats)]),
    ("pm_token_passing", ctypes.c_int, [c_vp, c_u32, ctypes.POINTER(TpStats)]),
    ("pm_tds", ctypes.c_int, [c_vp, c_u32, c_vp, c_vp, ctypes.POINTER(TpStats)]),
    ("pm_post_token_passing", ctypes.c_int, [c_vp, c_u32, ctypes.POINTER(c_u32)]),
    ("pm_run_beta", ctypes.c_int, [c_vp, c_char_p, c_u64, ctypes.POINTER(RunStats)]),
    ("pm_export_state", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(c_u64)]),
    ("pm_rmat_csr", ctypes.c_int, [c_u64, c_u64, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_u64)]),
    ("pm_free_host", None, [c_vp]),
    ("pm_write_graph", ctypes.c_int, [c_char_p, c_u64, c_vp, c_vp, ctypes.c_int, c_u32, c_u64]),
    ("pm_read_graph", ctypes.c_int, [c_char_p, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_u64),
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(c_u32), ctypes.POINTER(c_u64)]),
    ("pm_pattern_summary", ctypes.c_int, [c_char_p, c_char_p, c_u64]),
    ("pm_debug_time_lcc_first", ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]),
    ("pm_debug_gather_floor", ctypes.c_int,
     [c_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64)]),
    ("pm_debug_layout_stats", ctypes.c_int, [c_vp, c_vp, ctypes.c_uint64]),
    ("pm_debug_tpub_census", ctypes.c_int, [c_vp, ctypes.c_int, c_vp]),
    ("pm_write_rmat_text", ctypes.c_int, [c_u64, c_u64, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(c_u64)]),
    ("pm_write_label_text", ctypes.c_int, [c_vp, c_u64, ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(c_u64)]),
    ("pm_debug_copy_gbs", ctypes.c_int, [ctypes.c_int, c_u64, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    ("pm_debug_rccl_selftest", ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_int]),
    ("pm_build_arch", c_char_p, []),
    ("pm_comm_unique_id", ctypes.c_int, [c_vp, c_u64]),
    ("pm_create_shard", c_vp, [ctypes.POINTER(ShardDesc), c_char_p, ctypes.c_int, c_vp]),
    ("pm_create_shard_host_comm", c_vp, [ctypes.POINTER(ShardDesc), c_char_p, ctypes.c_int,
                                         ctypes.POINTER(HostComm)]),
    ("pm_run_beta_local_shards", ctypes.c_int, [ctypes.POINTER(GraphDesc), c_char_p, ctypes.c_int, c_u32, c_vp,
                                                c_char_p, c_u64, ctypes.POINTER(RunStats)]),
    ("pm_rmat_edges", ctypes.c_int, [c_u64, c_u64, c_u64, c_u64, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_u64)]),
    ("pm_rmat_csr_gpu", ctypes.c_int, [c_u64, c_u64, ctypes.c_int, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                       ctypes.POINTER(c_u64)]),
    ("pm_create_rmat", c_vp, [c_u64, c_u64, c_char_p, ctypes.c_int, c_u32, c_u64, ctypes.POINTER(ctypes.c_double)]),
    ("pm_create_rmat_shard", c_vp, [c_u64, c_u64, c_char_p, ctypes.c_int, c_u32, c_u64, c_u32, c_u32, c_vp,
                                    ctypes.POINTER(ctypes.c_double)]),
    ("pm_run_rmat_local_shards", ctypes.c_int, [c_u64, c_u64, c_char_p, ctypes.c_int, c_u32, c_u32, c_u64, c_char_p,
                                                c_u64, ctypes.POINTER(RunStats)]),
    ("pm_run_rmat_local_shards2", ctypes.c_int, [c_u64, c_u64, c_char_p, ctypes.c_int, c_u32, c_u32, c_u64, c_vp,
                                                 c_char_p, c_u64, c_u32, ctypes.POINTER(RunStats)]),
    ("pm_mt19937_jump_outputs", ctypes.c_int, [c_u32, c_u64, c_vp, c_u64]),
    ("pm_vertex_data_files", ctypes.c_int, [c_vp, c_char_p]),
    ("pm_graph_size", ctypes.c_int, [c_vp, ctypes.POINTER(c_u64), ctypes.POINTER(c_u64), ctypes.POINTER(ctypes.c_int)]),
    ("pm_ingest_edge_list_gpu", ctypes.c_int, [c_vp, c_u32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_vp),
                                               ctypes.POINTER(c_vp), ctypes.POINTER(c_u64),
                                               ctypes.POINTER(ctypes.c_int)]),
    ("pm_create_edge_list", c_vp, [c_vp, c_u32, ctypes.c_int, c_char_p, ctypes.c_int, c_u32, c_u64,
                                   ctypes.POINTER(ctypes.c_double)]),
    ("pm_run_beta_local_shards2", ctypes.c_int, [ctypes.POINTER(GraphDesc), c_char_p, ctypes.c_int, c_u32, c_vp,
                                                 c_char_p, c_char_p, c_u64, c_u32, ctypes.POINTER(RunStats)]),
    ("pm_graph_partitions", ctypes.c_int, [c_char_p]),
    ("pm_read_graph_shard", ctypes.c_int, [c_char_p, c_u32, c_u32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                           ctypes.POINTER(c_vp), ctypes.POINTER(c_u64), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(c_u32), ctypes.POINTER(c_u64)]),
    ("pm_device_count", ctypes.c_int, []),
    ("pm_comm_info", ctypes.c_int, [c_vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32)]),
]

TRANSPORTS = {0: "none", 1: "rccl", 2: "host", 3: "threads"}  # PM_TRANSPORT_* (include/pm_abi.h)

_lib = None


def load():
    """Loads lib/libpm.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP path has no fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
