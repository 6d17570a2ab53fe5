"""MI355X-native label-constrained pattern matching (HavoqGT run_pattern_matching_beta hot path).

Host-side mirror of the reference's driver interface.  The compute runs in
lib/libpm.so (hand-written HIP kernels for gfx950) behind the C-ABI in
include/pm_abi.h; this module owns host buffers and forwards calls.

    g = rmat_graph(scale=16, p_gen=4)          # generate_rmat.cpp semantics
    m = PatternMatcher(g, "patterns/rmat_log2_tree_pattern")
    stats = m.run_beta("/tmp/results")          # run_pattern_matching_beta.cpp:539-1425
"""
import ctypes
import os

import numpy as np

from . import _abi

__all__ = ["Graph", "rmat_graph", "rmat_matcher", "rmat_shard_matcher", "mt19937_jump_outputs", "rmat_edges",
           "pattern_summary", "write_graph", "read_graph", "PatternMatcher", "ShardedPatternMatcher", "partition_edges",
           "comm_unique_id", "run_beta_local_shards", "run_beta_local_shards_each", "run_rmat_local_shards",
           "run_rmat_local_shards_each", "read_graph_shard", "graph_partitions", "device_count", "TorchHostComm",
           "PMError"]

DEFAULT_HUB_THRESHOLD = 1048576  # generate_rmat.cpp:106


class PMError(RuntimeError):
    pass


class Graph:
    """Row-sorted CSR with multiplicity: off[n+1] (u64), col[off[n]] (u32)."""

    def __init__(self, off, col, symmetric=True, nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD):
        self.off = np.ascontiguousarray(off, dtype=np.uint64)
        self.col = np.ascontiguousarray(col, dtype=np.uint32)
        self.n = int(self.off.shape[0] - 1)
        self.symmetric = bool(symmetric)
        self.nranks = int(nranks)
        self.hub_threshold = int(hub_threshold)

    @property
    def nnz(self):
        return int(self.off[-1])

    def degrees(self):
        return np.diff(self.off)

    @staticmethod
    def from_edges(src, dst, n=None, symmetric=None, nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD):
        """Directed edge list (with multiplicity) -> row-sorted CSR."""
        src = np.asarray(src, dtype=np.uint64)
        dst = np.asarray(dst, dtype=np.uint64)
        if n is None:
            n = int(max(src.max(initial=0), dst.max(initial=0)) + 1) if src.size else 0
        order = np.lexsort((dst, src))
        src, dst = src[order], dst[order]
        off = np.zeros(n + 1, dtype=np.uint64)
        np.add.at(off, src.astype(np.int64) + 1, 1)
        off = np.cumsum(off).astype(np.uint64)
        if symmetric is None:
            fwd = np.stack([src, dst], 1)
            rev = np.stack([dst, src], 1)
            a = fwd[np.lexsort((fwd[:, 1], fwd[:, 0]))]
            b = rev[np.lexsort((rev[:, 1], rev[:, 0]))]
            symmetric = bool(np.array_equal(a, b))
        return Graph(off, dst.astype(np.uint32), symmetric, nranks, hub_threshold)


def _lib():
    return _abi.load()


def _err(ctx=None):
    msg = _lib().pm_last_error(ctx)
    return PMError(msg.decode() if msg else "unknown error")


def _take_host_csr(off_p, col_p, n):
    lib = _lib()
    off = np.ctypeslib.as_array(ctypes.cast(off_p, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy()
    nnz = int(off[-1])
    col = (np.ctypeslib.as_array(ctypes.cast(col_p, ctypes.POINTER(ctypes.c_uint32)), shape=(max(nnz, 1),))[:nnz].copy())
    lib.pm_free_host(off_p)
    lib.pm_free_host(col_p)
    return off, col


def rmat_graph(scale, p_gen=1, nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD, device=None):
    """Symmetrized R-MAT graph of generate_rmat.cpp with P_gen generator ranks.

    device=None: host generator (one thread per generator rank); device=k: the GPU
    generator on device k (MT19937 jump-ahead substreams, same graph bit for bit)."""
    lib = _lib()
    off_p, col_p, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    if device is None:
        rc = lib.pm_rmat_csr(scale, p_gen, ctypes.byref(off_p), ctypes.byref(col_p), ctypes.byref(n))
    else:
        rc = lib.pm_rmat_csr_gpu(scale, p_gen, device, ctypes.byref(off_p), ctypes.byref(col_p), ctypes.byref(n))
    if rc != 0:
        raise _err()
    off, col = _take_host_csr(off_p, col_p, n.value)
    return Graph(off, col, True, nranks, hub_threshold)


def _file_array(files):
    files = [os.fspath(f).encode() for f in files]
    arr = (ctypes.c_char_p * max(len(files), 1))(*files)
    return arr, len(files)


def ingest_edge_list_gpu(files, undirected=False, device=0, nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD):
    """ingest_edge_list's text parse and graph construction on the GPU (pm_ingest.hip):
    "src dst [weight]" lines, undirected=True adds (dst, src).  Returns a host Graph."""
    lib = _lib()
    arr, nf = _file_array(files)
    off_p, col_p, n, sym = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
    if lib.pm_ingest_edge_list_gpu(arr, nf, int(bool(undirected)), device, ctypes.byref(off_p), ctypes.byref(col_p),
                                   ctypes.byref(n), ctypes.byref(sym)) != 0:
        raise _err()
    off, col = _take_host_csr(off_p, col_p, n.value)
    return Graph(off, col, bool(sym.value), nranks, hub_threshold)


def mt19937_jump_outputs(seed, skip, count):
    """Outputs skip .. skip+count-1 of std::mt19937(seed) by one GF(2) jump (host check)."""
    out = np.zeros(max(count, 1), np.uint32)
    if _lib().pm_mt19937_jump_outputs(seed, skip, out.ctypes.data, count) != 0:
        raise _err()
    return out[:count]


def rmat_edges(scale, p_gen, first=0, stride=1):
    """Directed pairs (u,v),(v,u) of generator ranks first, first+stride, ... < p_gen
    (generate_rmat.cpp:202-213): the share of one process of a sharded run."""
    lib = _lib()
    src_p, dst_p, m = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    if lib.pm_rmat_edges(scale, p_gen, first, stride, ctypes.byref(src_p), ctypes.byref(dst_p), ctypes.byref(m)) != 0:
        raise _err()
    k = max(m.value, 1)
    out = []
    for p in (src_p, dst_p):  # one array at a time: peak host memory = output + one stream copy
        out.append(np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(k,))[: m.value].copy())
        lib.pm_free_host(p)
    return out[0], out[1]


def partition_edges(src, dst, n, group=None, device="cpu", hub_threshold=DEFAULT_HUB_THRESHOLD):
    """Owner partitioning of a distributed edge list, the host form of what pm_create_rmat_shard does
    on the GPUs (delegate_partitioned_graph.ipp:818-969, 1402-1648): every process holds some directed
    edges; the global out-degrees are summed over the processes, then every edge (u, v) goes in one
    all-to-all to the owner of u (u % world), or, when u is a delegate (global degree >=
    hub_threshold, more than one process), to the owner of v.

    Returns (off[n+1] u64 by id -- rows held elsewhere empty, col u32 sorted within each row,
    degree[n] u32 global degrees).  Collective over `group` (gloo on CPU, nccl = RCCL on GPU)."""
    import torch
    import torch.distributed as dist
    G = dist.get_world_size(group)
    # u32 ids travel as int32 and widen on the device
    s = torch.from_numpy(np.ascontiguousarray(src, dtype=np.uint32).view(np.int32)).to(device).long() & 0xFFFFFFFF
    d = torch.from_numpy(np.ascontiguousarray(dst, dtype=np.uint32).view(np.int32)).to(device).long() & 0xFFFFFFFF
    # global out-degrees (scatter-add of this process's sources, summed over the processes)
    gdeg = torch.zeros(n, dtype=torch.int32, device=device).index_add_(
        0, s, torch.ones(s.shape[0], dtype=torch.int32, device=device))
    dist.all_reduce(gdeg, group=group)
    if G == 1:  # nothing to exchange
        rs, rd = s, d
    else:
        owner = torch.where(gdeg[s] >= hub_threshold, d, s) % G
        order = torch.argsort(owner, stable=True)
        s, d, owner = s[order], d[order], owner[order]
        send = torch.zeros(G, dtype=torch.int64, device=device).index_add_(0, owner, torch.ones_like(owner))
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=group)
        sc, rc = send.tolist(), recv.tolist()
        rs = torch.empty(sum(rc), dtype=torch.int64, device=device)
        rd = torch.empty(sum(rc), dtype=torch.int64, device=device)
        dist.all_to_all_single(rs, s, rc, sc, group=group)
        dist.all_to_all_single(rd, d, rc, sc, group=group)
        del owner, order
    del s, d
    key = torch.sort(rs * n + rd).values
    rs, rd = key // n, key % n
    del key
    deg = torch.zeros(n, dtype=torch.int32, device=device).index_add_(
        0, rs, torch.ones(rs.shape[0], dtype=torch.int32, device=device))
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(deg.cpu().numpy().astype(np.uint64))
    return off, rd.to(torch.int32).cpu().numpy().view(np.uint32).copy(), gdeg.cpu().numpy().view(np.uint32).copy()


def comm_unique_id():
    """RCCL communicator id (bytes) for pm_create_shard; created on one rank, sent to all."""
    buf = ctypes.create_string_buffer(256)
    k = _lib().pm_comm_unique_id(buf, len(buf))
    if k < 0:
        raise _err()
    return buf.raw[:k]


def run_beta_local_shards(graph, pattern_dir, nshards, result_dir="", max_iterations=0, device=0, labels=None):
    """The sharded search with `nshards` shards driven by threads of this process on one
    device (in-process exchange instead of RCCL): parity of the sharded path on one GPU."""
    desc = _abi.GraphDesc(graph.n, graph.off.ctypes.data, graph.col.ctypes.data, int(graph.symmetric), graph.nranks,
                          graph.hub_threshold)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.uint64)
    if result_dir:
        os.makedirs(result_dir, exist_ok=True)
    st = _abi.RunStats()
    rc = _lib().pm_run_beta_local_shards(ctypes.byref(desc), pattern_dir.encode(), device, nshards,
                                         None if lab is None else lab.ctypes.data, result_dir.encode(),
                                         max_iterations, ctypes.byref(st))
    if rc != 0:
        raise _err()
    return st.as_dict()


def run_beta_local_shards_each(graph, pattern_dir, nshards, result_dir="", max_iterations=0, device=0, labels=None,
                               label_prefix=None, repeats=1):
    """run_beta_local_shards with -v label files (label_prefix, parsed on the device once) or labels, the search
    repeated `repeats` times (result files from the first) and every shard's statistics (pm_run_beta_local_shards2:
    the drop-in executable's mode for a P-partition graph on fewer GPUs than P)."""
    desc = _abi.GraphDesc(graph.n, graph.off.ctypes.data, graph.col.ctypes.data, int(graph.symmetric), graph.nranks,
                          graph.hub_threshold)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.uint64)
    if result_dir:
        os.makedirs(result_dir, exist_ok=True)
    st = (_abi.RunStats * nshards)()
    rc = _lib().pm_run_beta_local_shards2(ctypes.byref(desc), pattern_dir.encode(), device, nshards,
                                          None if lab is None else lab.ctypes.data,
                                          None if label_prefix is None else os.fspath(label_prefix).encode(),
                                          result_dir.encode(), max_iterations, repeats, st)
    if rc != 0:
        raise _err()
    return [s.as_dict() for s in st]


def graph_partitions(base):
    """P of the graph files <base>_<r>_of_<P>."""
    p = _lib().pm_graph_partitions(os.fspath(base).encode())
    if p < 0:
        raise _err()
    return p


def read_graph_shard(base, nshards, shard):
    """Shard `shard` of `nshards` read from the graph files (pm_read_graph_shard): (off[n+1] by id -- the owned
    rows whole, a delegate's entries whose target this shard owns, other rows empty --, col, degree[n] global,
    info dict with symmetric / nranks / hub_threshold)."""
    lib = _lib()
    off_p, col_p, deg_p, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    sym, nr, hub = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint64()
    if lib.pm_read_graph_shard(os.fspath(base).encode(), nshards, shard, ctypes.byref(off_p), ctypes.byref(col_p),
                               ctypes.byref(deg_p), ctypes.byref(n), ctypes.byref(sym), ctypes.byref(nr),
                               ctypes.byref(hub)) != 0:
        raise _err()
    nv = n.value
    deg = np.ctypeslib.as_array(ctypes.cast(deg_p, ctypes.POINTER(ctypes.c_uint32)), shape=(max(nv, 1),))[:nv].copy()
    lib.pm_free_host(deg_p)
    off, col = _take_host_csr(off_p, col_p, nv)
    return off, col, deg, {"symmetric": bool(sym.value), "nranks": nr.value, "hub_threshold": hub.value, "n": nv}


def device_count():
    """HIP devices visible to this process (0 without a GPU)."""
    return int(_lib().pm_device_count())


def run_rmat_local_shards(scale, p_gen, pattern_dir, nshards, result_dir="", max_iterations=0, device=0, nranks=1,
                          hub_threshold=DEFAULT_HUB_THRESHOLD):
    """The sharded search over the R-MAT graph with `nshards` shards driven by threads of this process
    on one device: each shard generates its generator ranks' streams on the device and the entries
    reach their owners in one in-process all-to-all (pm_run_rmat_local_shards)."""
    if result_dir:
        os.makedirs(result_dir, exist_ok=True)
    st = _abi.RunStats()
    rc = _lib().pm_run_rmat_local_shards(scale, p_gen, pattern_dir.encode(), device, nshards, nranks, hub_threshold,
                                         result_dir.encode(), max_iterations, ctypes.byref(st))
    if rc != 0:
        raise _err()
    return st.as_dict()


def run_rmat_local_shards_each(scale, p_gen, pattern_dir, nshards, result_dir="", max_iterations=0, device=0,
                               nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD, labels=None, repeats=1):
    """run_rmat_local_shards with labels (None: degree labels), the search repeated `repeats` times (result
    files from the first run) and every shard's statistics of the last run: a list of nshards dicts (the
    shard_* fields give the partition balance and each shard's device time of the sharded part)."""
    if result_dir:
        os.makedirs(result_dir, exist_ok=True)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.uint64)
    st = (_abi.RunStats * nshards)()
    rc = _lib().pm_run_rmat_local_shards2(scale, p_gen, pattern_dir.encode(), device, nshards, nranks, hub_threshold,
                                          None if lab is None else lab.ctypes.data, result_dir.encode(),
                                          max_iterations, repeats, st)
    if rc != 0:
        raise _err()
    return [s.as_dict() for s in st]


def pattern_summary(pattern_dir):
    """Parsed pattern directory (graph.hpp / pattern_util.hpp rules) as a dict."""
    import json
    buf = ctypes.create_string_buffer(1 << 20)
    if _lib().pm_pattern_summary(pattern_dir.encode(), buf, len(buf)) != 0:
        raise _err()
    return json.loads(buf.value.decode())


def write_graph(base, g, nranks=None):
    nr = g.nranks if nranks is None else nranks
    rc = _lib().pm_write_graph(base.encode(), g.n, g.off.ctypes.data, g.col.ctypes.data, int(g.symmetric), nr,
                               g.hub_threshold)
    if rc != 0:
        raise _err()


def read_graph(base):
    lib = _lib()
    off_p, col_p, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    sym, nr, hub = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint64()
    if lib.pm_read_graph(base.encode(), ctypes.byref(off_p), ctypes.byref(col_p), ctypes.byref(n), ctypes.byref(sym),
                         ctypes.byref(nr), ctypes.byref(hub)) != 0:
        raise _err()
    off, col = _take_host_csr(off_p, col_p, n.value)
    return Graph(off, col, bool(sym.value), nr.value, hub.value)


class PatternMatcher:
    """One device context: graph resident in HBM + one pattern directory."""

    def __init__(self, graph, pattern_dir, device=0, labels=None):
        self.graph = graph
        self._desc = _abi.GraphDesc(graph.n, graph.off.ctypes.data, graph.col.ctypes.data, int(graph.symmetric),
                                    graph.nranks, graph.hub_threshold)
        self._ctx = _lib().pm_create(ctypes.byref(self._desc), pattern_dir.encode(), device)
        if not self._ctx:
            raise _err()
        if labels is not None:
            self.set_labels(labels)

    def close(self):
        if getattr(self, "_ctx", None):
            _lib().pm_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise _err(self._ctx)

    def set_labels(self, labels):
        lab = np.ascontiguousarray(labels, dtype=np.uint64)
        if lab.shape[0] != self.graph.n:
            raise ValueError("labels must have one entry per vertex id")
        self._check(_lib().pm_vertex_data_set(self._ctx, lab.ctypes.data))

    def labels_from_files(self, prefix):
        """-v <prefix>: label files parsed on the device (pm_vertex_data_files)."""
        self._check(_lib().pm_vertex_data_files(self._ctx, os.fspath(prefix).encode()))

    def degree_labels(self):
        self._check(_lib().pm_vertex_data_degree(self._ctx))

    def reset(self):
        self._check(_lib().pm_reset(self._ctx))

    def lcc_bsp(self, init_step, itr=0):
        st = _abi.LccStats()
        self._check(_lib().pm_lcc_bsp(self._ctx, int(init_step), itr, ctypes.byref(st)))
        return {f[0]: getattr(st, f[0]) for f in st._fields_ if f[0] != "reserved"}

    def token_passing(self, pl):
        st = _abi.TpStats()
        self._check(_lib().pm_token_passing(self._ctx, pl, ctypes.byref(st)))
        return {f[0]: getattr(st, f[0]) for f in st._fields_}

    def tds(self, pl, sink=None):
        """One TDS line through pm_tds: sink(rank, vertex_ids) is called for every kept walk
        (the lines the reference writes to subgraphs_<pl>_<rank>); returns the line stats."""
        st = _abi.TpStats()
        cb = _abi.PathSink(lambda user, rank, v, n: sink(rank, [v[i] for i in range(n)])) if sink else None
        self._check(_lib().pm_tds(self._ctx, pl, ctypes.cast(cb, ctypes.c_void_p) if cb else None, None,
                                  ctypes.byref(st)))
        return {f[0]: getattr(st, f[0]) for f in st._fields_}

    def post_token_passing(self, pl):
        d = ctypes.c_uint32()
        self._check(_lib().pm_post_token_passing(self._ctx, pl, ctypes.byref(d)))
        return bool(d.value)

    def run_beta(self, result_dir="", max_iterations=0):
        st = _abi.RunStats()
        if result_dir:
            os.makedirs(result_dir, exist_ok=True)
        self._check(_lib().pm_run_beta(self._ctx, result_dir.encode(), max_iterations, ctypes.byref(st)))
        return st.as_dict()

    def run_beta_into(self, st, max_iterations=0):
        """One search without result files into a caller-owned _abi.RunStats (no dict built: the bench's timed
        loop converts after the clock stops)."""
        self._check(_lib().pm_run_beta(self._ctx, b"", max_iterations, ctypes.byref(st)))
        return st

    def comm_info(self):
        """This context's place in its search: {"nshards", "shard", "comm_ranks" (the communicator's own count,
        RCCL: ncclCommCount), "transport"} (pm_comm_info)."""
        ns, sh = ctypes.c_uint32(), ctypes.c_uint32()
        cr, tr = ctypes.c_int32(), ctypes.c_int32()
        self._check(_lib().pm_comm_info(self._ctx, ctypes.byref(ns), ctypes.byref(sh), ctypes.byref(cr),
                                        ctypes.byref(tr)))
        return {"nshards": ns.value, "shard": sh.value, "comm_ranks": cr.value,
                "transport": _abi.TRANSPORTS.get(tr.value, str(tr.value))}

    def tpub_census(self, deferred_reset=False):
        """(nonzero T_pub entries of buffer 0, of buffer 1, positions nonzero in either buffer outside the
        current slist) -- diagnostics of the invariant the search-start clear relies on
        (pm_debug_tpub_census); deferred_reset=True first runs a search start's reset."""
        out = np.zeros(3, np.uint64)
        self._check(_lib().pm_debug_tpub_census(self._ctx, int(bool(deferred_reset)), out.ctypes.data))
        return tuple(int(x) for x in out)

    def export_state(self):
        """Returns (tpub[n] u16, mdeg[n] u32, nbrs u32) of the current state map."""
        n = self.graph.n
        tpub = np.zeros(n, np.uint16)
        mdeg = np.zeros(n, np.uint32)
        ne = ctypes.c_uint64()
        self._check(_lib().pm_export_state(self._ctx, tpub.ctypes.data, mdeg.ctypes.data, None, ctypes.byref(ne)))
        nbrs = np.zeros(max(ne.value, 1), np.uint32)
        self._check(_lib().pm_export_state(self._ctx, None, None, nbrs.ctypes.data, ctypes.byref(ne)))
        return tpub, mdeg, nbrs[: ne.value]


class _DeviceGraph:
    """Size of a graph that lives only in HBM (pm_create_rmat)."""

    def __init__(self, n, nnz, nranks, hub_threshold):
        self.n, self._nnz, self.nranks, self.hub_threshold = int(n), int(nnz), nranks, hub_threshold
        self.symmetric = True

    @property
    def nnz(self):
        return self._nnz


def rmat_matcher(scale, p_gen, pattern_dir, device=0, nranks=1, hub_threshold=DEFAULT_HUB_THRESHOLD):
    """PatternMatcher over an R-MAT graph generated on the device (the adjacency never
    visits the host).  Returns (matcher, generation seconds)."""
    secs = ctypes.c_double()
    ctx = _lib().pm_create_rmat(scale, p_gen, pattern_dir.encode(), device, nranks, hub_threshold,
                                ctypes.byref(secs))
    if not ctx:
        raise _err()
    m = PatternMatcher.__new__(PatternMatcher)
    m._ctx = ctx
    m.graph = _DeviceGraph(1 << scale, (1 << scale) * 32, nranks, hub_threshold)
    return m, secs.value


def rmat_shard_matcher(scale, p_gen, pattern_dir, nshards, shard, unique_id, device=0, nranks=1,
                       hub_threshold=DEFAULT_HUB_THRESHOLD):
    """One rank of a sharded search over the R-MAT graph (one process per GPU, collective): the rank
    generates its generator ranks' streams on its GPU and the entries reach their owners in one RCCL
    all-to-all (pm_create_rmat_shard).  Returns (matcher, seconds of generation + exchange + rows)."""
    secs = ctypes.c_double()
    uid = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
    ctx = _lib().pm_create_rmat_shard(scale, p_gen, os.fspath(pattern_dir).encode(), device, nranks, hub_threshold,
                                      nshards, shard, uid, ctypes.byref(secs))
    if not ctx:
        raise _err()
    m = PatternMatcher.__new__(PatternMatcher)
    m._ctx = ctx
    m.graph = _DeviceGraph(1 << scale, (1 << scale) * 32, nranks, hub_threshold)
    return m, secs.value


def edge_list_matcher(files, pattern_dir, undirected=False, device=0, nranks=1,
                      hub_threshold=DEFAULT_HUB_THRESHOLD):
    """PatternMatcher over text edge-list files ingested on the device (the adjacency never
    visits the host).  Returns (matcher, ingest seconds)."""
    arr, nf = _file_array(files)
    secs = ctypes.c_double()
    ctx = _lib().pm_create_edge_list(arr, nf, int(bool(undirected)), os.fspath(pattern_dir).encode(), device, nranks,
                                     hub_threshold, ctypes.byref(secs))
    if not ctx:
        raise _err()
    n, nnz, sym = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    _lib().pm_graph_size(ctx, ctypes.byref(n), ctypes.byref(nnz), ctypes.byref(sym))
    m = PatternMatcher.__new__(PatternMatcher)
    m._ctx = ctx
    m.graph = _DeviceGraph(n.value, nnz.value, nranks, hub_threshold)
    m.graph.symmetric = bool(sym.value)
    return m, secs.value


class TorchHostComm:
    """pm_host_comm (include/pm_abi.h) over a torch.distributed process group: the sharded search's
    collectives staged through host memory and carried by the group's backend (gloo on CPU tensors) --
    the exchange a maintainer binds to MPI_Allgather / MPI_Allreduce / MPI_Alltoallv in the reference's
    own MPI world.  The processes may share one device."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self._torch, self._dist, self._group = torch, dist, group
        self.nshards = dist.get_world_size(group)
        self.shard = dist.get_rank(group)
        self.error = None
        # the ctypes callbacks must outlive the context that calls them
        self._cbs = (_abi.HostAllgather(self._guard(self._allgather)),
                     _abi.HostAllreduce64(self._guard(self._allreduce64)),
                     _abi.HostAllreduce32(self._guard(self._allreduce32)),
                     _abi.HostAlltoallv(self._guard(self._alltoallv)))
        self.struct = _abi.HostComm(None, self.nshards, self.shard, *self._cbs)

    def _guard(self, fn):
        def call(*a):
            try:
                fn(*a)
                return 0
            except Exception as ex:  # noqa: BLE001 (reported through the C-ABI's status)
                self.error = ex
                return 1
        return call

    def _u8(self, addr, nbytes):
        return self._torch.frombuffer((ctypes.c_char * nbytes).from_address(addr), dtype=self._torch.uint8)

    def _allgather(self, user, send, recv, nbytes):
        if not nbytes:
            return
        out = self._u8(recv, nbytes * self.nshards)
        self._dist.all_gather(list(out.split(nbytes)), self._u8(send, nbytes), group=self._group)

    def _allreduce64(self, user, buf, count):
        if count:
            t = self._torch.frombuffer((ctypes.c_int64 * count).from_address(buf), dtype=self._torch.int64)
            self._dist.all_reduce(t, group=self._group)  # (two's complement: the u64 sum wraps alike)

    def _allreduce32(self, user, buf, count):
        if count:
            t = self._torch.frombuffer((ctypes.c_int32 * count).from_address(buf), dtype=self._torch.int32)
            w = t.to(self._torch.int64) & 0xFFFFFFFF
            self._dist.all_reduce(w, group=self._group)
            t.copy_(((w & 0xFFFFFFFF) - ((w & 0x80000000) << 1)).to(self._torch.int32))

    def _alltoallv(self, user, send, sbytes, recv, rbytes):
        G = self.nshards
        sb = [int(x) for x in (ctypes.c_uint64 * G).from_address(sbytes)]
        rb = [int(x) for x in (ctypes.c_uint64 * G).from_address(rbytes)]
        empty = self._torch.empty(0, dtype=self._torch.uint8)
        inp = self._u8(send, sum(sb)) if sum(sb) else empty
        out = self._u8(recv, sum(rb)) if sum(rb) else empty
        self._dist.all_to_all_single(out, inp, rb, sb, group=self._group)


class ShardedPatternMatcher(PatternMatcher):
    """One rank of a sharded search (one process per GPU; RCCL between the shards).

    off/col/degree come from partition_edges(); unique_id from comm_unique_id() on one rank,
    distributed to all.  Construction, run_beta, set_labels and export_state are collective.
    host_comm=TorchHostComm(group) (instead of unique_id) carries the exchanges through the host over a
    torch.distributed group (pm_create_shard_host_comm): processes that share a device, or a host transport."""

    def __init__(self, n, off, col, degree, pattern_dir, nshards, shard, unique_id=None, device=0, nranks=1,
                 hub_threshold=DEFAULT_HUB_THRESHOLD, symmetric=True, host_comm=None):
        self._off = np.ascontiguousarray(off, dtype=np.uint64)
        self._col = np.ascontiguousarray(col if len(col) else np.zeros(1, np.uint32), dtype=np.uint32)
        self._deg = np.ascontiguousarray(degree, dtype=np.uint32)
        self.graph = Graph(self._off, self._col[: int(self._off[-1])], symmetric, nranks, hub_threshold)
        self.graph.n = int(n)
        self._sdesc = _abi.ShardDesc(n, self._off.ctypes.data, self._col.ctypes.data, self._deg.ctypes.data,
                                     int(symmetric), nranks, hub_threshold, nshards, shard)
        self._host_comm = host_comm
        if host_comm is not None:
            self._ctx = _lib().pm_create_shard_host_comm(ctypes.byref(self._sdesc), pattern_dir.encode(), device,
                                                         ctypes.byref(host_comm.struct))
        else:
            uid = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
            self._ctx = _lib().pm_create_shard(ctypes.byref(self._sdesc), pattern_dir.encode(), device, uid)
        if not self._ctx:
            raise _err()
