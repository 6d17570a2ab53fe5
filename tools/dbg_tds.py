"""Repeats one parity case on the GPU (unsharded and sharded) and prints the walk counts."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import fuzzypatternmatching_amd as pm  # noqa: E402
import oracle  # noqa: E402
import pmtest  # noqa: E402

pat = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern")
g = pm.rmat_graph(10, 1)
g.nranks = 2
labels = pmtest.hash_labels(g.n, 8)
td = tempfile.mkdtemp()
so = oracle.run(g.off, g.col, pat, os.path.join(td, "o"), labels=labels, nranks=2, max_iterations=100)
print("oracle", {k: so[k] for k in ("iterations", "final_vertices", "final_edges", "tds_edges", "paths")}, flush=True)
for rep in range(3):
    m = pm.PatternMatcher(g, pat, labels=labels)
    s = m.run_beta(os.path.join(td, f"u{rep}"), 100)
    m.close()
    d = pmtest.compare_result_dirs(os.path.join(td, "o"), os.path.join(td, f"u{rep}"), 2)
    print("plain", rep, {k: s[k] for k in ("iterations", "final_vertices", "final_edges", "tds_edges", "walks")}, d[:2],
          flush=True)
for G in (1, 1, 2, 3):
    s = pm.run_beta_local_shards(g, pat, G, os.path.join(td, f"s{G}"), 100, labels=labels)
    d = pmtest.compare_result_dirs(os.path.join(td, "o"), os.path.join(td, f"s{G}"), 2)
    print("shards", G, {k: s[k] for k in ("iterations", "final_vertices", "final_edges", "tds_edges", "walks")}, d[:3],
          flush=True)


def lines(d):
    out = set()
    sd = os.path.join(d, "0", "all_ranks_subgraphs")
    for f in os.listdir(sd):
        if f.startswith("subgraphs_4_"):
            out |= set(l.strip() for l in open(os.path.join(sd, f)) if l.strip())
    return out


a, b = lines(os.path.join(td, "o")), lines(os.path.join(td, "s1"))
print("union sizes", len(a), len(b), "only oracle", sorted(a - b)[:4], "only gpu", sorted(b - a)[:4], flush=True)
