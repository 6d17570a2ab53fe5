"""Diagnostics: one sharded search (graph input, delegates) with PM_HANDOFF=1 and =2 in separate processes;
prints where their result directories differ (count files in full, vertex / edge set differences)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if len(sys.argv) > 1 and sys.argv[1] == "run":
    import fuzzypatternmatching_amd as pm
    scale, p_gen, thr, nranks, shards, out = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]),
                                              int(sys.argv[6]), sys.argv[7])
    g = pm.rmat_graph(scale, p_gen)
    st = pm.run_beta_local_shards(pm.Graph(g.off, g.col, True, nranks, thr),
                                  os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"), shards, out,
                                  max_iterations=100)
    print(st)
    sys.exit(0)

args = sys.argv[1:] or ["16", "4", "64", "4", "4"]
base = os.path.join(ROOT, "gpurun_out", "handoff_diff")
dirs = {}
for h in ("1", "2"):
    d = os.path.join(base, "h" + h)
    os.makedirs(d, exist_ok=True)
    env = dict(os.environ, PM_HANDOFF=h)
    r = subprocess.run([sys.executable, __file__, "run", *args, d], env=env, capture_output=True, text=True,
                       timeout=300)
    print(f"handoff {h}: rc {r.returncode} {r.stdout.strip()[-400:]} {r.stderr.strip()[-600:]}", flush=True)
    dirs[h] = d
for sub in ("all_ranks_active_vertices_count", "all_ranks_active_edges_count"):
    for fn in sorted(os.listdir(os.path.join(dirs["1"], "0", sub))):
        a = open(os.path.join(dirs["1"], "0", sub, fn)).read().split("\n")
        b = open(os.path.join(dirs["2"], "0", sub, fn)).read().split("\n")
        if a != b:
            print(f"{sub}/{fn}:\n  h1 {a}\n  h2 {b}")
for sub in ("all_ranks_active_vertices", "all_ranks_active_edges"):
    for fn in sorted(os.listdir(os.path.join(dirs["1"], "0", sub))):
        a = set(open(os.path.join(dirs["1"], "0", sub, fn)).read().split("\n"))
        b = set(open(os.path.join(dirs["2"], "0", sub, fn)).read().split("\n"))
        if a != b:
            print(f"{sub}/{fn}: only h1 {sorted(a - b)[:8]} ({len(a - b)}), only h2 {sorted(b - a)[:8]} ({len(b - a)})")
