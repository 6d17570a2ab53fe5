"""Diagnostics: the state after supersteps 0..K-1 of the first LCC call (PM_DEBUG_LCC_STOP=K, dumped by shard 0
with PM_DEBUG_STATE_DUMP) for one context, and for in-process shards with the replica hand-off after the first
(PM_HANDOFF=1) and the second (=2) later superstep; prints the rows that differ."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "run":
    import fuzzypatternmatching_amd as pm
    mode, scale, p_gen, thr, shards = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
    g = pm.rmat_graph(scale, p_gen)
    pat = os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern")
    if mode == "single":
        m = pm.PatternMatcher(pm.Graph(g.off, g.col, True, 1, thr), pat)
        m.run_beta("", 1)
        m.close()
    else:
        pm.run_beta_local_shards(pm.Graph(g.off, g.col, True, 1, thr), pat, shards, "", max_iterations=1)
    sys.exit(0)

scale, p_gen, thr, shards, stop = (sys.argv[1:] + ["16", "4", "64", "4", "3"][len(sys.argv) - 1:])[:5]
base = os.path.join(ROOT, "gpurun_out", "handoff_state")
os.makedirs(base, exist_ok=True)
dumps = {}
for mode, h in (("single", "2"), ("h1", "1"), ("h2", "2"), ("h2_nosort", "2")):
    f = os.path.join(base, f"{mode}_stop{stop}.txt")
    env = dict(os.environ, PM_HANDOFF=h, PM_DEBUG_LCC_STOP=stop, PM_DEBUG_STATE_DUMP=f)
    if mode.endswith("nosort"):
        env["PM_DEBUG_NO_HUB_SORT"] = "1"
    r = subprocess.run([sys.executable, __file__, "run", mode.split("_")[0], scale, p_gen, thr, shards], env=env,
                       capture_output=True, text=True, timeout=300)
    print(f"{mode}: rc {r.returncode} {r.stderr.strip()[-500:]}", flush=True)
    dumps[mode] = dict(l.split(" ", 1) for l in open(f).read().splitlines()) if os.path.exists(f) else {}
ref = dumps["single"]
for mode in ("h1", "h2", "h2_nosort"):
    d = dumps[mode]
    only_ref = sorted(set(ref) - set(d), key=int)
    only_d = sorted(set(d) - set(ref), key=int)
    diff = [v for v in ref if v in d and ref[v] != d[v]]
    print(f"{mode}: {len(d)} rows vs {len(ref)}; missing {len(only_ref)} {only_ref[:10]}, extra {len(only_d)} "
          f"{only_d[:10]}, differing {len(diff)}")
    for v in diff[:8]:
        print(f"   {v}: single [{ref[v][:300]}]\n   {' ' * len(v)}  {mode:6s} [{d[v][:300]}]")
