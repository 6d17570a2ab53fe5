"""Per-line / per-position device times of the fused NLC line kernel on a generated R-MAT graph with hash labels
(the C5 shape at any scale): sets PM_PHASE_TIMES=1 (pm_lines.hip, run_lines_fused) and runs one search; the
line times go to stderr, the search's stats to stdout as one JSON line.

usage: python3 tools/nlcc_phase_times.py [--scale 27] [--p-gen 8] [--alphabet 256] [--pattern rmat_log2_cycle4_pattern]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("PM_PHASE_TIMES", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fuzzypatternmatching_amd as pm  # noqa: E402
import pmtest  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=27)
    ap.add_argument("--p-gen", type=int, default=8)
    ap.add_argument("--alphabet", type=int, default=256)
    ap.add_argument("--pattern", default="rmat_log2_cycle4_pattern")
    ap.add_argument("--repeat", type=int, default=1)
    args = ap.parse_args()
    m, _ = pm.rmat_matcher(args.scale, args.p_gen, os.path.join(ROOT, "patterns", args.pattern), device=0)
    m.set_labels(pmtest.hash_labels(1 << args.scale, args.alphabet, salt=5))
    for _ in range(args.repeat):
        print(json.dumps(m.run_beta("", 64)), flush=True)


if __name__ == "__main__":
    main()
