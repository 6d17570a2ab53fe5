#!/bin/bash
# GPU box: C5's search with small alphabets (tools/c5_alphabet_growth.py): 8 letters scale by scale until the
# growth predicts a search past the budget, then 64 letters at S=27 (the config's scale), each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 280 python3 -u tools/c5_alphabet_growth.py --alphabets 8 --scales 12 13 14 15 16 17 18 19 20 21 22 \
  --budget 40 --search-limit 200 --oracle-edges 2e8 > gpurun_out/c5_growth_a8.jsonl 2> gpurun_out/c5_growth_a8.err
echo "alphabet 8 rc=$?"
cut -c1-220 gpurun_out/c5_growth_a8.jsonl
timeout -k 10 880 python3 -u tools/c5_alphabet_growth.py --alphabets 64 --scales 27 --budget 1000 --search-limit 840 \
  > gpurun_out/c5_growth_a64_s27.jsonl 2> gpurun_out/c5_growth_a64_s27.err
rc=$?
echo "alphabet 64 S=27 rc=$rc"
grep -v "c5 growth\]" gpurun_out/c5_growth_a64_s27.err | tail -3
cut -c1-400 gpurun_out/c5_growth_a64_s27.jsonl
exit 0
