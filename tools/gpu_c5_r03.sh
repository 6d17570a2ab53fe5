#!/bin/bash
# GPU box: the ingest tests (double-buffered staging), then config C5 at size (tools/c5_at_size.py): a small
# rehearsal, then SCALE (27) with the oracle at full size; JSON lines under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SCALE=${SCALE:-27}
df -h /dev/shm /tmp 2>&1 | tail -2
free -g | head -2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_configs.py::test_c5_ingested_edge_list_with_label_files \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ingest.log 2>&1 \
  || { tail -30 gpurun_out/pytest_ingest.log; exit 1; }
tail -1 gpurun_out/pytest_ingest.log
timeout -k 10 300 python3 -u tools/c5_at_size.py --scale 20 --oracle --out gpurun_out/c5_s20.json \
  2> gpurun_out/c5_s20.log || { tail -20 gpurun_out/c5_s20.log; exit 1; }
tail -3 gpurun_out/c5_s20.log
timeout -k 10 900 python3 -u tools/c5_at_size.py --scale $SCALE ${ORACLE---oracle} --out gpurun_out/c5_s$SCALE.json \
  2> gpurun_out/c5_s$SCALE.log
rc=$?; tail -12 gpurun_out/c5_s$SCALE.log; exit $rc
