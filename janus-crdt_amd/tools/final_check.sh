#!/bin/bash
# Round-end check on one GPU box, in one lease: the whole -m gpu suite, smoke(), then the profile pipeline
# (kernel traces, PMC passes, their summary) and the default bench line (tools/gpu_profile.sh, WITH_BENCH=1).
# Each GPU step has its own time limit; the first failure ends the script.
# Usage: bash janus-crdt_amd/tools/final_check.sh <gpurun_out dir> <round>
set -o pipefail
OUT=${1:-gpurun_out/final}
R=${2:-r04}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "GPU TESTS FAILED"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
echo "[$(date +%T)] smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$OUT/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[$(date +%T)] profile + bench"
WITH_BENCH=1 bash janus-crdt_amd/tools/gpu_profile.sh "$OUT/prof" "$R" > "$OUT/profile.log" 2>&1 || { echo "PROFILE FAILED"; tail -20 "$OUT/profile.log"; exit 1; }
tail -3 "$OUT/profile.log"
echo "[$(date +%T)] done"
