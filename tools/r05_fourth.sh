#!/bin/bash
# Round 5, fourth GPU call: the arena coherence A/B and the default line's
# rocprof summary (tools/r05_arena_ab.sh), then the over-fetch PMC passes
# (tools/r05_pmc_overfetch.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=r05d bash tools/r05_arena_ab.sh || exit $?
OUT=r05e bash tools/r05_pmc_overfetch.sh || exit $?
for shape in "10 1 200" "40 1 200" "256 1 200" "1024 1 200" "1024 1024 1024"; do
  timeout -k 10 120 python3 tools/small_diag.py $shape 200 50 >> gpurun_out/r05e/small_diag.jsonl 2>> gpurun_out/r05e/small_diag.err || exit $?
done
cat gpurun_out/r05e/small_diag.jsonl
echo all done
