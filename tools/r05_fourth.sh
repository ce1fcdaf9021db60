#!/bin/bash
# Round 5, fourth GPU call: the arena coherence A/B and the default line's
# rocprof summary (tools/r05_arena_ab.sh), then the over-fetch PMC passes
# (tools/r05_pmc_overfetch.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/r05d bash tools/r05_arena_ab.sh || exit $?
OUT=gpurun_out/r05e bash tools/r05_pmc_overfetch.sh || exit $?
echo all done
