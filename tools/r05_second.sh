#!/bin/bash
# Round 5, second GPU call: the per-call floor of a small flush (launch /
# copy / completion-wait costs beside the one-launch path), the small-tree
# kernel's duration per shape under rocprofv3, then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/${OUT:-r05b}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 ./build/launch_floor 2000 > "$OUT/launch_floor.json" 2> "$OUT/launch_floor.err"
rc=$?; cat "$OUT/launch_floor.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/launch_floor.err"; exit $rc; }
SHAPES="10:1:200:6e616b67 40:1:200:6e616b67 256:1:200:6e616b67 1024:1:200:6e616b67 1024:1024:1024:6e616b67"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_small" \
    -o small -- "$GRAFT_REPO_ROOT/build/small_flush" 1 300 /tmp $SHAPES ) > "$OUT/prof_small.log" 2>&1
rc=$?; tail -3 "$OUT/prof_small.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider tests/ \
    > "$OUT/gpu_suite.log" 2>&1
rc=$?; tail -5 "$OUT/gpu_suite.log"; [ $rc -eq 0 ] || exit $rc
echo done
