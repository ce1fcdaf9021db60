#!/bin/bash
# Round 6, twelfth GPU call: the all-lanes small kernels (tools/r06_eleventh.sh)
# and the all-lanes tree levels (tools/r06_ab_reduce_lanes.sh), then the GPU
# tests of the tree reduce.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06o}
mkdir -p $O
OUT=$(basename $O) bash tools/r06_eleventh.sh && \
timeout -k 10 600 bash tools/r06_ab_reduce_lanes.sh > $O/ab_reduce.txt 2>&1 && cat $O/ab_reduce.txt && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_round2.py tests/test_gpu_round3.py -x -q --timeout 120 \
    --timeout-method thread > $O/tests_reduce.txt 2>&1 && tail -1 $O/tests_reduce.txt && echo twelfth done
