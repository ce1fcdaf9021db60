#!/bin/bash
# Round 5, third GPU call: the small path after input staging in LDS and the
# host-visible completion word (parity first), its floor and per-shape kernel
# time, then the 1 Mi x 4 KiB flush with the arena host-coherent (the new
# default) and in default pinned memory (NKV_ARENA_COHERENT=0), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/${OUT:-r05c}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NKV_DEBUG=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_small.py tests/test_abi_c.py tests/test_cpp_api.py tests/test_gpu_api.py > "$OUT/small_tests.log" 2>&1
rc=$?; tail -3 "$OUT/small_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./build/launch_floor 2000 > "$OUT/launch_floor.json" 2> "$OUT/launch_floor.err"
rc=$?; cat "$OUT/launch_floor.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/launch_floor.err"; exit $rc; }
timeout -k 10 300 python -u bench.py --config small_flush > "$OUT/small_flush.json" 2> "$OUT/small_flush.err"
rc=$?; tail -c 600 "$OUT/small_flush.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/small_flush.err"; exit $rc; }
SHAPES="10:1:200:6e616b67 40:1:200:6e616b67 256:1:200:6e616b67 1024:1:200:6e616b67 1024:1024:1024:6e616b67"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_small" \
    -o small -- "$GRAFT_REPO_ROOT/build/small_flush" 1 300 /tmp $SHAPES ) > "$OUT/prof_small.log" 2>&1
rc=$?; tail -1 "$OUT/prof_small.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config api_flush > "$OUT/api_flush.json" 2> "$OUT/api_flush.err"
rc=$?; tail -c 1500 "$OUT/api_flush.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/api_flush.err"; exit $rc; }
NKV_ARENA_COHERENT=0 timeout -k 10 400 python -u bench.py --config api_flush --no-cpu-baseline \
    > "$OUT/api_flush_noncoherent.json" 2> "$OUT/api_flush_noncoherent.err"
rc=$?; tail -c 600 "$OUT/api_flush_noncoherent.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/api_flush_noncoherent.err"; exit $rc; }
echo done
