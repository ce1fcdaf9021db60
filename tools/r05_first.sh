#!/bin/bash
# Round 5, first GPU call: the new one-launch small-tree path and the plain-C
# caller against the oracle, the small_flush bench, then the driver's default
# line (with the config2_mixed / config1_records sub-records and the
# four-variant CPU baseline).  Every GPU step has its own time limit; the first
# failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/${OUT:-r05a}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NKV_DEBUG=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_small.py tests/test_abi_c.py > "$OUT/small_tests.log" 2>&1
rc=$?; tail -4 "$OUT/small_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config small_flush > "$OUT/small_flush.json" 2> "$OUT/small_flush.err"
rc=$?; tail -c 1500 "$OUT/small_flush.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/small_flush.err"; exit $rc; }
timeout -k 10 560 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?; tail -c 3000 "$OUT/bench_default.json"; [ $rc -eq 0 ] || { tail -30 "$OUT/bench_default.err"; exit $rc; }
echo done
