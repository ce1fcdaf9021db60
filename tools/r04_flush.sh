# Round 4: the C++ mirror's GPU test, then the host-inclusive flush
# (bench.py --config api_flush: copy threads with a retained heap, the copies on
# the caller's thread, and glibc's default heap), CPU baseline in the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_api.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r04_cpp.log 2>&1
rc=$?; tail -2 gpurun_out/r04_cpp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config api_flush --api-cycles 4 > gpurun_out/r04_api_flush.json 2> gpurun_out/r04_api_flush.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_api_flush.json"))
print(d["value"], d["vs_cpu_all_cores"], d["verified_vs_oracle"], d["glibc_default_heap"]["gib_s"], d["copies_on_caller_thread"]["gib_s"])
for m, r in d["cycles"].items():
    for c in r:
        print(m, c["cycle"], c["gib_s"], c["newleaf_ms"], c["new_call_ms"], c["materialize_ms"], c["walk_ms"], c["write_ms"], c["total_ms"])
PY
