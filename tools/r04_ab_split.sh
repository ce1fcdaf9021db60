# Round 4: the tree's chain levels split over two waves (helper wave computes
# W + K into LDS, the chain wave runs only the rounds) -- parity of the product
# build on every tree test, then the default line round-robin against the
# -DNKV_NO_SPLIT build (nakevaleng_amd/libnkv_nosplit.so) on one box, then
# rocprof kernel stats of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/split
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_round2.py tests/test_gpu_round3.py tests/test_gpu_fuzz.py tests/test_gpu_multi.py tests/test_gpu_sharded.py tests/test_gpu_api.py > gpurun_out/split/tests.log 2>&1
rc=$?; tail -2 gpurun_out/split/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in default nosplit; do
    if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/nakevaleng_amd/libnkv_$lib.so; fi
    timeout -k 10 150 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))" || exit 1
  done
done
unset NKV_LIB
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split -o default -- python3 bench.py --steps 50 --warmup 10 --no-capi --no-cpu-baseline > /dev/null 2>&1 || exit 1
NKV_LIB=$PWD/nakevaleng_amd/libnkv_nosplit.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split -o nosplit -- python3 bench.py --steps 50 --warmup 10 --no-capi --no-cpu-baseline > /dev/null 2>&1 || exit 1
python - <<'PY'
import csv
for f in ("default", "nosplit"):
    for r in csv.DictReader(open(f"gpurun_out/split/{f}_kernel_stats.csv")):
        if "reduce" in r["Name"] or "k_leaf" in r["Name"]:
            print(f, r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1000, 2))
PY
