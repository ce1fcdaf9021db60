# Round 4, VERDICT r03 item 6: the tree's top folded into k_reduce_wide's last
# workgroup.  Parity of the product build (coherent-store ticket) on the tree
# tests, then the same bench line round-robin over three builds on one box:
# default (coherent stores + ticket), fence (__threadfence + ticket, -DNKV_FOLD_FENCE),
# nofold (be08ef9: k_reduce_wide + k_reduce<256>, two launches); then rocprof
# kernel stats of the default and nofold builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_round2.py tests/test_gpu_round3.py tests/test_gpu_fuzz.py > gpurun_out/r04_fold_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_fold_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in default fence nofold; do
    if [ "$lib" = default ]; then unset NKV_LIB; else export NKV_LIB=$PWD/nakevaleng_amd/libnkv_$lib.so; fi
    timeout -k 10 150 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))" || exit 1
  done
done
unset NKV_LIB
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fold -o default -- python3 bench.py --steps 50 --warmup 10 --no-capi --no-cpu-baseline > /dev/null 2>&1 || exit 1
NKV_LIB=$PWD/nakevaleng_amd/libnkv_nofold.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fold -o nofold -- python3 bench.py --steps 50 --warmup 10 --no-capi --no-cpu-baseline > /dev/null 2>&1 || exit 1
grep -h "reduce" gpurun_out/prof_fold/*_kernel_stats.csv | cut -d, -f1-4
# the C++ mirror (copy pool, recycled node storage, threaded materialization) and the flush
timeout -k 10 300 python -u -m pytest tests/test_cpp_api.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r04_cpp.log 2>&1
rc=$?; tail -2 gpurun_out/r04_cpp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config api_flush --api-cycles 4 > gpurun_out/r04_api_flush.json 2> gpurun_out/r04_api_flush.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_api_flush.json"))
print("api_flush", d["value"], "x all-core", d.get("vs_cpu_all_cores"), "verified", d["verified_vs_oracle"])
for m, r in d["cycles"].items():
    for c in r:
        print(m, c["cycle"], c["gib_s"], c["newleaf_ms"], c["new_call_ms"], c["materialize_ms"], c["walk_ms"], c["write_ms"], c["total_ms"])
PY
