# Round 4: the tree levels of at most 64 parents in subtree_reduce run on wave 0
# alone, ordered by LDS waits instead of workgroup barriers (the other waves
# leave).  GPU suite on the new library, then a same-box A/B against the
# previous sources (tools/libnkvmerkle_base.so), cfg2 x4, every root verified,
# and rocprofv3 kernel stats of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_onewave_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_onewave_tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # lib, bench args
  local lib=$1; shift
  if [ "$lib" = new ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', '$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))"
}
for rep in 1 2 3 4; do
  one base || exit 1; one new || exit 1
done
export TMPDIR=/tmp
for lib in base new; do
  if [ "$lib" = new ]; then unset NKV_LIB; else export NKV_LIB=$PWD/tools/libnkvmerkle_$lib.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_onewave_$lib -o cfg2 -- python3 bench.py --steps 50 --warmup 5 --no-capi --no-cpu-baseline > /dev/null 2> gpurun_out/prof_onewave_$lib.err || exit 1
done
unset NKV_LIB
echo done
