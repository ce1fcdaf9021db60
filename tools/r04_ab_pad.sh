# Round 4: the uniform padding block (schedule and W + K on the scalar unit,
# k_leaf<0, 4> when every value's length is a multiple of 64) and the pair form
# of the parent compression (padding words as constants in waves without a
# lone node).  GPU suite on the new library, then a same-box A/B against the
# previous sources (tools/libnkvmerkle_base.so, built from HEAD) on cfg2 and
# the tree-only config, every root verified; then SQ_INSTS_VALU per wave of
# both under rocprofv3 --pmc (its own passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_pad_tests.log; [ $rc -eq 0 ] || exit $rc
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
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/pmc_pad_$lib -o pmc -- python3 bench.py --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing --no-clock --no-capi > /dev/null 2> gpurun_out/pmc_pad_$lib.err || exit 1
done
unset NKV_LIB
echo done
