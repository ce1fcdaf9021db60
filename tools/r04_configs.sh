# Round 4: every bench config, each verified against the committed oracle roots
# (tests/golden/bench_roots.json), on one box; the default line (with the
# configs[4] group child) first.
# OUT (default r04_configs): the directory under gpurun_out/ the lines go to.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-r04_configs}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_cpp_api.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$OUT/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/$OUT/$name.json 2> gpurun_out/$OUT/$name.err || { tail -5 gpurun_out/$OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/$OUT/$name.json')); print('$name', d['value'], d.get('kernel_ms'), d.get('sclk_mhz'), 'verified', d.get('verified_vs_oracle'), {k: (v.get('value'), v.get('verified_vs_oracle'), v.get('error')) for k, v in d.items() if k.startswith('capi_')})"
}
run default --steps 20 --warmup 5 || exit 1
run records --config records --no-capi --no-cpu-baseline || exit 1
run records_verify --config records_verify --no-capi --no-cpu-baseline || exit 1
run mixed --config mixed --no-capi --no-cpu-baseline || exit 1
run runs4 --config runs4 --no-cpu-baseline || exit 1
