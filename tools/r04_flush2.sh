# Round 4: the flush after Serialize(file) moved to a reused per-thread image
# buffer and nkv_write_file to parallel positioned writes: the C++ mirror's GPU
# test, then bench.py --config api_flush (4 cycles per mode, root verified).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_api.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r04_flush2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_flush2_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 600 python bench.py --config api_flush --api-cycles 4 > gpurun_out/r04_flush2_$rep.json 2> gpurun_out/r04_flush2_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r04_flush2_$rep.json'));print('api_flush',d['value'],d['vs_cpu_all_cores'],d['verified_vs_oracle'],d['breakdown_ms'])"
done
