# Round 4 check: GPU suite, the default bench line (the driver's form), the
# compaction read (records_verify, priced at the 737.9-VALU count), the default
# bench under rocprofv3 (kernel stats CSV), the host-inclusive flush.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04_bench.json'));print(d['value'],d['kernel_ms'],d['sclk_mhz'],d['verified_vs_oracle'],d['capi_group'].get('value'),d['capi_one_tree'].get('verified_vs_oracle'))"
timeout -k 10 300 python bench.py --config records_verify --no-capi > gpurun_out/r04_records_verify.json 2> gpurun_out/r04_records_verify.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04_records_verify.json'));print(d['value'],d['kernel_ms'],d['roofline']['valu_ceiling_basis'],d['roofline']['valu_frac'],d['verified_vs_oracle'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04 -o cfg2 -- python3 bench.py --steps 20 --warmup 5 --no-capi --no-cpu-baseline > gpurun_out/r04_bench_rocprof.json 2> gpurun_out/r04_rocprof.err || exit 1
timeout -k 10 600 python bench.py --config api_flush --api-cycles 4 > gpurun_out/r04_api_flush.json 2> gpurun_out/r04_api_flush.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04_api_flush.json'));print('api_flush',d['value'],d['vs_cpu_all_cores'],d['verified_vs_oracle'],d['breakdown_ms'])"
