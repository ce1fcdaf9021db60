# the line-path parity test, the whole GPU suite, and the driver's default bench forms
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_lines.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_lines.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_lines.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_form.json 2>/dev/null || exit 1
tail -c 700 gpurun_out/bench_driver_form.json
