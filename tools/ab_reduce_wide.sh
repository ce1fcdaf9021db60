set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tree_build or full_size or bfs or strided or tree_from_values" > gpurun_out/gpu_tests_reduce.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_reduce.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_reduce.txt
bash tools/ab_lib.sh nowide "" "--config records" "--leaves 8388608"
