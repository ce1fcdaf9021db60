set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_staging.py > gpurun_out/t.txt 2>&1 || { tail -30 gpurun_out/t.txt; exit 1; }
tail -1 gpurun_out/t.txt
bash tools/ab_libs.sh "--config records" default old
bash tools/ab_libs.sh "--config mixed" default old
bash tools/ab_libs.sh "--config records_verify" default old
