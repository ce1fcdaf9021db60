# GPU suite, then the launch-count change (queue set up by the sort, pass flags
# instead of the fold launch in the records entries) against the previous
# library (tools/libnkvmerkle_base.so), same box
set -o pipefail
mkdir -p gpurun_out/abl
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/abl/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/abl/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/abl/gpu_tests.txt
for cfg in "--config records" "--config records_verify" "--config mixed" ""; do
  bash tools/ab_tags.sh "$cfg" base || exit 1
done
