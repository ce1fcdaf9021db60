# k_leaf_records with whole 128-byte lines into registers (default) vs the
# LDS-DMA segment stage (experiment library, NKV_RECORDS_LINES=0): GPU suite,
# then same-box records / mixed A/B, verified against the oracle
set -o pipefail
mkdir -p gpurun_out/lines
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/lines/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/lines/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/lines/gpu_tests.txt
bash tools/ab_tags.sh "--config records" stage || exit 1
bash tools/ab_tags.sh "--config records --key-bytes 20" stage || exit 1
bash tools/ab_tags.sh "--config mixed" stage || exit 1
