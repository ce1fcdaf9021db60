set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sort
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py > gpurun_out/sort/tests.txt 2>&1 || { tail -30 gpurun_out/sort/tests.txt; exit 1; }
tail -1 gpurun_out/sort/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sort -o mixed -- python3 bench.py --config mixed --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/sort/mixed.json || exit 1
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/sort/mixed_kernel_stats.csv")))[:12]:
    print("%-40s %.1f us" % (r["Name"].split("(")[0][-40:], float(r["AverageNs"]) / 1e3))
PY
