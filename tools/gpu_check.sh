# full GPU test suite, smoke(), and the three bench configs (verified) on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for cfg in "" "--config records" "--config mixed"; do
  timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['kernel_ms'], d['roofline']['achieved'], d.get('verified_vs_oracle'))" || exit 1
done
