# GPU suite + smoke, PMC traffic for records and mixed, then the three bench configs verified
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/pmc_config.sh records --config records || exit 1
bash tools/pmc_config.sh mixed --config mixed || exit 1
for cfg in "" "--config records" "--config mixed"; do
  timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline']['step_frac'], d.get('verified_vs_oracle'))" || exit 1
done
