# 128-byte register runs (LOAD 4) as the default aligned load path: GPU suite,
# same-box A/B against the LDS-DMA stage (--leaf-load 1), and the new cfg2
# leaf kernel's PMC traffic (one --pmc pass per TCC group)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/runs
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/runs/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/runs/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/runs/gpu_tests.txt
for i in 1 2 3; do
  for l in 0 1; do
    timeout -k 10 120 python bench.py --leaf-load $l --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[load $l]', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['kernel'], d.get('verified_vs_oracle'))" || exit 1
  done
done
bash tools/pmc_config.sh cfg2_runs || exit 1
python3 tools/pmc_traffic_cfg.py cfg2_runs "void nkv::k_leaf<0, 4>" 4294967296 1048576 || exit 1
# records: the segment stage (product) vs 128-byte register runs at each value's own address (experiment library)
for i in 1 2 3; do
  for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_rruns.so; do
    NKV_LIB=$lib timeout -k 10 120 python bench.py --config records --no-cpu-baseline --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[records $lib]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
  done
done
