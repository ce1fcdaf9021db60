# tree reduce plans: k_reduce2 while a level holds >= 64 Ki (product) / 256 Ki / 512 Ki nodes, then 1024-node slabs
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tree_build or full_size or bfs or strided" > gpurun_out/gpu_tests_reduce.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_reduce.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_reduce.txt
for i in 1 2; do
for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_r256k.so tools/libnkvmerkle_r512k.so; do
  NKV_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$lib]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
