set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "line_pair or strided or records" > gpurun_out/lp_tests.txt 2>&1 || { tail -40 gpurun_out/lp_tests.txt; exit 1; }
tail -1 gpurun_out/lp_tests.txt
for i in 1 2; do
for ll in 0 9 10; do
  timeout -k 10 200 python bench.py --config records --leaf-load $ll --no-cpu-baseline --steps 50 --warmup 10 $( [ $i = 1 ] && echo --verify ) 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('records load=$ll', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
for ll in 0 9 10; do
  timeout -k 10 200 python bench.py --leaf-load $ll --no-cpu-baseline --steps 50 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('cfg2 load=$ll', d['value'], d['kernel_ms'])" || exit 1
done
