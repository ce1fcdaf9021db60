set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_crc.py > gpurun_out/vt.txt 2>&1 || { tail -30 gpurun_out/vt.txt; exit 1; }
tail -1 gpurun_out/vt.txt
for i in 1 2; do
for lib in nakevaleng_amd/libnkvmerkle.so tools/libnkvmerkle_oldcrc.so; do
  for cl in -1 0 1 8; do
    echo -n "$lib crc_load=$cl: "; NKV_LIB=$lib timeout -k 10 120 python tools/bench_crc.py --crc-load $cl --verify 2>&1 | tail -1 || exit 1
  done
  NKV_LIB=$lib timeout -k 10 120 python bench.py --config records_verify --no-cpu-baseline --steps 100 --verify 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$lib records_verify]', d['value'], d['kernel_ms'], d.get('verified_vs_oracle'))" || exit 1
done
done
