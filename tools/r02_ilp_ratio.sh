# Lone-wave ILP probe (one vs two messages per lane) and same-box step ratio
# records / cfg2 (no profiler), alternating.
set -o pipefail
mkdir -p gpurun_out/ilp
hipcc --offload-arch=gfx950 -O3 -I nakevaleng_amd/csrc tools/lone_wave.hip -o /tmp/lone_wave.bin || exit 1
NKV_LONE_ILP=1 timeout -k 10 120 /tmp/lone_wave.bin > gpurun_out/ilp/lone_ilp.txt 2>&1 || exit 1
cat gpurun_out/ilp/lone_ilp.txt
for i in 1 2; do
  for cfg in "" "--config records" "--config mixed"; do
    timeout -k 10 200 python bench.py $cfg --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
  done
done
