# Root gather at world size 1 on the one GPU (the N > 1 code path): one
# collective per timed loop (batch, default) vs one per table (step) vs no
# process group, same box, two rounds
set -o pipefail
mkdir -p gpurun_out/abg
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bench_launch.py || exit 1
port=29541
for i in 1 2; do
  for g in batch step none; do
    port=$((port+1))
    if [ $g = none ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/abg/$g$i.json 2>/dev/null || exit 1
    else
      timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --dist --gather $g --no-cpu-baseline > gpurun_out/abg/$g$i.json 2>/dev/null || exit 1
    fi
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/abg/$g$i.json').read().splitlines() if l.startswith('{')][-1]); print('[$g]', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('root_gather_ok'), d['config']['parallelism'])" || exit 1
  done
done
