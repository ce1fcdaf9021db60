# last evidence lines with the final bench.py: default line (verified, CPU baseline),
# the RCCL world-1 line, and the one_tree config (plain and under the process group)
set -o pipefail
mkdir -p gpurun_out/last
timeout -k 10 300 python bench.py --verify > gpurun_out/last/bench_default.json 2>/dev/null || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --dist --steps 50 --warmup 10 --no-cpu-baseline --verify > gpurun_out/last/bench_rccl_world1.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config one_tree --no-cpu-baseline --verify > gpurun_out/last/one_tree.json 2>/dev/null || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --dist --config one_tree --steps 20 --warmup 5 --no-cpu-baseline --verify > gpurun_out/last/one_tree_dist.json 2>/dev/null || exit 1
for f in bench_default bench_rccl_world1 one_tree one_tree_dist; do
  python -c "import json; d=json.loads([l for l in open('gpurun_out/last/$f.json').read().splitlines() if l.startswith('{')][-1]); print('[$f]', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('verified_vs_oracle'), d.get('root_gather_ok'))" || exit 1
done
