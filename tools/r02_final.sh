# Round-2 evidence on one box: GPU suite + smoke, default bench line (with CPU
# baseline), rocprofv3 kernel summaries of cfg2 / records / mixed / cfg5 per-GPU table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/final/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/final/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/final/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py --verify > gpurun_out/final/bench_default.json 2>/dev/null || exit 1
tail -c 400 gpurun_out/final/bench_default.json
# the N > 1 code path on the one GPU: torch.distributed.run, nccl (RCCL) group, per-step root all-gather
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --dist --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/final/bench_rccl_world1.json 2> gpurun_out/final/bench_rccl_world1.err || exit 1
tail -c 300 gpurun_out/final/bench_rccl_world1.json
for v in "cfg2:" "records:--config records" "mixed:--config mixed" "records_verify:--config records_verify" "cfg5_per_gpu:--leaves 8388608"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final -o r02_$tag -- python3 bench.py $args --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/final/r02_$tag.json || exit 1
done
python3 - <<'PY'
import csv
for t in ["cfg2", "records", "mixed", "records_verify", "cfg5_per_gpu"]:
    rows = list(csv.DictReader(open(f"gpurun_out/final/r02_{t}_kernel_stats.csv")))
    print(t, "; ".join("%s %.1f us" % (r["Name"].split("(")[0][-28:], float(r["AverageNs"]) / 1e3) for r in rows[:4]))
PY
