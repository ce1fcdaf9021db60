# rocprofv3 kernel-trace summaries for the round-1 commands (copied into profiles/ afterwards)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o cfg2 -- python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof/cfg2.json &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o cfg3 -- python3 bench.py --config mixed --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof/cfg3.json &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o crc -- python3 tools/bench_crc.py --steps 30 --warmup 10 > gpurun_out/prof/crc.json
