# rocprofv3 kernel-trace summaries for the round-1 commands (copied into profiles/ afterwards
# by tools/collect_profiles.py).  Each step has its own time limit; the chain stops at a failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
prof() {  # name, command...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o "$name" -- "$@" > "gpurun_out/prof/$name.json"
}
prof cfg2 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline &&
prof cfg3 python3 bench.py --config mixed --steps 30 --warmup 10 --no-cpu-baseline &&
prof records python3 bench.py --config records --steps 30 --warmup 10 --no-cpu-baseline &&
prof crc python3 tools/bench_crc.py --steps 30 --warmup 10 &&
prof bloom python3 tools/bench_bloom.py --steps 30 --warmup 10
