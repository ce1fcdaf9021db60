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
prof records_verify python3 bench.py --config records_verify --steps 30 --warmup 10 --no-cpu-baseline &&
prof crc python3 tools/bench_crc.py --steps 30 --warmup 10 &&
prof bloom python3 tools/bench_bloom.py --steps 30 --warmup 10

# HBM traffic of the cfg2 leaf kernel: one --pmc pass per counter group (TCC
# limits: 4 counters; FETCH_SIZE takes 3, WRITE_SIZE 2), kernel trace only
pmc() {  # name, counters
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc -o "$name" -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > "gpurun_out/pmc/$name.json"
}
mkdir -p gpurun_out/pmc
pmc req TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCC_BUBBLE TCC_EA0_RDREQ_32B &&
pmc fetch FETCH_SIZE &&
pmc write WRITE_SIZE &&
pmc sizes TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B
