# HBM traffic of one bench config's leaf kernel: one --pmc pass per TCC counter
# group (FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2), kernel trace only.
#   bash tools/pmc_config.sh <tag> [bench args...]   -> gpurun_out/pmc_<tag>/
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
d=gpurun_out/pmc_$tag
mkdir -p $d
run() {
  local name=$1 ctr=$2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $d -o "$name" -- \
    python3 bench.py $BARGS --steps 3 --warmup 1 --preroll-s 0 --no-cpu-baseline --no-kernel-timing > "$d/$name.json" 2>&1
}
BARGS="$*"
run req "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM" &&
run fetch "FETCH_SIZE" &&
run write "WRITE_SIZE" &&
run sizes "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"
