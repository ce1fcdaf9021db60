# round-2 baseline on one box: GPU suite, smoke, three bench configs verified,
# then rocprofv3 kernel-trace summaries of cfg2 and the records form.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/prof
prof() {  # name, command...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o "$name" -- "$@" > "gpurun_out/prof/$name.json"
}
prof r02_cfg2 python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline &&
prof r02_records python3 bench.py --config records --steps 30 --warmup 10 --no-cpu-baseline
