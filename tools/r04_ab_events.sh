# Round 4: the cost of the per-call timing events inside the timed loop (three
# hipEventRecord per tree call; the kernel trace shows ~4.8 us before the
# reduce and ~8 us before the next leaf kernel).  Same box, alternating x4:
# the default line (events + clock probe), --no-kernel-timing (clock probe
# only; the kernel split then comes from a second loop), neither, and the
# events on every 4th step (--timing-every 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_round3.py -m gpu -x -q -k "timing" --timeout 250 --timeout-method thread 2>&1 | tail -2 || exit 1
one() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-capi "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['kernel_ms'], d['sclk_mhz'], d.get('verified_vs_oracle'))"
}
for rep in 1 2 3 4; do
  one events || exit 1; one no_events --no-kernel-timing || exit 1; one none --no-kernel-timing --no-clock || exit 1
  one every4 --timing-every 4 || exit 1
done
