#!/bin/bash
# Round 5: the NewLeaf arena in host-coherent pinned memory (NKV_OPT_ARENA_COHERENT
# 1, the new default: the small path reads it in place) against default pinned
# memory, for the 1 Mi x 4 KiB flush with Session::Reserve (the recommended
# form) and without (the arena grows by doubling in the first flush), twice
# each, alternating, on one box; then the rocprofv3 summary of the default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/${OUT:-r05d}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=$(mktemp -d /tmp/nkvab.XXXX)
for rep in 1 2; do
  for coh in 1 0; do
    for res in 1 0; do
      NKV_ARENA_COHERENT=$coh timeout -k 10 120 ./build/api_flush 1048576 4096 5 "$D" 1 0x6e616b65 1 -1 1 $res \
          > "$OUT/arena_c${coh}_r${res}_${rep}.jsonl" 2> "$OUT/arena_c${coh}_r${res}_${rep}.err"
      rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/arena_c${coh}_r${res}_${rep}.err"; exit $rc; }
      echo "coherent=$coh reserve=$res rep=$rep: $(python3 -c "
import json,sys
c=[json.loads(l) for l in open('$OUT/arena_c${coh}_r${res}_${rep}.jsonl')]
print(' '.join('%.1f/%.1f' % (x['gib_s'], x['upload_ms']) for x in c))")"
      rm -f "$D"/*
    done
  done
done
rmdir "$D"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_default" \
    -o default -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-capi --no-subconfigs --no-cpu-baseline ) \
    > "$OUT/prof_default.log" 2>&1
rc=$?; grep '^{' "$OUT/prof_default.log" | tail -c 600; [ $rc -eq 0 ] || { tail -5 "$OUT/prof_default.log"; exit $rc; }
echo done
