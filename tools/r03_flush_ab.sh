#!/bin/bash
# Round 3: flush path A/B on one box -- the C++ mirror with a std::vector per
# node's Data and a deque of nodes (build/api_flush_old, the previous header)
# against the inline-digest Data and the reserved node vector (build/api_flush).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O /tmp/af
for r in a b c; do
  for v in old new; do
    exe=build/api_flush; [ $v = old ] && exe=build/api_flush_old
    timeout -k 10 120 $exe 1048576 4096 4 /tmp/af 1 0x6e616b65 1 > $O/af_${v}_$r.jsonl 2> $O/af_${v}_$r.err || exit $?
    python -c "
import json
c=[json.loads(l) for l in open('$O/af_${v}_$r.jsonl') if l.startswith('{')][1:]
print('$v $r', ' | '.join('%.2f GiB/s newleaf %.0f new %.1f mat %.1f walk %.1f' % (x['gib_s'], x['newleaf_ms'], x['new_call_ms'], x['materialize_ms'], x['walk_ms']) for x in c))"
  done
done
