#!/bin/bash
# Round 6 check on the committed tree: the whole GPU suite, smoke(), then the
# default line as the driver runs it (every sub-record) and its rocprofv3
# summary (the headline kernel's trace on this build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r06i}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1 \
    || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/default_line.json 2> $O/default_line.err \
    || { tail -5 $O/default_line.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('default', d['value'], d['sclk_mhz'], d['roofline']['frac'], d['roofline']['valu_frac'], d['verified_vs_oracle'], d['cpu_baseline']['value'])
for k in ('capi_group','capi_one_tree','capi_config4','config2_mixed','config1_records','config1_records_verify','api_flush'):
    v=d.get(k,{}); print(k, v.get('value'), v.get('verified_vs_oracle'), v.get('error'), (v.get('roofline') or {}).get('frac'), (v.get('cpu_baseline') or {}).get('value'), v.get('wall_s'))
" $O/default_line.json
tail -1 $O/default_line.err
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$O/prof" -o default -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 \
    --no-capi --no-subconfigs --no-cpu-baseline ) > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
grep -E "k_leaf<0, 4>|k_reduce" $O/prof/default_kernel_stats.csv | cut -c1-160
echo all done
