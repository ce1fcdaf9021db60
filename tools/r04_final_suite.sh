# Round 4 close: the GPU suite and smoke() on the round's last tree (what the
# driver runs at round end), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_close_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_close_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r04_close_bench.json 2> gpurun_out/r04_close_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04_close_bench.json'));print(d['value'],d['kernel_ms'],d['sclk_mhz'],d['roofline']['valu_frac'],d['verified_vs_oracle'],d['capi_group'].get('value'),d['capi_one_tree'].get('verified_vs_oracle'))"
