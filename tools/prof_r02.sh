# rocprofv3 kernel stats of the round-2 library: cfg2, records, mixed
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof6
for v in "cfg2:" "records:--config records" "mixed:--config mixed"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o r02_$tag -- python3 bench.py $args --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/prof6/r02_$tag.json || exit 1
done
python3 - <<'PY'
import csv
for t in ["cfg2", "records", "mixed"]:
    print(t)
    for r in list(csv.DictReader(open(f"gpurun_out/prof6/r02_{t}_kernel_stats.csv")))[:5]:
        print("  %-50s calls=%s avg_us=%.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"])/1e3))
PY
