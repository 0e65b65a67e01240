#!/bin/bash
# rocprofv3 kernel stats of the search leg alone (cfg3: 1M corpus x 1000 queries), 20 timed steps.
# usage: tools/search_only_prof.sh <tag>
set -u
TAG=${1:-s}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sprof_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 > $OUT/sprof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 - "$OUT/sprof_$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:14]:
    print(x["Name"][:60].ljust(60), x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us", round(float(x["TotalDurationNs"]) / 1e3), "us total")
PY
grep -o '"search": {"metric"[^}]*' $OUT/sprof_$TAG.log | head -c 330; echo
