#!/bin/bash
# Search-path check: GPU search tests + rocprofv3 kernel stats of a short bench run (small quantize batch).
# usage: tools/search_prof.sh <tag>
set -u
TAG=${1:-s}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/test_gpu_search.py -q -rf -x > $OUT/t_search_$TAG.log 2>&1; rc=$?
tail -3 $OUT/t_search_$TAG.log
[ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --n-emb 100000 > $OUT/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - "$OUT/prof_$TAG" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:10]:
    print(x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us")
PY
grep -o '"search": {"metric"[^}]*' $OUT/prof_$TAG.log | head -c 330; echo
exit 0
