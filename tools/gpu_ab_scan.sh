#!/bin/bash
# A/B of level-0 scan options on the search leg: tools/gpu_ab_scan.sh "opt1=v1,opt2=v2" "..." ...
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  opts=""
  for o in ${spec//,/ }; do [ "$o" != "default" ] && opts="$opts --option $o"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --n-emb 10000 --no-cpu --no-stream --no-precomputed --no-ingest --no-frames --search-steps 20 $opts > gpurun_out/ab_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -3 gpurun_out/ab_$i.log; exit $rc; }
  echo "[$spec] $(python3 tools/prof_summary.py gpurun_out/ab_$i | grep -E 'k_scan0g|k_sample_topf' | tr -s ' ' | cut -c1-90 | tr '\n' ';') $(grep -o '"search": {"metric[^}]*' gpurun_out/ab_$i.log | grep -o '"value": [0-9.]*')"
done
