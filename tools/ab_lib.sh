#!/bin/bash
# A/B a bench leg between the in-tree library and variant builds (HQ_LIB_VARIANT), one box.
# usage: tools/ab_lib.sh "<bench args>" <variant.so>...   ("-" = the in-tree library)
ARGS=$1; shift
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = "-" ]; then r=$(timeout -k 10 300 python bench.py $ARGS 2>/dev/null); else r=$(HQ_LIB_VARIANT=$v timeout -k 10 300 python bench.py $ARGS 2>/dev/null); fi || { echo "fail $v"; exit 1; }
  echo "$v: $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(d[k]['value']), round(d[k]['roofline']['frac'],3)) for k in ('stream','search','precomputed','frames') if k in d}, round(d['value']))")"
done
done
