#!/bin/bash
# A/B: sample-pass wave count (sample_waves) after the epilogue fix; k_scanov at 3 waves per SIMD with a deeper
# prefetch (ov_occ 3 + ov_pf 2 / 3)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
bash tools/ab_bench_search.sh r06_13_ab "default|" "sample_waves=4096|--option sample_waves=4096" "sample_waves=1024|--option sample_waves=1024" "ov_occ=3 ov_pf=2|--option ov_occ=3 --option ov_pf=2" "ov_occ=3 ov_pf=3|--option ov_occ=3 --option ov_pf=3" || exit 1
