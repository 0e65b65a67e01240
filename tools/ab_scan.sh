#!/bin/bash
# A/B of k_scan0f build variants (tools/ubench/lib_*.so) with tools/scan_expt.py
for f in tools/ubench/lib_*.so; do
  HQ_LIB_VARIANT=$PWD/$f SCAN_EXPT_ONLY=default timeout -k 10 120 python tools/scan_expt.py 2>&1 | grep default | sed "s|^|$(basename $f) |"
done
