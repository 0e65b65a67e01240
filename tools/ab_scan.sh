#!/bin/bash
# A/B of level-0 scan build variants (tools/ubench/lib_*.so) with tools/scan_expt.py; lib_nb2* run with HQ_SCAN_NB=2
for f in tools/ubench/lib_*.so; do
  nb=4; case $f in *nb2*) nb=2;; esac
  HQ_SCAN_NB=$nb HQ_LIB_VARIANT=$PWD/$f SCAN_EXPT_ONLY=default timeout -k 10 120 python tools/scan_expt.py 2>&1 | grep default | sed "s|^|$(basename $f) |"
done
