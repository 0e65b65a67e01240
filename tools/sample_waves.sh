for w in 256 512 1024 2048 4096; do
  HQ_SAMPLE_WAVES=$w SCAN_EXPT_ONLY=default timeout -k 10 120 python tools/scan_expt.py 2>&1 | grep default | sed "s/^/waves=$w /"
done
