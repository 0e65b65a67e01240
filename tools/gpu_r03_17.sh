#!/bin/bash
# tiled cosine prepare, one wave per 16-row tile: parity (incl. the bench-shape test) + frames bench + prepare times
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_fullsize.py -q -x -k "cosine or frames" --timeout 200 --timeout-method thread > gpurun_out/r03_t17a.log 2>&1
rc=$?; echo "cos tests rc=$rc"; tail -3 gpurun_out/r03_t17a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r03_17 -o run --output-format csv -- python3 bench.py --no-search --no-stream --no-precomputed --no-ingest --no-cpu --steps 2 > gpurun_out/r03_b17.json 2>/dev/null
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/prof_r03_17/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
d = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in rows if "k_cos_prepare" in r["Kernel_Name"]]
print("k_cos_prepare_tiled us per call", d)
fr = json.load(open("gpurun_out/r03_b17.json"))["frames"]
print("frames", round(fr["value"] / 1e9, 2), round(fr["roofline"]["frac"], 3), round(fr["ms_per_step"], 3))
PY
