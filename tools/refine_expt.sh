for e in 0 1 2; do
HQ_REFINE_EXPT=$e bash tools/search_only_prof.sh x$e > /dev/null 2>&1
python3 - gpurun_out/sprof_x$e <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in csv.DictReader(open(f)):
    if 'refine' in x['Name']: print(sys.argv[1], x["Name"][:40], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us")
PY
done
