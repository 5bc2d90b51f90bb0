# per-launch durations of the sorted-group kernel variants (profiles/group_split.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/gsplit_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp MFF_PDF_OVERLAP=0 MFF_HL_STREAM=0; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o trace --output-format csv -- python3 $R/profiles/group_split.py 5000 500 > $OUT/run.log 2>&1 || { echo SPLIT_FAILED; tail -20 $OUT/run.log; exit 1; }
find $OUT -name "*kernel_trace.csv" -delete
grep 'pass ms' $OUT/run.log
python3 - <<PY
import csv, glob
for f in glob.glob("$OUT/tr/**/*kernel_stats.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        if "mff" in x["Name"]:
            print(f"{x['Name'][:70]:72s} {x['Calls']:>4s} {float(x['AverageNs'])/1e6:9.3f} ms")
PY
