# per-launch durations of the sorted-group kernel variants (profiles/group_split.py), one
# process per factor set so the kernel stats separate them
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/gsplit_${1:-a}
D=${2:-500}
mkdir -p $OUT
export TMPDIR=/tmp MFF_PDF_OVERLAP=0 MFF_HL_STREAM=0; cd /tmp
for set in ORD LVL LVLPDF ALL; do
  SPLIT_SET=$set timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$set -o trace --output-format csv -- python3 $R/profiles/group_split.py 5000 $D > $OUT/$set.log 2>&1 || { echo SPLIT_FAILED $set; tail -20 $OUT/$set.log; exit 1; }
  find $OUT/$set -name "*kernel_trace.csv" -delete
  grep 'pass ms' $OUT/$set.log
  SET=$set python3 - <<PY
import csv, glob, os
for f in glob.glob("$OUT/$set/**/*kernel_stats.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        if "mff" in x["Name"]:
            print(f"   {x['Name'][:66]:68s} {x['Calls']:>4s} {float(x['AverageNs'])/1e6:9.3f} ms")
PY
done
