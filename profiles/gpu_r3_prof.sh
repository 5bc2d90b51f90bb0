# Round-3 stage-1 profile (GPU box): headline bench line, overlapped pass kernel trace
# (per-pass timeline), and the launches one at a time (MFF_STAGE1_SERIAL=1:
# standalone per-kernel durations).  usage: bash profiles/gpu_r3_prof.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $OUT/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$OUT/bench.log') if l.startswith('{')][0]); print('value', round(d['value']/1e6,2), 'M/s  ms/step', round(d['ms_per_step'],2), 'pass ms', d['roofline']['avg_kernel_ms'], 'frac', d['roofline']['frac'])"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/overlap -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 4 --warmup 1 > $OUT/overlap.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/overlap.log; exit 1; }
python3 $R/profiles/pass_span.py $OUT/overlap $OUT/pass_spans.csv > $OUT/pass_timeline.log 2>&1 || true
export MFF_STAGE1_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 4 --warmup 1 > $OUT/serial.log 2>&1 || { echo PROF2_FAILED; tail -20 $OUT/serial.log; exit 1; }
find $OUT -name "*kernel_trace.csv" -delete
tail -8 $OUT/pass_timeline.log
python3 - <<PY
import csv, glob
for tag in ("overlap", "serial"):
    for f in glob.glob("$OUT/%s/**/*kernel_stats.csv" % tag, recursive=True):
        print("==", tag)
        for x in csv.DictReader(open(f)):
            if "mff" in x["Name"]:
                print(f"{x['Name'][:70]:72s} {x['Calls']:>4s} {float(x['AverageNs'])/1e6:9.3f} ms")
PY
