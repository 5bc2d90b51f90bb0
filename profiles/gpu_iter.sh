# iteration loop: GPU tests (optionally filtered by $PYTEST_K), then kernel stats of a
# short default bench.  usage (gpurun): bash profiles/gpu_iter.sh [tag]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-iter}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 3 --warmup 1 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $OUT/bench.log; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -delete
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value']/1e6,2), 'M/s  ms/step', round(d['ms_per_step'],2), 'pass ms', d['roofline']['avg_kernel_ms'])"
python3 - <<PY
import csv, glob
for f in glob.glob('$OUT/prof/**/*kernel_stats.csv', recursive=True):
    for x in csv.DictReader(open(f)):
        if 'mff' in x['Name']:
            print(f"{x['Name'][:64]:66s} {x['Calls']:>4s} {float(x['AverageNs'])/1e6:9.3f} ms")
PY
