# the default bench line (c4, extras, CPU baseline) as the driver runs it
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/bench_${1:-r03}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','ms_per_step')})); print(json.dumps(d['roofline']['kernels'])); print(json.dumps(d['extras'])); print(json.dumps(d['cpu_baseline']))"
