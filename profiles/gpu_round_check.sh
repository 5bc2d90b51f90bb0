# round-end style check of the working tree: every -m gpu test, smoke(), the default bench
# line (c4, extras, CPU baseline).  usage: bash profiles/gpu_round_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','ms_per_step')})); print(json.dumps(d['roofline']['kernels'])); print(json.dumps(d['extras'])); print(json.dumps(d['cpu_baseline']))"
