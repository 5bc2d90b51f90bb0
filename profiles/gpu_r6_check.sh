# round-6 check of the working tree: every -m gpu test (or TESTS="..."), smoke(), the
# default bench line.  usage: bash profiles/gpu_r6_check.sh TAG [nobench]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06}
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
[ "$2" = "nobench" ] && exit 0
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','ms_per_step')})); print(json.dumps(d['roofline']['kernels'])); print(json.dumps(d['extras']))"
