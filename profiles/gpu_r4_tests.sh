# round-4 GPU test run: the given test files first (fail fast), then optionally the rest.
# usage: bash profiles/gpu_r4_tests.sh TAG "tests/test_a.py tests/test_b.py" [all]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04}
FIRST=${2:-tests/test_gpu_nulls.py}
OUT=$R/gpurun_out/tests_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/first.log 2>&1 || { echo FIRST_FAILED; tail -60 $OUT/first.log; exit 1; }
tail -3 $OUT/first.log
if [ "$3" = "all" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/all.log 2>&1 || { echo ALL_FAILED; tail -60 $OUT/all.log; exit 1; }
  tail -3 $OUT/all.log
fi
