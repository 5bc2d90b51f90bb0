# round 5: a subset of the -m gpu tests (TESTS="file ..."), or all of them
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_tests
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|error|assert" $OUT/gpu_tests.log | head -40; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
