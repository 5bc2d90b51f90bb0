# GPU test run (pytest -m gpu) of the given test files (default: all)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/t
cd $R
timeout -k 10 400 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t/tests.log; exit 1; }
tail -3 gpurun_out/t/tests.log
