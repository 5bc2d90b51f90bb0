set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ing
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ingest.py tests/test_gpu_dropin.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ing/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ing/tests.log; exit 1; }
tail -3 gpurun_out/ing/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ing/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/ing/bench.log; exit 1; }
tail -2 gpurun_out/ing/bench.log
