set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 3 --warmup 1 > $R/gpurun_out/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof.log; exit 1; }
find $R/gpurun_out/prof -name "*kernel_trace.csv" -delete; find $R/gpurun_out/prof -name "*stats*"
