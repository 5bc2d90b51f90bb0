# kernel-trace stats of the default bench + per-family stage-1 timings (GPU box)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01b}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u profiles/family_times.py 5000 250 > $OUT/family_times.log 2>&1 || { echo FAM_FAILED; tail -20 $OUT/family_times.log; exit 1; }
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 3 --warmup 1 > $OUT/trace_bench.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/trace_bench.log; exit 1; }
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -type f | xargs ls -la
cat $OUT/family_times.log | tail -3
