# stage-3 rank: parity tests, then all 58 rows at c4 with k_xs_rank_day (default) and the
# 1,024-thread k_xs_rank_bucket (MFF_XS_RANK_IMPL=bucket), alternating, plus a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4rank
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "stage3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for impl in day bucket; do
    echo -n "$impl$rep "
    MFF_XS_RANK_IMPL=$impl timeout -k 10 200 python3 profiles/stage3_probe.py --all-only 2>&1 | grep "all rows" || exit 1
  done
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/profiles/stage3_probe.py --all-only > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -12
