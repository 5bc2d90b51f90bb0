# per-pass timeline of the overlapped stage-1 pass (rocprofv3 kernel trace + pass_span.py)
# for each in-tree build mff/libmff_<v>.so (VARIANTS)
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
OUT=$R/gpurun_out/timeline
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS:-a b}; do
  MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$v -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 4 --warmup 1 > $OUT/$v.log 2>&1 || { echo "PROF $v FAILED"; tail -20 $OUT/$v.log; exit 1; }
  python3 $R/profiles/pass_span.py $OUT/$v $OUT/${v}_spans.csv > $OUT/${v}_timeline.log 2>&1 || true
  find $OUT/$v -name "*kernel_trace.csv" -delete
  echo "== $v"; tail -7 $OUT/${v}_timeline.log
done
