# A/B of mff/libmff_a.so and mff/libmff_b.so on the c4 headline (bench.py) and on the c4
# dense vs c5 ragged pass (profiles/ragged_probe.py), interleaved a b a b.
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
OUT=$R/gpurun_out/abrag
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in ${VARIANTS:-a b}; do
    MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 8 --warmup 2 > $OUT/b_$v$rep.log 2>&1 || { echo "BENCH $v FAILED"; tail -20 $OUT/b_$v$rep.log; exit 1; }
    MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 python -u profiles/ragged_probe.py > $OUT/r_$v$rep.log 2>&1 || { echo "PROBE $v FAILED"; tail -20 $OUT/r_$v$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$v$rep.log') if l.startswith('{')][0]); print('$v$rep headline', round(d['value']/1e6,2), 'M/s')"
    grep "pass" $OUT/r_$v$rep.log | grep -v "^[EWI]20" | sed "s/^/$v$rep /"
  done
done
