# every stage-1 launch alone (bench --kernel-times: serial, HIP events) for each in-tree
# build mff/libmff_<v>.so (VARIANTS), alternating, twice; ENV_<v>="NAME=value ..." sets
# extra environment for variant <v>
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
OUT=$R/gpurun_out/alone
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in ${VARIANTS:-a b}; do
    eval "XENV=\${ENV_$v:-}"
    ( [ -n "$XENV" ] && export $XENV
      MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --kernel-times --steps 5 --warmup 2 > $OUT/$v$rep.log 2>&1 ) || { echo "RUN $v$rep FAILED"; tail -20 $OUT/$v$rep.log; exit 1; }
    grep '^{' $OUT/$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('$v$rep', round(d['value']/1e6,1), ' '.join(f'{n.split(\"<\")[0].split(\" \")[0]}={x[\"ms\"]}' for n,x in k.items() if isinstance(x,dict)))"
  done
done
