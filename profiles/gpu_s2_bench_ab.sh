# A/B of stage-2 builds on the bench's own extra (stage 2 z, N = 20, over the c4 stage-1
# output): bench.py with extras per in-tree mff/libmff_<v>.so (VARIANTS), twice each
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
cd $R
for rep in 1 2; do
  for v in ${VARIANTS:-a b}; do
    MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 600 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --e2e-days 2 --ingest-days 2 > gpurun_out/s2b_$v$rep.log 2>&1 || { tail -20 gpurun_out/s2b_$v$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/s2b_$v$rep.log') if l.startswith('{')][0]); e=d['extras']; print('$v$rep', e['stage2_z20_all58_ms'], e['stage3_rank_all58_ms'], round(d['value']/1e6,1))"
  done
done
