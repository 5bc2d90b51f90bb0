# A/B timing on one GPU box: bench with libmff_a.so (HEAD) and libmff_b.so (working
# tree), alternating A B A B, each under rocprofv3 kernel stats (profiles/ab_build.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
OUT=$R/gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
for run in a1 b1 a2 b2; do
  v=${run:0:1}
  MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$run -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 3 --warmup 1 ${BENCH_ARGS:-} > $OUT/$run.log 2>&1 || { echo "RUN $run FAILED"; tail -20 $OUT/$run.log; exit 1; }
  find $OUT/$run -name "*kernel_trace.csv" -delete
done
python3 - <<'PY'
import csv, glob, json
R = '/root/repo/gpurun_out/ab'
rows = {}
for run in ('a1', 'b1', 'a2', 'b2'):
    d = json.loads([l for l in open(f'{R}/{run}.log') if l.startswith('{')][0])
    rows.setdefault('value M/s', {})[run] = d['value'] / 1e6
    for f in glob.glob(f'{R}/{run}/**/*kernel_stats.csv', recursive=True):
        for x in csv.DictReader(open(f)):
            if 'mff' in x['Name']:
                rows.setdefault(x['Name'][:60], {})[run] = float(x['AverageNs']) / 1e6
print(f"{'':62s} {'a1':>8s} {'b1':>8s} {'a2':>8s} {'b2':>8s} {'b/a':>7s}")
for k, v in rows.items():
    a = (v.get('a1', 0) + v.get('a2', 0)) / 2
    b = (v.get('b1', 0) + v.get('b2', 0)) / 2
    print(f"{k:62s} " + " ".join(f"{v.get(r, 0):8.3f}" for r in ('a1', 'b1', 'a2', 'b2')) + f" {b / a if a else 0:7.3f}")
PY
