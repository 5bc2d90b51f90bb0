# A/B timing on one GPU box: bench with libmff_a.so (HEAD) and libmff_b.so (working
# tree), alternating A B A B, each under rocprofv3 kernel stats (profiles/ab_build.sh).
# VARIANTS="a b c ..." times more in-tree builds mff/libmff_<v>.so the same way;
# ENV_<v>="NAME=value ..." sets extra environment for variant <v> (e.g. ENV_b="MFF_PDF_OVERLAP=0").
set -o pipefail
R=$GRAFT_REPO_ROOT
PKG=replication-of-minute-frequency-factor_amd
OUT=$R/gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
VARIANTS=${VARIANTS:-a b}
RUNS=""
for rep in 1 2; do for v in $VARIANTS; do RUNS="$RUNS $v$rep"; done; done
for run in $RUNS; do
  v=${run:0:1}
  eval "XENV=\${ENV_$v:-}"
  ( [ -n "$XENV" ] && export $XENV
  MFF_LIBRARY=$R/$PKG/mff/libmff_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$run -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 3 --warmup 1 ${BENCH_ARGS:-} > $OUT/$run.log 2>&1 ) || { echo "RUN $run FAILED"; tail -20 $OUT/$run.log; exit 1; }
  find $OUT/$run -name "*kernel_trace.csv" -delete
done
VARIANTS="$VARIANTS" python3 - <<'PY'
import csv, glob, json, os
R = '/root/repo/gpurun_out/ab'
V = os.environ['VARIANTS'].split()
runs = [f'{v}{r}' for r in (1, 2) for v in V]
rows = {}
for run in runs:
    d = json.loads([l for l in open(f'{R}/{run}.log') if l.startswith('{')][0])
    rows.setdefault('value M/s', {})[run] = d['value'] / 1e6
    for k, x in ((d.get('roofline') or {}).get('kernels') or {}).items():
        if isinstance(x, dict):
            rows.setdefault('alone ' + k[:54], {})[run] = x['ms']
    for f in glob.glob(f'{R}/{run}/**/*kernel_stats.csv', recursive=True):
        for x in csv.DictReader(open(f)):
            if 'mff' in x['Name']:
                rows.setdefault(x['Name'][:60], {})[run] = float(x['AverageNs']) / 1e6
print(f"{'':62s} " + " ".join(f"{v:>8s}" for v in V) + "   (mean of 2 runs; ratio to the first)")
for k, x in rows.items():
    m = [(x.get(f'{v}1', 0) + x.get(f'{v}2', 0)) / 2 for v in V]
    print(f"{k:62s} " + " ".join(f"{y:8.3f}" for y in m) + "  " + " ".join(f"{y / m[0] if m[0] else 0:6.3f}" for y in m[1:]))
PY
