# FETCH_SIZE calibration for the serial kernels' access pattern (guide: calibrate other
# access widths on a known byte count): profiles/ubench/rowload.bin reads two [D][S][240]
# f32 planes (2.4 GB, past the Infinity Cache) four ways; one rocprofv3 --pmc pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/fetch_calib
mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k[ABCD]" -d $OUT/p -o pmc --output-format csv -- $R/profiles/ubench/rowload.bin > $OUT/run.log 2>&1 || { echo CALIB_FAILED; tail -20 $OUT/run.log; exit 1; }
cat $OUT/run.log | grep -v "^\[" | tail -6
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/p/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for x in csv.DictReader(open(f)):
    acc[x["Kernel_Name"].split("(")[0]].append(float(x["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:6s} dispatches {len(v)}  FETCH_SIZE {sum(v) / len(v) / 1e6:.1f} MB per dispatch (KiB units: x1024 -> {sum(v) / len(v) * 1024 / 1e9:.3f} GB) vs 2.400 GB read")
PY
