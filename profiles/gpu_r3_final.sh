# round-3 measurement of the working tree: stage-1 profile (bench line, overlapped pass
# timeline, serial per-kernel stats) and the PMC passes.  usage: bash profiles/gpu_r3_final.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03d}
cd $R
bash profiles/gpu_r3_prof.sh $TAG || exit 1
bash profiles/gpu_pmc.sh $TAG || exit 1
python3 - <<PY
import json
d = json.load(open("$R/gpurun_out/pmc_$TAG/pmc_stage1.json"))
print("hbm GB", round(d["hbm_bytes_per_launch"] / 1e9, 1))
for k, v in d["per_kernel"].items():
    print(f"{k:30s} valu/sd {v['valu_per_stock_day']:7.1f}  f64 {v['f64_share']:.3f}  wait {v['wait_frac']:.3f}  hbm GB {v['hbm_bytes'] / 1e9:6.1f}")
PY
