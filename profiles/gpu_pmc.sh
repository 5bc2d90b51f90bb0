# PMC passes (one counter group per run, gfx950 slot limits) over a short bench run.
# usage: bash profiles/gpu_pmc.sh TAG [stocks] [days]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
S=${2:-5000}
D=${3:-250}
KRE=${4:-mff}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" -d $OUT/p$i -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 0 --stocks $S --days $D > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/profiles/pmc_table.py $OUT > $OUT/table.txt
python3 $R/profiles/pmc_json.py $OUT $S $D $TAG $OUT/pmc_stage1.json
