# SQ counter passes over one C3 forward per variant (scripts/ab_env.py --reps 0), e.g.
#   bash scripts/pmc_ab.sh "--cutoff 5.7" NLOSGR_FREG=0 NLOSGR_FREG=1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_ab; mkdir -p $O
ARGS=$1; shift
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
i=0
for C in "$C1" "$C2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmcab_$i -o p -- python3 scripts/ab_env.py --reps 0 $ARGS "$@" > $O/log_$i.txt 2>&1 || { tail -5 $O/log_$i.txt; exit 1; }
  f=$(find /tmp/pmcab_$i -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_sum.py $f > $O/sum_$i.txt; cat $O/sum_$i.txt
done
