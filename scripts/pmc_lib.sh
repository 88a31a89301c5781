# SQ/LDS counter passes over one C3 forward (scripts/ab_env.py --reps 0) per library build:
#   bash scripts/pmc_lib.sh name=path ...   (path "-" = the default library)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_lib; mkdir -p $O
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
for v in "$@"; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$l; fi
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmclib_${n}_$i -o p -- python3 scripts/ab_env.py --reps 0 - > $O/log_${n}_$i.txt 2>&1 || { tail -5 $O/log_${n}_$i.txt; exit 1; }
    f=$(find /tmp/pmclib_${n}_$i -name "*counter_collection.csv" | head -1)
    echo "== $n pass $i"; python3 scripts/pmc_sum.py $f
  done
done
