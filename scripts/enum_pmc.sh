# SQ counters of the C3 forward/backward with diagnostic flags (5.7 sigma, no ray cache):
#   flags 2 = pair setup only, 1 = + enumeration, 4 = + segment records, 0 = all
set -o pipefail
export TMPDIR=/tmp PHASE_CUTOFF=5.7 PHASE_CACHE=0
O=gpurun_out/enum_pmc; mkdir -p $O
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
for F in 2 1 4; do
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d /tmp/enum_${F}_$i -o p -- python3 scripts/phase_once.py $F $F > $O/log_${F}_$i.txt 2>&1 || { tail -5 $O/log_${F}_$i.txt; exit 1; }
    f=$(find /tmp/enum_${F}_$i -name "*counter_collection.csv" | head -1)
    echo "== flags $F pass $i"; python3 scripts/pmc_sum.py $f
  done
done
