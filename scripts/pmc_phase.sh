# SQ counter passes over one C3 fwd+bwd (scripts/phase_once.py) at flags 0 and 4 (no bins)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_phase; mkdir -p $O
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
for fl in 0 4; do
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d /tmp/pmc_${fl}_$i -o p -- python3 scripts/phase_once.py $fl $fl > $O/log_${fl}_$i.txt 2>&1 || { tail -5 $O/log_${fl}_$i.txt; exit 1; }
    f=$(find /tmp/pmc_${fl}_$i -name "*counter_collection.csv" | head -1)
    python3 scripts/pmc_sum.py $f > $O/sum_${fl}_$i.txt; cat $O/sum_${fl}_$i.txt
  done
done
