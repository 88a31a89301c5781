# LDS / instruction counters of one C3 (3 sigma) forward: default build vs the bank-sorted drain
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_sort; mkdir -p $O
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
for v in default sort; do
  if [ $v = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/ab/libnlosgr_$v.so; fi
  i=0
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d /tmp/pmc_${v}_$i -o p -- python3 scripts/phase_once.py 0 2 > $O/log_${v}_$i.txt 2>&1 || { tail -5 $O/log_${v}_$i.txt; exit 1; }
    f=$(find /tmp/pmc_${v}_$i -name "*counter_collection.csv" | head -1)
    echo "== $v $i"; python3 scripts/pmc_sum.py $f | tee $O/sum_${v}_$i.txt | grep fwd
  done
done
