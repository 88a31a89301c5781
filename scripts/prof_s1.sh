set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof; mkdir -p $P gpurun_out/prof
rocprofv3 -L > $P/counters.txt 2>&1 || true
grep -oE "^\s*(SQ_|TCC_|TCP_|GRBM_)[A-Z0-9_]+" $P/counters.txt | sort -u | tr -d ' ' > gpurun_out/prof/counter_names.txt || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o s1 -- python bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline > $P/kt.log 2>&1; rc=$?
tail -3 $P/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/pmc1 -o s1 -- python bench.py --config S1 --steps 1 --warmup 0 --no-cpu-baseline > $P/pmc1.log 2>&1; rc=$?
tail -3 $P/pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $P/pmc2 -o s1 -- python bench.py --config S1 --steps 1 --warmup 0 --no-cpu-baseline > $P/pmc2.log 2>&1; rc=$?
tail -3 $P/pmc2.log
find $P -name "*.csv" -size -20M -exec cp {} gpurun_out/prof/ \;
ls -la gpurun_out/prof
exit $rc
