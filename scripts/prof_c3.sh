# Round profile of the bench command (C3): kernel-trace stats + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ) as MI355X_MICROARCH.md prescribes.  Output -> gpurun_out/prof_c3.
set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof_c3; O=gpurun_out/prof_c3; mkdir -p $P $O
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1; rc=$?
tail -1 $O/bench_default.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o c3 -- python3 bench.py --no-cpu-baseline > $P/kt.log 2>&1; rc=$?
tail -1 $P/kt.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o c3 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/fetch.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 $P/fetch.log; exit $rc; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o c3 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/write.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 $P/write.log; exit $rc; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $P/sq -o c3 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/sq.log 2>&1; rc=$?
for d in kt fetch write sq; do
  for f in $(find $P/$d -name "*.csv" -size -20M); do cp $f $O/${d}_$(basename $f); done
done
ls $O
exit $rc
