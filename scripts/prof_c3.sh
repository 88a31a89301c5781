# Round profile of the driver's bench command (bench.py --steps 20 --warmup 5, C3 defaults):
# the bench line itself, a kernel-trace stats pass of the same command, then separate PMC passes
# (FETCH_SIZE; WRITE_SIZE; SQ + GRBM) as MI355X_MICROARCH.md prescribes.  Output -> gpurun_out/prof_c3.
#   bash scripts/prof_c3.sh [extra bench args]
set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof_c3; O=gpurun_out/prof_c3; mkdir -p $P $O
ARGS="--steps 20 --warmup 5 $*"
timeout -k 10 600 python bench.py $ARGS > $O/bench_default.log 2>&1; rc=$?
tail -1 $O/bench_default.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o prof -- python3 bench.py $ARGS --no-cpu-baseline > $P/kt.log 2>&1; rc=$?
tail -1 $P/kt.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o prof -- python3 bench.py $ARGS --no-cpu-baseline > $P/fetch.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 $P/fetch.log; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o prof -- python3 bench.py $ARGS --no-cpu-baseline > $P/write.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 $P/write.log; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq -o prof -- python3 bench.py $ARGS --no-cpu-baseline > $P/sq.log 2>&1; rc=$?
for d in kt fetch write sq; do
  for f in $(find $P/$d -name "*.csv" -size -40M); do cp $f $O/${d}_$(basename $f); done
done
ls $O
exit $rc
