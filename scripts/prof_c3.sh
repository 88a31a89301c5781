# Round profile of the driver's bench command (bench.py --steps 20 --warmup 5, C3 defaults):
# the bench line itself, a kernel-trace stats pass of the same command, then separate PMC passes
# (FETCH_SIZE; WRITE_SIZE; SQ + GRBM; LDS) as MI355X_MICROARCH.md prescribes.  Output -> gpurun_out/prof_c3.
#   [OUT=gpurun_out/name] PASSES="bench kt fetch write sq lds" bash scripts/prof_c3.sh [extra bench args]
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
O=${OUT:-gpurun_out/prof_c3}; P=/tmp/$(basename $O); mkdir -p $P $O
ARGS="--steps 20 --warmup 5 $*"
PASSES=${PASSES:-"bench kt fetch write sq lds"}
pass() {   # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d $P/$name -o prof -- python3 bench.py $ARGS --no-cpu-baseline > $O/$name.log 2>&1
  local r=$?
  [ $r -eq 0 ] || { tail -5 $O/$name.log; return $r; }
  for f in $(find $P/$name -name "*.csv" -size -40M); do cp $f $O/${name}_$(basename $f); done
}
for ps in $PASSES; do
  case $ps in
    bench) timeout -k 10 600 python bench.py $ARGS > $O/bench_default.log 2> $O/bench_default.err; rc=$?
           tail -1 $O/bench_default.log | cut -c1-400; [ $rc -eq 0 ] || { tail -5 $O/bench_default.err; exit $rc; } ;;
    kt) pass kt --kernel-trace --stats || exit $? ;;
    fetch) pass fetch --pmc FETCH_SIZE || exit $? ;;
    write) pass write --pmc WRITE_SIZE || exit $? ;;
    sq) pass sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit $? ;;
    lds) pass lds --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $? ;;
  esac
done
ls $O
