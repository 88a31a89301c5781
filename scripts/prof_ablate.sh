# Per-phase instruction counters: rocprofv3 SQ counters over scripts/ablate.py (flags 0/4/1/2
# = full / no drain / enumerate only / pair setup only; each run twice, fwd then bwd).
set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof_abl; O=gpurun_out/prof_abl; mkdir -p $P $O
cfg=${ABN_CFG:-C3}
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $P/sq -o abl -- python3 scripts/ablate.py $cfg > $P/sq.log 2>&1; rc=$?
tail -2 $P/sq.log
for f in $(find $P/sq -name "*counter_collection.csv"); do cp $f $O/; done
exit $rc
