# occlusion engine counters at S1 (one step), then all 8 C5 bands timed on one GPU
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
O=gpurun_out/occl_prof; mkdir -p $O
timeout -k 10 300 python bench.py --config S1 --mode occl --cutoff 3.0 --steps 1 --warmup 1 --no-cpu-baseline > $O/s1.log 2> $O/s1.err || { tail -5 $O/s1.err; exit 1; }
tail -1 $O/s1.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/oc_kt -o p -- python3 bench.py --config S1 --mode occl --cutoff 3.0 --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
cp $(find /tmp/oc_kt -name "*kernel_stats.csv") $O/
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d /tmp/oc_sq -o p -- python3 bench.py --config S1 --mode occl --cutoff 3.0 --steps 1 --warmup 0 --no-cpu-baseline > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
cp $(find /tmp/oc_sq -name "*counter_collection.csv") $O/
timeout -k 10 900 python bench.py --config C5 --band 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_bands.log 2> gpurun_out/bench_c5_bands.err || { tail -5 gpurun_out/bench_c5_bands.err; exit 1; }
tail -1 gpurun_out/bench_c5_bands.log | cut -c1-600
