# Round-3 lines beside the headline: netf, C5 (all 8 row-interleaved shards on one GPU), occlusion with
# path C's AABB selection (batched step), AABB selection without occlusion
set -o pipefail
OUT=gpurun_out/prof_c3_netf PASSES="bench kt" bash scripts/prof_c3.sh --mode netf --steps 5 --warmup 2 || exit 1
mkdir -p gpurun_out/c5 && NLOSGR_BENCH_PROGRESS=1 timeout -k 10 600 python bench.py --config C5 --band 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5/bench_band8.log 2> gpurun_out/c5/bench_band8.err || exit 1
tail -1 gpurun_out/c5/bench_band8.log | cut -c1-300
OUT=gpurun_out/prof_c3_occl_aabb PASSES="bench kt" bash scripts/prof_c3.sh --mode occl --selection aabb --steps 3 --warmup 1 --no-cpu-baseline || exit 1
