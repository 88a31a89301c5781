# Round-3 lines beside the headline: occlusion (batched step), netf, C5 (all 8 row-interleaved shards on one GPU)
set -o pipefail
OUT=gpurun_out/prof_c3_occl_aabb_b PASSES="kt" bash scripts/prof_c3.sh --mode occl --selection aabb --steps 2 --warmup 1 --no-cpu-baseline || exit 1
OUT=gpurun_out/prof_c3_netf PASSES="bench kt" bash scripts/prof_c3.sh --mode netf --steps 5 --warmup 2 || exit 1
mkdir -p gpurun_out/c5 && NLOSGR_BENCH_PROGRESS=1 timeout -k 10 600 python bench.py --config C5 --band 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5/bench_band8.log 2> gpurun_out/c5/bench_band8.err || exit 1
tail -1 gpurun_out/c5/bench_band8.log | cut -c1-300
