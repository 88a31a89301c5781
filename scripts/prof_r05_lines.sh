# Round-5 lines beside the headline (each a bench.py run; JSON lines under gpurun_out/lines_r05):
# netf, occlusion with path C's AABB selection, occlusion over the full 5.7-sigma support, AABB selection
# without occlusion, C5 (all 8 row-interleaved shards on one GPU), C2 forward, C1 dense torch preset,
# and the C4 analytic-vs-numerical cross-check.
set -o pipefail
O=gpurun_out/lines_r05; mkdir -p $O
run() {   # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  NLOSGR_BENCH_PROGRESS=1 timeout -k 10 $t python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  tail -1 $O/$n.json | cut -c1-240
}
run c3_netf 400 --mode netf --steps 5 --warmup 2 --no-cpu-baseline || exit 1
run c3_occl_aabb 400 --mode occl --selection aabb --steps 3 --warmup 1 --no-cpu-baseline || exit 1
run c3_aabb 400 --selection aabb --steps 3 --warmup 1 --no-cpu-baseline || exit 1
run c3_occl 600 --mode occl --steps 2 --warmup 1 --no-cpu-baseline || exit 1
run c5_band8 900 --config C5 --band 8 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
run c2 300 --config C2 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run c1_torch_dense 600 --config C1 --preset torch --cutoff 0 --steps 20 --warmup 5 || exit 1
timeout -k 10 600 python scripts/c4_crosscheck.py > $O/c4.json 2> $O/c4.err || { tail -3 $O/c4.err; exit 1; }
tail -1 $O/c4.json | cut -c1-300
