# Round-6 lines beside the headline (each a bench.py run with >= 5 timed steps; JSON lines under
# gpurun_out/lines_r06): occlusion with path C's AABB selection, AABB selection without occlusion,
# occlusion over the full 5.7-sigma support, netf; then the tile-engine phase counters (diagnostic build)
# with and without the tile bins.   LINES="occl_aabb aabb occl netf diag" bash scripts/prof_r06_lines.sh
set -o pipefail
O=gpurun_out/lines_r06; mkdir -p $O
export TMPDIR=/tmp
run() {   # name, timeout, bench args...  (under rocprofv3 --kernel-trace --stats: kernel stats beside the line)
  local n=$1 t=$2; shift 2
  rm -rf /tmp/kt_$n
  NLOSGR_BENCH_PROGRESS=1 timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$n -o prof -- python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  cp $(find /tmp/kt_$n -name "*kernel_stats.csv" | head -1) $O/${n}_kernel_stats.csv
  tail -1 $O/$n.json | cut -c1-240
}
for l in ${LINES:-occl_aabb aabb occl netf diag}; do
  case $l in
    occl_aabb) run c3_occl_aabb 400 --mode occl --selection aabb --steps 5 --warmup 1 --no-cpu-baseline || exit 1 ;;
    aabb) run c3_aabb 400 --selection aabb --steps 5 --warmup 1 --no-cpu-baseline || exit 1 ;;
    occl) run c3_occl 900 --mode occl --steps 5 --warmup 1 --no-cpu-baseline || exit 1 ;;
    netf) run c3_netf 400 --mode netf --steps 5 --warmup 2 --no-cpu-baseline || exit 1 ;;
    diag) for v in "" nobin; do
            NLOSGR_LIB=$PWD/ab/diag.so timeout -k 10 300 python scripts/occl_diag.py occl aabb $v > $O/diag_aabb_$v.txt 2>&1 || exit 1
            NLOSGR_LIB=$PWD/ab/diag.so timeout -k 10 300 python scripts/occl_diag.py occl support $v > $O/diag_support_$v.txt 2>&1 || exit 1
          done; grep -h "tiles" $O/diag_*.txt ;;
  esac
done
