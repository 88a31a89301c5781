# kernel-trace stats of the C3 variant lines (occlusion at 3 sigma, netf at 5.7 sigma): the bench
# line and a rocprofv3 --kernel-trace --stats pass of the same command each -> gpurun_out/prof_var
set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof_var; O=gpurun_out/prof_var; mkdir -p $P $O
run() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 600 python bench.py "$@" --no-cpu-baseline > $O/${name}_bench.log 2>&1 || { tail -5 $O/${name}_bench.log; return 1; }
  tail -1 $O/${name}_bench.log | cut -c1-300
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$name -o prof -- python3 bench.py "$@" --no-cpu-baseline > $O/${name}_kt.log 2>&1 || { tail -5 $O/${name}_kt.log; return 1; }
  for f in $(find $P/$name -name "*stats*.csv" -size -40M); do cp $f $O/${name}_$(basename $f); done
}
run occl --mode occl --cutoff 3.0 --steps 1 --warmup 1 || exit 1
run netf --mode netf --steps 2 --warmup 1 || exit 1
ls $O
