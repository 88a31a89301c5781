# round-2 lines for the other BASELINE configs (each JSON line -> gpurun_out/cfg_<name>.json)
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
run() {   # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" > gpurun_out/cfg_$name.log 2> gpurun_out/cfg_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/cfg_$name.err; return 1; }
  tail -1 gpurun_out/cfg_$name.log > gpurun_out/cfg_$name.json
  python -c "import json;d=json.load(open('gpurun_out/cfg_$name.json'));print('$name', d['value'], d['unit'], d.get('phase_ms'))"
}
run c1_torch_dense 400 --config C1 --preset torch --cutoff 0 --steps 10 --warmup 2 || exit 1
run c2 400 --config C2 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
run c3_netf 600 --mode netf --steps 3 --warmup 1 --no-cpu-baseline || exit 1
run c3_occl 600 --mode occl --cutoff 3.0 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
