# A/B: default build vs libnlosgr_alt.so (C3 bench phases), after the GPU parity tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for lib in default alt; do
  if [ $lib = alt ]; then export NLOSGR_LIB=$PWD/nlos-gaussian-renderer_amd/nlosgr/libnlosgr_alt.so; fi
  timeout -k 10 600 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$lib.log 2>&1 || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/bench_$lib.log').read().strip().splitlines()[-1]);print('$lib',d['value'],d['phase_ms'])"
done
