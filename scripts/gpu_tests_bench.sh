# GPU test suite, then one short bench line (with the CPU baseline).  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --lines 3.0 $* > gpurun_out/bench_short.log 2>&1 || { tail -20 gpurun_out/bench_short.log; exit 1; }
tail -1 gpurun_out/bench_short.log | cut -c1-3000
