set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL $?; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s1.log 2>&1; rc=$?
tail -1 gpurun_out/bench_s1.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c3.log | cut -c1-800
exit $rc
