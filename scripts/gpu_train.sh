# training-step parity + the full GPU suite + one default bench line (stops at the first failure)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_train.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
tail -1 gpurun_out/bench_default.log | cut -c1-900
exit $rc
