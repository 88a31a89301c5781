# new GPU tests, the round profile of the bench command, then the occlusion engine's C3 timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_rays.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_new.log | tail -30
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_new.log | tail -20; exit $rc; }
bash scripts/prof_c3.sh || exit $?
bash scripts/gpu_occl_bench.sh
