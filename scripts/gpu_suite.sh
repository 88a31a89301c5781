# full GPU suite (log in gpurun_out/pytest_gpu.log)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
