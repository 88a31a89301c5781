# tile-engine parity tests (occlusion / AABB selection), then the rest of the GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_occl.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_occl.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_occl.log | tail -40
exit $rc
