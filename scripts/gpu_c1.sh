# GPU tests, then the C1 (torch preset, dense) bench line.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C1 --preset torch --cutoff 0 --steps 5 --warmup 1 > gpurun_out/variants/c1_torch_dense.log 2>&1 || { tail -20 gpurun_out/variants/c1_torch_dense.log; exit 1; }
tail -1 gpurun_out/variants/c1_torch_dense.log | cut -c1-600
