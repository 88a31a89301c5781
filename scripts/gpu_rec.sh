# parity of the recurrence drains + training step, then A/B phase timing vs the per-bin exp2 build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rec.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_rec.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_abn.sh default nlos-gaussian-renderer_amd/nlosgr/libnlosgr_v0.so
