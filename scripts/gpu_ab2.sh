# parity of the current build, then A/B phase timing against alternative builds given as args
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_abn.sh default "$@"
