# forward drain A/B at C3 (5.7 / 3 sigma): one EXEC region per round (default build), + full-round fast path, HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_exec.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_exec.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_exec.log | head -20; exit $rc; }
export NLOSGR_LIB=$PWD/ab/libnlosgr_full.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "C3" --timeout 200 --timeout-method thread > gpurun_out/pytest_exec_full.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_exec_full.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_exec_full.log | head -20; exit $rc; }
for c in 5.7 3.0; do
for v in default full head; do
  if [ $v = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/ab/libnlosgr_$v.so; fi
  NLOSGR_ABLATE_CACHE=0 NLOSGR_ABLATE_CUTOFF=$c timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo $c $v; tail -1 gpurun_out/ab_$v.log | cut -c1-110
done
done
