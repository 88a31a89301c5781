# forward A/B at C3 (5.7 and 3 sigma): compact 7-wave quad layout (default build) vs the general 6-wave layout
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_compact.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_compact.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_compact.log | head -20; exit $rc; }
for c in 5.7 3.0; do
for v in default nc; do
  if [ $v = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/ab/libnlosgr_$v.so; fi
  NLOSGR_ABLATE_CACHE=0 NLOSGR_ABLATE_CUTOFF=$c timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo $c $v; tail -1 gpurun_out/ab_$v.log | cut -c1-140
done
done
