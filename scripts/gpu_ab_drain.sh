# forward drain A/B at C3, 5.7 sigma: masked losers (default build), round-1 pads, bank-slot claims
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default base slot; do
  if [ $v = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/ab/libnlosgr_$v.so; fi
  NLOSGR_ABLATE_CUTOFF=5.7 timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo $v; tail -1 gpurun_out/ab_$v.log | cut -c1-200
done
