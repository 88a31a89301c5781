# backward variants at C3: ray cache on/off, per-wave vs shared rows, at 5.7 and 3 sigma
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cut in 5.7 3.0; do
  for cache in 1 0; do
    for sh in 0 1; do
      NLOSGR_BSHARED=$sh NLOSGR_ABLATE_CACHE=$cache NLOSGR_ABLATE_CUTOFF=$cut timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/bv_${cut}_${cache}_${sh}.log 2>&1 || { tail -3 gpurun_out/bv_${cut}_${cache}_${sh}.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/bv_${cut}_${cache}_${sh}.log').read().strip().splitlines()[-1]);b=d['bwd_ms_by_flags'];print('cut $cut cache $cache shared $sh fwd', round(d['fwd_ms_by_flags']['0']), 'bwd', {k: round(v) for k, v in b.items()})"
    done
  done
done
