# refill-threshold sweep at the parity cutoff (C3 phase timing, default build vs ab/lib_*.so)
set -o pipefail
export TMPDIR=/tmp NLOSGR_ABLATE_CUTOFF=5.7 NLOSGR_ABLATE_CACHE=0
mkdir -p gpurun_out
for v in ${SWEEP:-default R16 R48 B4 B16}; do
  if [ $v = default ]; then L=""; else L=$PWD/ab/lib_$v.so; fi
  NLOSGR_LIB=$L timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ablate_$v.log 2>&1 || { tail -5 gpurun_out/ablate_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ablate_$v.log').read().strip().splitlines()[-1]);print('$v fwd',round(d['fwd_ms_by_flags']['0'],1),'bwd',round(d['bwd_ms_by_flags']['0'],1))"
done
