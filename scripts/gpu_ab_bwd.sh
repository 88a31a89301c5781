# backward A/B: GPU parity suite on the default build, then C3 phase timing (5.7 sigma, no cache)
# for the default and the alternative build, and the 3 sigma cached line of the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=${ALT:-libnlosgr_bpk0.so}
ALTPATH=${ALTPATH:-$PWD/nlos-gaussian-renderer_amd/nlosgr/$ALT}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|err " gpurun_out/pytest_gpu.log | head -20; exit $rc; }
NLOSGR_ABLATE_CUTOFF=5.7 NLOSGR_ABLATE_CACHE=0 timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ablate_new.log 2>&1 || { tail -5 gpurun_out/ablate_new.log; exit 1; }
tail -1 gpurun_out/ablate_new.log
NLOSGR_LIB=$ALTPATH NLOSGR_ABLATE_CUTOFF=5.7 NLOSGR_ABLATE_CACHE=0 timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ablate_alt.log 2>&1 || { tail -5 gpurun_out/ablate_alt.log; exit 1; }
tail -1 gpurun_out/ablate_alt.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --lines 3.0 > gpurun_out/bench_c3.log 2>&1 || { tail -5 gpurun_out/bench_c3.log; exit 1; }
python -c "import json;L=open('gpurun_out/bench_c3.log').read().strip().splitlines();d=json.loads(L[-1]);print('C3',d['value'],d['phase_ms'],d.get('lines'))"
