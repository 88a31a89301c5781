set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_occl.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_occl.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_occl.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_occl.log | head; exit $rc; }
NLOSGR_TILES_DIAG=1 timeout -k 10 300 python bench.py --config S1 --mode occl --cutoff 3.0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/tdiag.log 2> gpurun_out/tdiag.err || { tail -5 gpurun_out/tdiag.err; exit 1; }
grep tiles gpurun_out/tdiag.err
timeout -k 10 300 python bench.py --config S1 --mode occl --cutoff 3.0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/occl_s1.log 2> gpurun_out/occl_s1.err || { tail -5 gpurun_out/occl_s1.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/occl_s1.log').read().strip().splitlines()[-1]);print('S1 occl', d['value'], d['phase_ms'])"
