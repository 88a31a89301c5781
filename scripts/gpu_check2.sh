# full GPU suite, then a short C3 bench (5.7 sigma + the 3 sigma line)
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --lines 3.0 --no-cpu-baseline > gpurun_out/bench_iter.log 2> gpurun_out/bench_iter.err || { tail -5 gpurun_out/bench_iter.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['phase_ms'], d.get('lines'))" | cut -c1-600
