# iteration check: full GPU suite, C3 phase ablation at the parity cutoff, short bench
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
NLOSGR_ABLATE_CUTOFF=5.7 timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ablate.log 2>&1 || { tail -5 gpurun_out/ablate.log; exit 1; }
tail -1 gpurun_out/ablate.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_iter.log 2> gpurun_out/bench_iter.err || { tail -5 gpurun_out/bench_iter.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['phase_ms'])"
