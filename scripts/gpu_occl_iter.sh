# occlusion engine: parity tests, S1 and C3 (3 sigma) timing
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_occl.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_occl.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_occl.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_occl.log | head; exit $rc; }
timeout -k 10 300 python bench.py --config S1 --mode occl --cutoff 3.0 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/occl_s1.log 2> gpurun_out/occl_s1.err || { tail -5 gpurun_out/occl_s1.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/occl_s1.log').read().strip().splitlines()[-1]);print('S1 occl', d['value'], d['phase_ms'])"
timeout -k 10 600 python bench.py --mode occl --cutoff 3.0 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/occl_c3.log 2> gpurun_out/occl_c3.err || { tail -5 gpurun_out/occl_c3.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/occl_c3.log').read().strip().splitlines()[-1]);print('C3 occl 3', d['value'], d['phase_ms'])"
