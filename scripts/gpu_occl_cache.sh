# occlusion row cache: occl parity tests, the GPU suite, then the C3 occl line (3 sigma)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|err " gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 500 python bench.py --mode occl --cutoff 3.0 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_occl_3.0.log 2>&1 || { tail -5 gpurun_out/bench_occl_3.0.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_occl_3.0.log').read().strip().splitlines()[-1]);print('occl 3.0', d['value'], d['phase_ms'])"
