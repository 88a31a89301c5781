# round-2 re-entry check: GPU suite, S1 + C3 short bench lines (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s1.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_s1.log').read().strip().splitlines()[-1]);print('S1',d['value'],d['phase_ms'])"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]);print('C3',d['value'],d['phase_ms'])"
