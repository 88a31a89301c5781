# netf: parity / full-size / train tests, then the C3 netf bench line (5.7 sigma)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|err " gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --mode netf --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_netf.log 2>&1 || { tail -5 gpurun_out/bench_netf.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_netf.log').read().strip().splitlines()[-1]);print('C3 netf',d['value'],d['phase_ms'])"
