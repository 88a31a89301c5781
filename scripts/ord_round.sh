set -o pipefail
mkdir -p gpurun_out/ord
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_occl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ord/tests.log 2>&1; tail -3 gpurun_out/ord/tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ord/bench.log 2> gpurun_out/ord/bench.err || exit 1
NLOSGR_BWD_ORDER=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ord/bench0.log 2> gpurun_out/ord/bench0.err || exit 1
python -c "
import json
for f in ('gpurun_out/ord/bench.log','gpurun_out/ord/bench0.log'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['phase_ms'])"
