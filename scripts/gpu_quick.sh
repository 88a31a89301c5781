# parity + C3/S1 timing (no profile); stops at the first failure
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL $?; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s1.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_s1.log').read().strip().splitlines()[-1]);print('S1',d['value'],d['phase_ms'])"
timeout -k 10 600 python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]);print('C3',d['value'],d['phase_ms'],d['roofline_valu']['frac'])"
