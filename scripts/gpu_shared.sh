# shared-row backward: parity (default + forced shared layout) then C3 / C5-band timing per layout
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
NLOSGR_BSHARED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_shared.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_gpu_shared.log
[ $rc -eq 0 ] || exit $rc
for sh in 0 1; do
  NLOSGR_BSHARED=$sh timeout -k 10 600 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_sh$sh.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_c3_sh$sh.log').read().strip().splitlines()[-1]);print('C3 shared=$sh',d['value'],d['phase_ms'])"
done
for sh in 0 1; do
  NLOSGR_BSHARED=$sh timeout -k 10 600 python bench.py --config C5 --band 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5band_sh$sh.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_c5band_sh$sh.log').read().strip().splitlines()[-1]);print('C5b shared=$sh',d['value'],d['phase_ms'])"
done
