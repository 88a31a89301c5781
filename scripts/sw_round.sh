set -o pipefail
mkdir -p gpurun_out/sw2
timeout -k 10 60 ./scripts/reduce_probe > gpurun_out/sw2/probe.log 2>&1; cat gpurun_out/sw2/probe.log
for L in ab/lib_exact.so ab/lib_mask.so; do NLOSGR_LIB=$L timeout -k 10 120 python scripts/sweep_diag.py >> gpurun_out/sw2/diag.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw2/bench.log 2> gpurun_out/sw2/bench.err || exit 1
NLOSGR_FSWEEP=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw2/bench_ls.log 2> gpurun_out/sw2/bench_ls.err || exit 1
grep -A4 "^lib" gpurun_out/sw2/diag.log
python -c "
import json
for f in ('gpurun_out/sw2/bench.log','gpurun_out/sw2/bench_ls.log'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['phase_ms'])"
