# C3 single-GPU sanity + C5's eight row-interleaved shards timed in turn on one GPU (5.7 sigma)
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['phase_ms'])"
timeout -k 10 900 python bench.py --config C5 --band 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_rows.log 2> gpurun_out/bench_c5_rows.err || { tail -5 gpurun_out/bench_c5_rows.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/bench_c5_rows.log').read().strip().splitlines()[-1]);print('C5', d['value'], d['ms_per_step'])
for b in d['bands']: print(b['band'], round(b['ms_per_step'],1), round(b['fwd_ms'],1), round(b['bwd_ms'],1))"
