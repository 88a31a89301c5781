# ray-cache crossover: backward with / without the cache at 4 and 5 sigma, then a short bench
set -o pipefail
export TMPDIR=/tmp NLOSGR_BENCH_PROGRESS=1
mkdir -p gpurun_out
for cut in 4.0 5.0; do
  for cache in 1 0; do
    NLOSGR_ABLATE_CACHE=$cache NLOSGR_ABLATE_CUTOFF=$cut timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/cc_${cut}_${cache}.log 2>&1 || { tail -3 gpurun_out/cc_${cut}_${cache}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/cc_${cut}_${cache}.log').read().strip().splitlines()[-1]);print('cut $cut cache $cache bwd', round(d['bwd_ms_by_flags']['0']))"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; tail -2 gpurun_out/pytest_full.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --lines 3.0 > gpurun_out/bench_iter.log 2> gpurun_out/bench_iter.err || { tail -5 gpurun_out/bench_iter.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['phase_ms'], d['lines'])"
