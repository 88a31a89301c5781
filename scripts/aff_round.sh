set -o pipefail
mkdir -p gpurun_out/aff
timeout -k 10 300 python scripts/ab_env.py --reps 2 --cutoff 5.7 --bwd NLOSGR_BAFF=1 NLOSGR_BAFF=0 > gpurun_out/aff/ab.log 2>&1 || { tail -5 gpurun_out/aff/ab.log; exit 1; }
tail -1 gpurun_out/aff/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/aff/tests.log 2>&1; tail -3 gpurun_out/aff/tests.log
