set -o pipefail
mkdir -p gpurun_out/c4
timeout -k 10 300 python -u -m pytest tests/test_gpu_analytic.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c4/tests.log 2>&1; tail -3 gpurun_out/c4/tests.log
timeout -k 10 300 python scripts/c4_crosscheck.py --cutoffs 5.7 > gpurun_out/c4/c4.json 2> gpurun_out/c4/c4.err || exit 1
tail -c 700 gpurun_out/c4/c4.json
