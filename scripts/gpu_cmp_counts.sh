set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/cmp_counts.py > gpurun_out/cmp_tight.log 2>&1 || exit $?
NLOSGR_LIB=$PWD/ab/libnlosgr_loose.so timeout -k 10 200 python scripts/cmp_counts.py > gpurun_out/cmp_loose.log 2>&1 || exit $?
tail -n 1 gpurun_out/cmp_tight.log; tail -n 1 gpurun_out/cmp_loose.log
