# Phase ablation at the parity cutoff, then the round profile of the driver's bench command.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
NLOSGR_ABLATE_CUTOFF=5.7 timeout -k 10 300 python scripts/ablate.py C3 > gpurun_out/ablate_c3_57.log 2>&1 || { tail -20 gpurun_out/ablate_c3_57.log; exit 1; }
tail -1 gpurun_out/ablate_c3_57.log
bash scripts/prof_c3.sh
