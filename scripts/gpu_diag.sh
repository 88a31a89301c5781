set -o pipefail
timeout -k 10 600 python scripts/diag_cutoff2.py > gpurun_out/diag.log 2>&1; rc=$?
cat gpurun_out/diag.log | grep -v amdgpu.ids
exit $rc
