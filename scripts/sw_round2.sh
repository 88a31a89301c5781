set -o pipefail
mkdir -p gpurun_out/sw3
NLOSGR_LIB=ab/lib_dbg.so timeout -k 10 120 python scripts/sweep_diag.py > gpurun_out/sw3/dbg.log 2>&1 || exit 1
grep -c "sweep dbg" gpurun_out/sw3/dbg.log; grep "sweep dbg" gpurun_out/sw3/dbg.log | head -20; grep -A3 "^lib" gpurun_out/sw3/dbg.log
bash scripts/pmc_ab.sh "--cutoff 5.7" - NLOSGR_FSWEEP=0
