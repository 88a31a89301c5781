set -o pipefail
mkdir -p gpurun_out/sw6
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "c3_full_size_train or c3_occl" > gpurun_out/sw6/full.log 2>&1; tail -5 gpurun_out/sw6/full.log
timeout -k 10 200 python scripts/sweep_diag2.py > gpurun_out/sw6/d2.log 2>&1; tail -4 gpurun_out/sw6/d2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sw6/tests.log 2>&1; tail -3 gpurun_out/sw6/tests.log
NLOSGR_FSWEEP=1 NLOSGR_LIB=ab/lib_dbg.so timeout -k 10 200 python scripts/ab_env.py --reps 0 --cutoff 5.7 - > gpurun_out/sw6/eff.log 2>&1 || exit 1
python - <<'PY'
import re
win=0;slots=0;passes=[];n=0
for l in open('gpurun_out/sw6/eff.log'):
    m=re.search(r'slots (\d+) windows (\d+) eff ([\d.]+) passes (\d+) batches (\d+)',l)
    if m: slots+=int(m.group(1)); win+=int(m.group(2)); n+=1
print('waves',n,'eff',slots/(1024*win) if win else 0)
PY
grep -c "sweep dbg" gpurun_out/sw6/eff.log || true
for L in "" ab/lib_cap256.so; do echo "lib=$L"; NLOSGR_FSWEEP=1 NLOSGR_LIB=$L timeout -k 10 200 python scripts/ab_env.py --reps 2 --cutoff 5.7 - NLOSGR_FSWEEP=0 2>&1 | tail -1 || exit 1; done
