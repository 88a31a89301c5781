set -o pipefail
mkdir -p gpurun_out/sw4
timeout -k 10 200 python scripts/sweep_diag2.py > gpurun_out/sw4/d2.log 2>&1 || exit 1
cat gpurun_out/sw4/d2.log | grep "^ng"
NLOSGR_LIB=ab/lib_dbg.so timeout -k 10 200 python scripts/ab_env.py --reps 0 --cutoff 5.7 - > gpurun_out/sw4/eff.log 2>&1 || exit 1
python - <<'PY'
import re
effs=[];win=0;slots=0;passes=[];batches=[]
for l in open('gpurun_out/sw4/eff.log'):
    m=re.search(r'slots (\d+) windows (\d+) eff ([\d.]+) passes (\d+) batches (\d+)',l)
    if m:
        slots+=int(m.group(1)); win+=int(m.group(2)); passes.append(int(m.group(4))); batches.append(int(m.group(5)))
print('waves',len(passes),'eff',slots/(1024*win) if win else 0,'mean passes',sum(passes)/max(1,len(passes)),'mean batches',sum(batches)/max(1,len(batches)))
PY
grep -c "sweep dbg" gpurun_out/sw4/eff.log || true
