# Same-box A/B of library builds on the C3 bench (interleaved): lib_ab.sh name=path ... (path "-" = default lib)
set -o pipefail
mkdir -p gpurun_out/libab
for rep in 1 2; do
  for v in "$@"; do
    n=${v%%=*}; l=${v#*=}
    if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$l; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/libab/$n.$rep.log 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/libab/$n.$rep.log').read().strip().splitlines()[-1]); print('$n', $rep, round(d['value'],4), {k: round(v,1) for k,v in d['phase_ms'].items()})"
  done
done
