set -o pipefail
mkdir -p gpurun_out/walkab
for rep in 1 2; do
for v in cur=- all=ab/walk_all.so; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/$l; fi
  timeout -k 10 300 python bench.py --selection aabb --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/walkab/aabb_$n.log 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/walkab/aabb_$n.log').read().strip().splitlines()[-1]); print('$n', $rep, round(d['value'],4), {k: round(v,1) for k,v in d['phase_ms'].items()})"
done
done
