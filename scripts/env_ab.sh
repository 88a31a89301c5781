# Interleaved C3 bench A/B of environment variants: env_ab.sh name:VAR=a+VAR2=b name2:- ...
set -o pipefail
mkdir -p gpurun_out/envab
for rep in 1 2; do
  for v in "$@"; do
    n=${v%%:*}; e=${v#*:}
    envs=""; [ "$e" != "-" ] && envs=$(echo $e | tr '+' ' ')
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/envab/$n.$rep.log 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/envab/$n.$rep.log').read().strip().splitlines()[-1]); print('$n', $rep, round(d['value'],4), {k: round(v,1) for k,v in d['phase_ms'].items()})"
  done
done
