# Same-box A/B of the tile backward's pair-walk variants on the occlusion lines (bench.py, short runs):
#   bash scripts/occl_walk_ab.sh name=lib.so ...   ("-" = the in-tree library)
set -o pipefail
mkdir -p gpurun_out/walkab
for v in "$@"; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/$l; fi
  for w in "aabb:--selection aabb --steps 3 --warmup 1" "support:--steps 2 --warmup 1"; do
    wn=${w%%:*}; wa=${w#*:}
    timeout -k 10 300 python bench.py --mode occl $wa --no-cpu-baseline > gpurun_out/walkab/$n.$wn.log 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/walkab/$n.$wn.log').read().strip().splitlines()[-1]); print('$n', '$wn', round(d['value'],4), {k: round(v,1) for k,v in d['phase_ms'].items()})"
  done
done
