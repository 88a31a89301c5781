# A/B of library builds on the ray-tile lines: occl_ab.sh name=path ... (path "-" = the in-tree library)
set -o pipefail
for v in "$@"; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/$l; fi
  timeout -k 10 300 python bench.py --mode occl --selection aabb --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/occl_aabb_$n.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/occl_aabb_$n.json').read().strip().splitlines()[-1]); print('aabb $n', round(d['value'],4), d['phase_ms'])"
done
# full-support occlusion line (one variant per argument again, 2 timed steps)
for v in "$@"; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = "-" ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/$l; fi
  [ -n "$OCCL_FULL" ] || continue
  timeout -k 10 400 python bench.py --mode occl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/occl_full_$n.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/occl_full_$n.json').read().strip().splitlines()[-1]); print('full $n', round(d['value'],4), d['phase_ms'])"
done
