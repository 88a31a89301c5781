set -o pipefail
mkdir -p gpurun_out/slab
for S in "16,8" "8,8" "32,8" "16,4" "16,16" "32,16" "64,8" "8,4"; do
  NLOSGR_SLAB=$S timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/slab/b_$S.log 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/slab/b_$S.log').read().strip().splitlines()[-1]); print('$S', round(d['value'],4), d['phase_ms'])"
done
