# C3 timing of the ray-tile engine (occlusion, support selection at 3 / 5.7 sigma; AABB selection)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cut in 3.0 5.7; do
  timeout -k 10 400 python bench.py --mode occl --cutoff $cut --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_occl_$cut.log 2>&1 || { tail -5 gpurun_out/bench_occl_$cut.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_occl_$cut.log').read().strip().splitlines()[-1]);print('occl $cut', d['value'], d['phase_ms'])"
done
timeout -k 10 400 python bench.py --mode occl --selection aabb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_occl_aabb.log 2>&1 || { tail -5 gpurun_out/bench_occl_aabb.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_occl_aabb.log').read().strip().splitlines()[-1]);print('occl aabb', d['value'], d['phase_ms'])"
