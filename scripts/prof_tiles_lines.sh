# Ray-tile engine lines (C3, 5.7 sigma): occlusion + path C AABB selection, AABB without occlusion,
# occlusion over the whole support; bench line + kernel stats each
set -o pipefail
OUT=gpurun_out/prof_c3_occl_aabb PASSES="bench kt" bash scripts/prof_c3.sh --mode occl --selection aabb --steps 3 --warmup 1 --no-cpu-baseline || exit 1
OUT=gpurun_out/prof_c3_aabb PASSES="bench kt" bash scripts/prof_c3.sh --selection aabb --steps 3 --warmup 1 --no-cpu-baseline || exit 1
OUT=gpurun_out/prof_c3_occl PASSES="bench" bash scripts/prof_c3.sh --mode occl --steps 2 --warmup 1 --no-cpu-baseline || exit 1
