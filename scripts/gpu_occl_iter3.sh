# occlusion engine iteration: phase counters (S1), GPU suite, C3 occl line (3 sigma)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tiles_diag.sh || exit 1
bash scripts/gpu_occl_cache.sh
