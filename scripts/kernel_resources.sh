# VGPR / SGPR / scratch per kernel of one source file (device-only assembly for gfx950).
#   bash scripts/kernel_resources.sh nlosgr_volume [pattern]
set -e
src=${1:-nlosgr_volume}; pat=${2:-.}
out=/tmp/nlosgr_isa; mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -fno-slp-vectorize -fno-vectorize \
  -I "$(dirname "$0")/../include" --cuda-device-only -S -o $out/$src.s \
  "$(dirname "$0")/../nlos-gaussian-renderer_amd/csrc/$src.hip" 2>/dev/null
awk '/^ +\.name:/{n=$2} /\.private_segment_fixed_size:/{p=$2} /\.sgpr_count:/{s=$2} /\.vgpr_count:/{print n, "vgpr="$2, "sgpr="s, "scratch="p}' \
  $out/$src.s | c++filt | sed 's/(anonymous namespace):://; s/(KArgs)//' | grep -E "$pat" || true
