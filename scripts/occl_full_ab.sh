# forward-only A/B of in-tree builds on the C3 full-support occlusion line: bash scripts/occl_full_ab.sh v1 v2 ...
set -e
L=$PWD/nlos-gaussian-renderer_amd/nlosgr
for v in "$@"; do
  NLOSGR_LIB=$L/libnlosgr_$v.so timeout -k 10 300 python bench.py --mode occl --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/abf_$v.json 2>/dev/null
  echo "$v done"
done
