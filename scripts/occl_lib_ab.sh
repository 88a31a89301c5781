set -e
L=$PWD/nlos-gaussian-renderer_amd/nlosgr
for v in "$@"; do
  NLOSGR_LIB=$L/libnlosgr_$v.so timeout -k 10 200 python bench.py --mode occl --selection aabb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abo_$v.json 2>/dev/null
  echo "$v done"
done
