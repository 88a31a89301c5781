# A/B of in-tree builds on the C5 eight-band projection: bash scripts/c5_ab.sh v1 v2 ...
set -e
L=$PWD/nlos-gaussian-renderer_amd/nlosgr
for v in "$@"; do
  NLOSGR_LIB=$L/libnlosgr_$v.so NLOSGR_BENCH_PROGRESS=1 timeout -k 10 400 python bench.py --config C5 --band 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab5_$v.json 2> gpurun_out/ab5_$v.err
  echo "$v done"
done
