# A/B of alternative in-tree builds (libnlosgr_<v>.so) on a C3 bench line, in one process per build:
#   bash scripts/netf_ab.sh v1 v2 ...            (netf)
#   MODE=noocl bash scripts/netf_ab.sh v1 v2 ...  (the headline's mode)
set -e
L=$PWD/nlos-gaussian-renderer_amd/nlosgr
M=${MODE:-netf}
for v in "$@"; do
  NLOSGR_LIB=$L/libnlosgr_$v.so timeout -k 10 200 python bench.py --mode $M --steps 4 --warmup 1 > gpurun_out/ab_${M}_$v.json 2>/dev/null
  echo "$v done"
done
