# Timing of the in-tree library and alternative builds ab/<name>.so (one process each):
#   bash scripts/ab_libs.sh "<ab_env args>" name1 name2 ...
mkdir -p gpurun_out
ARGS=$1; shift
timeout -k 10 200 python scripts/ab_env.py $ARGS - > gpurun_out/ab_libs_cur.json 2>/dev/null || exit 1
echo current; cat gpurun_out/ab_libs_cur.json
for L in "$@"; do
  NLOSGR_LIB=$PWD/ab/$L.so timeout -k 10 200 python scripts/ab_env.py $ARGS - > gpurun_out/ab_libs_$L.json 2>/dev/null || exit 1
  echo $L; cat gpurun_out/ab_libs_$L.json
done
