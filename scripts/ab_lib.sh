# Same-config timing of the in-tree library against an alternative build (ab/<name>.so), one process each:
#   bash scripts/ab_lib.sh <name> [ab_env.py args]
mkdir -p gpurun_out
ALT=$1; shift
timeout -k 10 200 python scripts/ab_env.py "$@" - > gpurun_out/ab_lib_cur.json 2>/dev/null || exit 1
NLOSGR_LIB=$PWD/ab/$ALT.so timeout -k 10 200 python scripts/ab_env.py "$@" - > gpurun_out/ab_lib_alt.json 2>/dev/null || exit 1
echo current; cat gpurun_out/ab_lib_cur.json; echo $ALT; cat gpurun_out/ab_lib_alt.json
