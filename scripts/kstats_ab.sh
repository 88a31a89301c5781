# rocprofv3 kernel stats of scripts/ab_env.py for the in-tree package and variants (same box), summarised.
#   bash scripts/kstats_ab.sh "<ab_env args>" [pkg:DIR | lib:PATH.so ...]
export TMPDIR=/tmp
ARGS=$1; shift
O=gpurun_out/kstats_ab; mkdir -p $O
i=0
for v in cur "$@"; do
  P=/tmp/kst$i; rm -rf $P
  case $v in
    cur) extra=""; lib=""; name=cur ;;
    pkg:*) extra="--pkg ${v#pkg:}"; lib=""; name=$(basename ${v#pkg:}) ;;
    lib:*) extra=""; lib=$PWD/${v#lib:}; name=$(basename ${v#lib:} .so) ;;
  esac
  NLOSGR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o prof -- python3 scripts/ab_env.py $ARGS $extra - > $O/$name.log 2>&1 || exit $?
  f=$(find $P -name "*kernel_stats.csv" | head -1)
  cp $f $O/${name}_kernel_stats.csv
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:6]:
    print('$name', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
"
  i=$((i+1))
done
