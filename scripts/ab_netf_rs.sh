mkdir -p gpurun_out
for L in default n20 n24; do
  if [ $L = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/ab/$L.so; fi
  timeout -k 10 200 python scripts/ab_env.py --config C3 --cutoff 5.7 --reps 2 --bwd --mode netf - > gpurun_out/ab_netf_$L.json 2>/dev/null || exit 1
  echo $L; cat gpurun_out/ab_netf_$L.json
done
