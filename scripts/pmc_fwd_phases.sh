# SQ / LDS counters of one C3 forward (TrainStep's slab order) per phase-ablation flag: 0 = full forward,
# 4 = no drain (segment records only), 2 = pair setup only; the differences attribute LDS-array and
# bank-conflict cycles to the drain, the enumeration and the setup.  -> gpurun_out/pmc_fwd_phases/
set -o pipefail
O=gpurun_out/pmc_fwd_phases; mkdir -p $O
for f in ${FLAGS:-0 4 2}; do
  bash scripts/pmc_ab.sh "--flags $f --order slab" - > $O/flags_$f.txt 2>&1 || { tail -5 $O/flags_$f.txt; exit 1; }
  echo "flags $f"; grep fwd_kernel $O/flags_$f.txt
done
