set -o pipefail
for L in "" ab/lib_cap256.so; do echo "lib=$L"; NLOSGR_LIB=$L timeout -k 10 200 python scripts/ab_env.py --reps 2 --cutoff 5.7 NLOSGR_FSWEEP=1 NLOSGR_FSWEEP=0 2>&1 | tail -1 || exit 1; done
