# Phase ablation (scripts/ablate.py C3) for each library build given as an argument
# (paths relative to the repo; "default" = nlosgr/libnlosgr.so).  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${ABN_CFG:-C3}
for lib in "$@"; do
  if [ "$lib" = default ]; then unset NLOSGR_LIB; else export NLOSGR_LIB=$PWD/$lib; fi
  timeout -k 10 300 python scripts/ablate.py $cfg > gpurun_out/abn_$(basename $lib).log 2>&1 || { tail -5 gpurun_out/abn_$(basename $lib).log; exit 1; }
  echo "$lib $(grep -v amdgpu.ids gpurun_out/abn_$(basename $lib).log | tail -1)"
done
