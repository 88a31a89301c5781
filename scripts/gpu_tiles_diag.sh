# ray-tile engine phase counters: build ab/libnlosgr_diag.so first on the CPU side with
#   python nlos-gaussian-renderer_amd/build.py --out ab/libnlosgr_diag.so -D NLOSGR_TILES_DIAG_BUILD=1
set -o pipefail
export TMPDIR=/tmp NLOSGR_TILES_DIAG=1 NLOSGR_LIB=$PWD/ab/libnlosgr_diag.so
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config S1 --mode occl --cutoff 3.0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/tdiag.log 2> gpurun_out/tdiag.err || { tail -5 gpurun_out/tdiag.err; exit 1; }
grep tiles gpurun_out/tdiag.err
