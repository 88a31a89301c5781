# SURVEY §8d variant bench lines: C1 (torch preset, dense, every sample) and C3 netf.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/variants
timeout -k 10 300 python bench.py --config C1 --preset torch --cutoff 0 --steps 5 --warmup 1 > gpurun_out/variants/c1_torch_dense.log 2>&1 || { tail -20 gpurun_out/variants/c1_torch_dense.log; exit 1; }
tail -1 gpurun_out/variants/c1_torch_dense.log | cut -c1-400
timeout -k 10 400 python bench.py --config C3 --mode netf --steps 3 --warmup 1 > gpurun_out/variants/c3_netf.log 2>&1 || { tail -20 gpurun_out/variants/c3_netf.log; exit 1; }
tail -1 gpurun_out/variants/c3_netf.log | cut -c1-400
