set -o pipefail
timeout -k 10 600 python scripts/ablate.py S1 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python scripts/ablate.py C3 2>&1 | grep -v amdgpu.ids
