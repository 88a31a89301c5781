# Run GPU steps in order, each under its own time limit; stop at the first step whose exit status is not
# 0 or 1 (1 = pytest found failing tests: the kernels ran to completion), i.e. after any fault, abort,
# segfault, timeout or hang.  Usage: bash scripts/gpu_steps.sh "<seconds> <out> <cmd...>" ...
for step in "$@"; do
  set -- $step
  lim=$1; out=$2; shift 2
  echo "[step] $* (limit ${lim}s) -> $out"
  timeout -k 10 "$lim" "$@" > "$out" 2>&1
  rc=$?
  echo "[step] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] stopping: rc $rc"; exit $rc
  fi
done
exit 0
