#!/bin/bash
# Run GPU parity suites; stop at the first crash/timeout (exit > 1), keep going on plain test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for suite in "$@"; do
  name=$(basename "$suite" .py)
  timeout -k 10 900 python -m pytest "$suite" -q -rf -p no:cacheprovider > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
