#!/bin/bash
# Full round check: every GPU test file, the default bench (with CPU baseline), then the
# kernel trace + PMC passes of tools/gpu_profile.sh.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --conv-math bf16 --no-cpu-baseline > gpurun_out/${TAG}_bench_bf16.json 2>> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench bf16 rc=$rc"
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_profile.sh $TAG
