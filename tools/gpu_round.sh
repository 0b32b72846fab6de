#!/bin/bash
# tests -> bench -> rocprof kernel-trace stats; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_herlev.py tests/test_gpu_eval.py tests/test_gpu_augment.py || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
exit $rc
