#!/bin/bash
# kernel trace of the bf16-arithmetic step (config 3): per-kernel totals of one step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-bf16}
mkdir -p gpurun_out/$TAG
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --secondary-steps 0 --conv-math bf16"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/A -o run -- python3 bench.py $ARGS > gpurun_out/$TAG/A.log 2>&1 || exit $?
python3 tools/step_compare.py gpurun_out/$TAG/A gpurun_out/$TAG/A
