#!/bin/bash
# kernel traces of bench.py steps under two environments (A/B), per-kernel totals of the
# last step side by side.  usage: tools/ab_trace.sh TAG "ENV_A" "ENV_B"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out/$TAG
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --secondary-steps 0 ${AB_ARGS:-}"
for side in A B; do
  if [ $side = A ]; then E="$2"; else E="$3"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/$side -o run -- python3 bench.py $ARGS > gpurun_out/$TAG/$side.log 2>&1 || exit $?
done
python3 tools/step_compare.py gpurun_out/$TAG/A gpurun_out/$TAG/B
