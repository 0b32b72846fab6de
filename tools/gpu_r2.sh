#!/bin/bash
# round-2 check: chosen GPU suites, bench, kernel trace, one LDS PMC pass.  Stops at the first
# crash/timeout.  usage: tools/gpu_r2.sh TAG "suite args..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out/$TAG
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest $2 -q -rf -s --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/$TAG/tests.log
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'])"
[ $rc -ne 0 ] && exit $rc
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --secondary-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py $ARGS > gpurun_out/$TAG/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/$TAG/pmc_SQ_WAVE_CYCLES -o run -- python3 bench.py $ARGS > gpurun_out/$TAG/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
