#!/bin/bash
# Round-end pass on one box, in two parts (each fits one gpurun call):
#   bash tools/gpu_final.sh TAG tests   -- every GPU test file, the fp32 bench line (with the CPU
#                                          baseline), the bf16 line and the Herlev 256^2 line
#   bash tools/gpu_final.sh TAG prof    -- kernel trace + PMC passes, fp32 and bf16
# Stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; PART=${2:?tests|prof}
mkdir -p gpurun_out
case $PART in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
    [ $rc -gt 1 ] && exit $rc
    timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
    rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${TAG}_bench.json
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python bench.py --conv-math bf16 --no-cpu-baseline > gpurun_out/${TAG}_bench_bf16.json 2>> gpurun_out/${TAG}_bench.err
    rc=$?; echo "bench bf16 rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 600 python bench.py --workload herlev --res 256 > gpurun_out/${TAG}_herlev256.json 2>> gpurun_out/${TAG}_bench.err
    rc=$?; echo "herlev rc=$rc"; exit $rc ;;
  prof)
    bash tools/gpu_profile.sh $TAG || exit $?
    EXTRA='--conv-math bf16' bash tools/gpu_profile.sh ${TAG}_bf16 ;;
esac
