#!/bin/bash
# Round-3 GPU session: selected tests, then benches (config 2 default, config 3 bf16,
# config 4 Herlev at 256 and 224), then the U-map stream probe.  Each step has its own
# time limit; the script stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r3}
TESTS=${2:-"tests/test_gpu_models.py::test_umap_side_stream_is_bit_identical"}
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.out 2> gpurun_out/${TAG}_$name.err
  local rc=$?
  echo "$name rc=$rc"; tail -c 1500 gpurun_out/${TAG}_$name.out
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/${TAG}_$name.err; exit $rc; fi
}
if [ "$TESTS" != "none" ]; then
  step tests 600 python -u -m pytest $TESTS -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider
fi
step bench 600 python bench.py
step bench_bf16 300 python bench.py --conv-math bf16 --no-cpu-baseline --secondary-steps 0
step herlev256 600 python bench.py --workload herlev --res 256
step herlev224 300 python bench.py --workload herlev --res 224 --no-cpu-baseline
step probe 300 python tools/umap_stream_probe.py --steps 4 --reps 2
