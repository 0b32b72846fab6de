#!/bin/bash
# kernel-trace durations of the image-layer forward for library variants (A/B)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for ns in "" --nostats; do
    d=gpurun_out/kt_$(basename $lib .so)$ns
    UGPG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run -- python3 tools/conv_bench.py --maths x6 --rounds 3 --layers inc.0 $ns > $d.log 2>&1
    echo "== $lib $ns"
    python3 tools/kt_summary.py $d/run_results.db --match conv3x3 --top 3
  done
done
