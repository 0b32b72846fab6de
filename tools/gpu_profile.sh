#!/bin/bash
# rocprofv3 kernel-trace stats (CSV) + PMC passes for HBM traffic and MFMA activity.
# EXTRA: more bench.py arguments (e.g. EXTRA='--conv-math bf16' for config 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r1}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --secondary-steps 0 ${EXTRA:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
echo trace ok
for ctr in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$tag -o run -- python3 bench.py $ARGS > $OUT/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $OUT/pmc_$tag.log; exit 1; }
  echo pmc $tag ok
done
find $OUT -name "*.csv" | head -20
