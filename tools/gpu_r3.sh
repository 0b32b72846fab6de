#!/bin/bash
# Round-3 GPU session: diagnostics, then test files, then benches.  Each step has its own
# time limit; a plain test failure (rc 1) continues, a crash / timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r3}
shift
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.out 2> gpurun_out/${TAG}_$name.err
  local rc=$?
  echo "== $name rc=$rc"; grep -v "amdgpu.ids" gpurun_out/${TAG}_$name.out | tail -c 1200
  if [ $rc -gt 1 ]; then tail -20 gpurun_out/${TAG}_$name.err; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    bisect) step bisect 300 python tools/stream_bisect.py --reps 4 --main fwdbwd ;;
    bisect:*) m=${s#bisect:}; step bisect_$m 300 python tools/stream_bisect.py --reps 6 --main $m ;;
    dpsingle) step dpsingle 300 python tools/dp_probe.py single ;;
    xproc:*) IFS=: read -r _ st bs np it <<< "$s"
            step xproc_${st}_${bs}_${np} 300 python tools/xproc_bisect.py --stage $st --batch $bs --procs $np --iters ${it:-60} ;;
    micro:*) IFS=: read -r _ st bs it lib <<< "$s"
            step micro_${st}_${bs}_${lib:-tree} 300 env ${lib:+UGPG_LIB=exp/$lib.so} python tools/xproc_bisect.py --micro --stage $st --batch $bs --procs 2 --iters ${it:-60} ;;
    poison) step poison 400 python tools/dp_probe.py poison ;;
    dp) step dp 300 python tools/dp_probe.py dp ;;
    dpser) step dpser 300 env AMD_SERIALIZE_KERNEL=3 python tools/dp_probe.py dp ;;
    progprobe) step progprobe 600 python tools/prog_probe.py ;;
    probe) step probe 300 python tools/umap_stream_probe.py --steps 4 --reps 2 ;;
    stamps) step stamps 300 env UGPG_LIB=exp/lib_stamp.so python tools/clock_probe.py --stamps --seconds 1 --layers inc.3,down1.3,down2.3,down3.3,up4.0 &&
            step stamps16 300 env UGPG_LIB=exp/lib_stamp.so python tools/clock_probe.py --stamps --seconds 1 --math bf16 --out16 --layers inc.3,down1.3,down2.3,down3.3,up4.0 ;;
    wstamp:*) IFS=: read -r _ lib math <<< "$s"
            step wstamp_${lib}_${math} 300 env UGPG_LIB=exp/$lib.so python tools/clock_probe.py --stamps --wgrad --seconds 1 --math $math --out16 --layers inc.3,down1.3,down2.3,down3.3,up4.0 ;;
    stamp:*) IFS=: read -r _ lib math <<< "$s"
            step stamp_${lib}_${math} 300 env UGPG_LIB=exp/$lib.so python tools/clock_probe.py --stamps --seconds 1 --math $math --out16 --layers inc.3,down1.3,down2.3,down3.3,up4.0 ;;
    tests:*@@*) f=${s#tests:}; file=${f%%@@*}; kx=${f#*@@}; n=$(basename "$file" .py)
            step t_${n} 900 python -u -m pytest "$file" -k "$kx" -q -rf -x --timeout 400 --timeout-method thread -p no:cacheprovider ;;
    tests:*) f=${s#tests:}; n=$(basename "${f%% *}" .py); step t_${n%%::*} 900 python -u -m pytest $f -q -rf -x --timeout 400 --timeout-method thread -p no:cacheprovider ;;
    alltests) step alltests 1100 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread -p no:cacheprovider ;;
    ab:*) IFS=: read -r _ libs layers <<< "$s"
            step ab 400 python tools/conv_bench.py --rounds ${ROUNDS:-4} --maths ${MATHS:-x6,bf16} --layers ${layers:-inc.3,down1.0,down2.3,up4.0,up4.3} --libs $libs ${EXTRA:-} ;;
    abstep:*) IFS=@ read -r sa sb <<< "${s#abstep:}"
            step abstep 400 python tools/ab_step.py --a "$sa" --b "$sb" ${EXTRA:-} ;;
    convbench) step convbench 500 python tools/conv_bench.py --rounds 3 --maths ${MATHS:-bf16,x6} ${EXTRA:-} ;;
    bench) step bench 600 python bench.py ;;
    bench_bf16) step bench_bf16 300 python bench.py --conv-math bf16 --no-cpu-baseline --secondary-steps 0 ;;
    herlev256) step herlev256 600 python bench.py --workload herlev --res 256 ;;
    herlev224) step herlev224 300 python bench.py --workload herlev --res 224 --no-cpu-baseline ;;
  esac
done
