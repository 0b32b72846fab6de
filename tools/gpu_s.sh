#!/bin/bash
# One targeted GPU session (round 5): named steps, each under its own time limit, stopping
# at the first crash / timeout / fault (exit > 1 for pytest; any nonzero otherwise).
#   bash tools/gpu_s.sh TAG step [step ...]
# steps:
#   t:<file>[:<-k expr>]   pytest -m gpu on one test file (optionally -k)
#   ab3v4                  same-box A/B: round-3 and round-4 final trees' bench, alternating
#   bench[:args]           bench.py (default line, no CPU baseline) with extra args ('+' = space)
#   prof[:args]            rocprofv3 --kernel-trace --stats of a short bench run
#   stamps:<x6|bf16>       in-kernel stamps (exp/lib_stamp.so) of five layers
#   abstep:<lib>:<math>   tools/ab_step.py in-tree vs exp/<lib>.so (x6 or bf16)
#   abx@<a>@<b>@<math>     tools/ab_step.py of two settings (lib:path / module._NAME=v)
#   cb:<args>              tools/conv_bench.py with args ('+' = space)
#   bin:<name>             a probe binary exp/<name> (e.g. tools/store_probe.cpp)
#   env:VAR=VAL / unenv:VAR   set / unset an environment variable for the following steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 sec=$2; shift 2
  timeout -k 10 "$sec" "$@" > "gpurun_out/${TAG}_${name}.out" 2> "gpurun_out/${TAG}_${name}.err"
  local rc=$?
  echo "[$TAG] $name rc=$rc"; tail -4 "gpurun_out/${TAG}_${name}.out"
  return $rc
}
for s in "$@"; do
  case $s in
    t:*)
      IFS=: read -r _ f k <<< "$s"
      n=$(basename "$f" .py)${k:+_k}
      if [ -n "$k" ]; then
        run "$n" 900 python -u -m pytest "tests/$f" -m gpu -x -q -rfP -k "$k" --timeout 300 --timeout-method thread -p no:cacheprovider
      else
        run "$n" 900 python -u -m pytest "tests/$f" -m gpu -x -q -rfP --timeout 300 --timeout-method thread -p no:cacheprovider
      fi
      rc=$?; [ $rc -gt 1 ] && exit $rc ;;
    ab3v4)
      for i in 1 2 3; do
        for t in r3 r4; do
          run "ab_${t}_$i" 300 python exp/${t}tree/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
        done
      done ;;
    bench*)
      a=${s#bench}; a=${a#:}; a=${a//+/ }
      nb=$((nb+1)); run "bench${nb}" 600 python bench.py --no-cpu-baseline $a || exit $? ;;
    prof*)
      a=${s#prof}; a=${a#:}; a=${a//+/ }
      run "prof${a// /}" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_${TAG}${a// /}" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline $a || exit $? ;;
    cb:*)
      a=${s#cb:}; a=${a//+/ }
      nc=$((nc+1)); run "convbench${nc}" 600 python tools/conv_bench.py $a || exit $? ;;
    stamps:*)  # in-kernel loader/compute stamps of exp/lib_stamp.so (-D X6R_STAMP=1), math x6 or bf16
      m=${s#stamps:}; ns=$((ns+1))
      run "stamps${ns}_$m" 300 env UGPG_LIB=exp/lib_stamp.so python tools/clock_probe.py --stamps --seconds 1 --math $m $( [ "$m" = bf16 ] && echo --out16 ) --layers ${STAMP_LAYERS:-inc.3,down1.3,down2.3,down3.3,up4.0} || exit $? ;;
    stampsl:*)  # stamps of another stamp build: stampsl:<exp lib name>:<math>
      IFS=: read -r _ l m <<< "$s"; ns=$((ns+1))
      run "stamps${ns}_${l}_$m" 300 env UGPG_LIB=exp/$l.so python tools/clock_probe.py --stamps --seconds 1 --math $m $( [ "$m" = bf16 ] && echo --out16 ) --layers ${STAMP_LAYERS:-inc.3,down1.3,down2.3,down3.3,up4.0} || exit $? ;;
    wstamps:*)  # weight-gradient loader stamps of exp/lib_wstamp.so (-D X6W_STAMP=1)
      m=${s#wstamps:}; ns=$((ns+1))
      run "wstamps${ns}_$m" 300 env UGPG_LIB=exp/lib_wstamp.so python tools/clock_probe.py --stamps --wgrad --seconds 1 --math $m $( [ "$m" = bf16 ] && echo --out16 ) --layers ${STAMP_LAYERS:-inc.3,down1.3,down2.3,down3.3,up4.0} || exit $? ;;
    abstep:*)  # in-process whole-step A/B: in-tree library vs exp/<lib>.so, arithmetic m
      IFS=: read -r _ l m <<< "$s"; na=$((na+1))
      run "abstep${na}_${l}_$m" 600 python tools/ab_step.py --a lib:ug-pg-unet_amd/ugpg/libugpg.so --b lib:exp/$l.so --conv-math $m --rounds 6 || exit $? ;;
    abx@*)  # in-process whole-step A/B of two settings: abx@<a>@<b>@<math> (tools/ab_step.py)
      IFS=@ read -r _ sa sb m <<< "$s"; na=$((na+1))
      run "abx${na}_$m" 600 python tools/ab_step.py --a "$sa" --b "$sb" --conv-math $m --rounds 6 || exit $? ;;
    py:*)  # python <args> ('+' = space), e.g. py:tools/img_bench.py+--libs+a.so,b.so
      a=${s#py:}; a=${a//+/ }; npy=$((npy+1))
      run "py${npy}" 600 python $a || exit $? ;;
    bin:*)  # a prebuilt probe binary under exp/: bin:<name>
      b=${s#bin:}; run "bin_$b" 300 exp/$b || exit $? ;;
    env:*) export "${s#env:}"; echo "[$TAG] export ${s#env:}" ;;
    unenv:*) unset "${s#unenv:}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
