timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_conv.log 2>&1; rc=$?; tail -3 gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit $rc
for f in 0 1; do echo "== x6_wgrad=$f"; UGPG_X6_WGRAD=$f timeout -k 10 300 python tools/conv_bench.py --rounds 2 --maths x6 --pipes 1 --wgrad 2>&1 | grep -v amdgpu.ids | sed 's/fwd_x6=[^ ]* //; s/dgrad_x6=[^ ]* //' || exit 1; done
