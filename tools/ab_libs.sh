# In-process A/B of libugpg builds (exp/*.so plus the in-tree library) on selected
# conv layers: every variant timed in interleaved rounds inside ONE process.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
L=${LAYERS:-inc.3,down2.3,up4.0}
LIBS=ug-pg-unet_amd/ugpg/libugpg.so$(for f in exp/*.so; do printf ",%s" "$f"; done)
timeout -k 10 ${TMO:-240} python tools/conv_bench.py --rounds ${ROUNDS:-4} --maths x6 --pipes ${PIPES:-1,2} \
  --layers $L --libs $LIBS ${EXTRA:-} 2>&1 | grep -v amdgpu.ids
