# A/B of experimental libugpg variants (exp/*.so, built with build.py -D ... --out) on
# selected conv layers; one process per variant, all forms timed inside each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
L=${LAYERS:-inc.3,down2.3,up1.0,up3.0,up4.0}
for lib in ug-pg-unet_amd/ugpg/libugpg.so exp/*.so; do
  echo "== $lib"
  UGPG_LIB=$lib timeout -k 10 120 python tools/conv_bench.py --rounds 2 --maths x6 --pipes ${PIPES:-0,1,2} --layers $L 2>&1 | grep -v amdgpu.ids || exit 1
done
