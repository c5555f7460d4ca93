# round 5: dw_debug.py over library variants (CTN_HIP_LIB)
cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  echo "== $lib"
  CTN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python tools/exp/dw_debug.py 32 3199 1 0 2>&1 | grep -v amdgpu.ids | grep -E "mismatches|rows|channels" || exit 1
done
