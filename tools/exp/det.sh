set -eo pipefail
cd $GRAFT_REPO_ROOT
echo "== TPos + per-tile stats"; CTN_HIP_LIB=$PWD/build/var/lib_tpos.so timeout -k 10 120 python tools/exp/det_check.py
