# Kernel-time comparison of library variants (build/var/lib<tag>.so) on one box:
# a short profiled bench per variant, summarising the named kernels.
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-var}; shift
PAT=${PAT:-gemm_cols_kernel}
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = "0" ]; then L=$GRAFT_REPO_ROOT/conv-tasnet_amd/libctn_hip.so; else L=$GRAFT_REPO_ROOT/build/var/lib$v.so; fi
  CTN_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/b$v.json 2> $O/b$v.err
  echo "== $v $(cut -c60-90 $O/b$v.json)"
  python tools/prof_summary.py $O/p$v/run_kernel_stats.csv 20 16 | grep -E "$PAT" || true
done
