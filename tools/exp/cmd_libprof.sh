# rocprofv3 kernel stats of a short bench run per library build (build/ab/lib_<name>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-libprof}; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for n in "$@"; do
  CTN_HIP_LIB=$PWD/build/ab/lib_$n.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof_$n.log 2>&1 || exit 1
  echo "== $n"
  python tools/prof_summary.py $(ls $O/prof_$n/*kernel_stats.csv | head -1) 7 8
done
