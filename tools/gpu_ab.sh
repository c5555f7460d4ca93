# A/B of environment variants on one box: for each "VAR=val" argument (or "base"),
# a short bench and rocprofv3 kernel stats.  usage: bash tools/gpu_ab.sh TAG base CTN_X=0 ...
# (one variant may set several variables: CTN_X=0,CTN_Y=1)
set -eo pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  n=${v//[^A-Za-z0-9]/_}
  if [ "$v" = base ]; then E=(); else IFS=, read -ra E <<< "$v"; fi
  env "${E[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$n.log 2>&1
  echo "$v $(tail -1 $O/bench_$n.log | cut -c1-140)"
done
for v in "$@"; do
  n=${v//[^A-Za-z0-9]/_}
  if [ "$v" = base ]; then E=(); else IFS=, read -ra E <<< "$v"; fi
  for kv in "${E[@]}"; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof_$n.log 2>&1
  for kv in "${E[@]}"; do unset "${kv%%=*}"; done
  echo "== $v"; python tools/prof_summary.py $(ls $O/prof_$n/*kernel_stats.csv | head -1) 7 10
done
