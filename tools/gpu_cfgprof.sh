# c4 / c5 bench lines and rocprofv3 kernel stats (round-2 config profiles)
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cfgp}
mkdir -p $O
export TMPDIR=/tmp
for c in c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 > $O/$c.json 2> $O/$c.err
  tail -1 $O/$c.json | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 > $O/prof_$c.log 2>&1
  echo "== $c"; python tools/prof_summary.py $(ls $O/prof_$c/*kernel_stats.csv | head -1) 4 14
done
