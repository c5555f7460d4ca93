# bench.py throughput with the live kernel timer bracketing every launch of the timed
# kernel (stride 1), every 8th, or (practically) none, alternated on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-timer_ab}
mkdir -p $O
for r in 1 2; do
  for st in 1 8 100000; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --timer-stride $st > $O/b_${st}_$r.json 2> $O/b_${st}_$r.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['launches'], r['mean_ms'])" $O/b_${st}_$r.json "stride=$st run=$r"
  done
done
