set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-host1}
mkdir -p $O
for b in 4 8 16 32; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --batch $b > $O/b$b.log 2>&1
  echo "batch $b $(tail -1 $O/b$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
