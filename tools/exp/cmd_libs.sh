# bench line per library build (build/ab/lib_<name>.so, CTN_HIP_LIB), alternating twice;
# BENCH_ARGS overrides the bench arguments
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-libs}; shift
O=gpurun_out/$T
mkdir -p $O
for r in 1 2; do for n in "$@"; do
  CTN_HIP_LIB=$PWD/build/ab/lib_$n.so timeout -k 10 200 python bench.py ${BENCH_ARGS:---no-cpu-baseline --steps 20 --warmup 5} > $O/bench_${n}_$r.log 2>&1 || exit 1
  python - "$O/bench_${n}_$r.log" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["roofline"]["kernel"][:28], d["roofline"]["mean_ms"])
PY
done; done
