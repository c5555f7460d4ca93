# round 4: cLN dual ring look-ahead 3 (variant library) vs the default 5 at c4
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4pfc}
O=gpurun_out/$T; mkdir -p $O
V=$GRAFT_REPO_ROOT/build/var/libpfc3.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/base$i.json 2> $O/base$i.err || exit 1
  CTN_HIP_LIB=$V timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/pfc3_$i.json 2> $O/pfc3_$i.err || exit 1
done
for f in $O/*.json; do echo "$f $(tail -1 $f | cut -c60-140)"; done
CTN_HIP_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "cln or c4 or causal or determin" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
