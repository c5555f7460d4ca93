# round 5: the whole -m gpu suite, smoke(), the default bench line and c4 / c5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} --maxfail=5 -v -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
grep -E "FAILED|Error" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log | cut -c1-200
timeout -k 10 300 python bench.py --config c5 --steps 6 --warmup 2 > $O/c5.log 2>&1 || exit 1
tail -1 $O/c5.log | cut -c1-200
