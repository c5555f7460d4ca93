# One parametrised GPU command script (run on the MI355X box through gpurun, from the
# repository root; results under gpurun_out/<tag>/, summaries copied into profiles/ by hand).
#
#   bash tools/gpu.sh suite <tag>                 whole -m gpu suite, smoke(), bench line, c4 and c5 lines
#   bash tools/gpu.sh tests <tag> <pytest args>   a pytest subset (-m gpu)
#   bash tools/gpu.sh bench <tag> [bench args]    one bench line (no CPU baseline)
#   bash tools/gpu.sh ab <tag> base VAR=v[,W=u]   bench lines per environment variant, alternated twice
#   bash tools/gpu.sh prof <tag>                  rocprofv3 kernel stats of the bench (live timer line beside it),
#                                                 FETCH/WRITE passes (per kernel + whole step), MFMA pass, c4 stats
#   bash tools/gpu.sh cfgprof <tag> c4|c5         kernel stats of one more config
#   bash tools/gpu.sh mb <tag> "<bin args>" ...   microbenchmark binaries under build/ (one quoted item each)
#   bash tools/gpu.sh pmcmb <tag> "<counters>" "<bin args>" ...   one --pmc pass per microbenchmark item
#   bash tools/gpu.sh rehearse <tag>              the N=2 bench job on one GPU over gloo (code path only)
#
# Every GPU step runs under its own time limit and the steps are chained: the first failure
# ends the call (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
cmd=$1; tag=$2; shift 2
O=gpurun_out/$tag
mkdir -p "$O"
ROOT=$(pwd)

line() {   # the bench JSON line's headline fields
  grep '^{' "$1" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], 'frac', r['frac'], 'mean_ms', r['mean_ms'], r['kernel'][:40])"
}

case $cmd in
suite)
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} --maxfail=5 -v -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  tail -1 $O/tests.log
  grep -E "FAILED|Error" $O/tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  echo "smoke ok"
  timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
  line $O/bench.log
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.log 2>&1 || exit 1
  line $O/c4.log
  timeout -k 10 300 python bench.py --config c5 --steps 6 --warmup 2 > $O/c5.log 2>&1 || exit 1
  line $O/c5.log
  ;;
tests)
  timeout -k 10 900 python -u -m pytest "$@" -x -v -m gpu --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error|assert|passed|failed" $O/tests.log | cut -c1-600 | tail -40
  exit $rc
  ;;
bench)
  timeout -k 10 500 python bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
  line $O/bench.log
  ;;
ab)
  for rep in 1 2; do
    for v in "$@"; do
      n=${v//[^A-Za-z0-9]/_}
      if [ "$v" = base ]; then E=(); else IFS=, read -ra E <<< "$v"; fi
      env "${E[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_${n}_$rep.log 2>&1 || { tail $O/bench_${n}_$rep.log; exit 1; }
      echo "$v: $(line $O/bench_${n}_$rep.log)"
    done
  done
  ;;
prof)
  # the live-timer line and the kernel statistics from one profiled run (the profiler's
  # overhead is the ratio of this line's ms/step to an unprofiled line's)
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_unprof.log 2>&1 || exit 1
  echo "unprofiled: $(line $O/bench_unprof.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-copy-peak --steps 10 --warmup 3 --profile-steps 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
  echo "profiled:   $(line $O/prof.log)"
  python3 tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 13 16 | tee $O/kernel_summary.txt
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $ROOT/$O/pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --no-copy-peak --steps 3 --warmup 1 --profile-steps 0 > $O/pmc_p$i.log 2>&1 || exit 1
  done
  python3 tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json
  python3 tools/pmc_step.py $O/pmc $(ls $O/prof/*kernel_trace.csv | head -1) 52.95 $O/pmc_step.json
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $ROOT/$O/pmc/mfma -o run -- python3 bench.py --no-cpu-baseline --no-copy-peak --steps 3 --warmup 1 --profile-steps 0 > $O/pmc_mfma.log 2>&1 || exit 1
  python3 tools/pmc_mfma.py $O/pmc/mfma $O/pmc_mfma.json | tee $O/mfma_util.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/profc4 -o run --output-format csv -- python3 bench.py --config c4 --no-copy-peak --steps 4 --warmup 2 --profile-steps 0 > $O/profc4.log 2>&1 || exit 1
  python3 tools/prof_summary.py $(ls $O/profc4/*kernel_stats.csv | head -1) 6 12 | tee $O/c4_kernel_summary.txt
  ;;
cfgprof)
  c=$1
  timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 3 > $O/${c}_bench.log 2>&1 || exit 1
  echo "$c: $(line $O/${c}_bench.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof$c -o run --output-format csv -- python3 bench.py --config $c --no-copy-peak --steps 4 --warmup 2 --profile-steps 0 > $O/prof$c.log 2>&1 || exit 1
  python3 tools/prof_summary.py $(ls $O/prof$c/*kernel_stats.csv | head -1) 6 16 | tee $O/${c}_kernel_summary.txt
  ;;
mb)
  for item in "$@"; do
    n=$(echo "$item" | tr -c 'A-Za-z0-9_\n' '_')
    timeout -k 10 120 $item > $O/mb_$n.log 2>&1 || { echo "FAILED: $item"; tail -20 $O/mb_$n.log; exit 1; }
    echo "== $item"; grep -vE "amdgpu.ids|^\s*$" $O/mb_$n.log | tail -${MB_TAIL:-12}
  done
  ;;
pmcmb)
  ctrs=$1; shift
  i=0
  for item in "$@"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $ROOT/$O/i$i/p1 -o run -- $item > $O/pmc_$i.log 2>&1 || { echo "FAILED: $item"; tail $O/pmc_$i.log; exit 1; }
    echo "== $item"; python3 tools/pmc_kernels.py $O/i$i "${PAT:-}" > $O/pmc_$i.txt
    cat $O/pmc_$i.txt
  done
  ;;
rehearse)
  export CTN_BENCH_REHEARSAL=1
  for ch in 4 1; do
    CTN_FLAT_CHUNKS=$ch timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + ch)) bench.py --gpus 2 --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline --no-copy-peak > $O/n2_chunks$ch.log 2>&1 || { tail -20 $O/n2_chunks$ch.log; exit 1; }
    tail -1 $O/n2_chunks$ch.log | cut -c1-220
  done
  ;;
*)
  echo "unknown command $cmd"; exit 2
  ;;
esac
