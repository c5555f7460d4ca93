# round 5: rocprofv3 kernel statistics of the default bench, the FETCH_SIZE / WRITE_SIZE
# passes (per-kernel and whole-step HBM traffic), the MFMA-busy pass, and c4 statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5prof}
O=gpurun_out/$T
mkdir -p $O/pmc
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 0 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 14 | tee $O/kernel_summary.txt
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --profile-steps 0 > $O/pmc/p$i.log 2>&1 || exit 1
done
python tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json
python tools/pmc_step.py $O/pmc $(ls $O/prof/*kernel_trace.csv | head -1) 52.95 $O/pmc_step.json
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc/mfma -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --profile-steps 0 > $O/pmc/mfma.log 2>&1 || exit 1
python tools/pmc_mfma.py $O/pmc/mfma $O/pmc_mfma.json | tee $O/mfma_util.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/profc4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --profile-steps 0 > $O/profc4.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/profc4/*kernel_stats.csv | head -1) 4 12 | tee $O/c4_kernel_summary.txt
