# Round-2 deliverables on one MI355X: the bench line (with CPU baseline), rocprofv3
# kernel stats, HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and MFMA utilisation
# (SQ_VALU_MFMA_BUSY_CYCLES pass) of the timed kernels.  One counter group per pass,
# kernel trace only.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02}
mkdir -p $O/pmc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 7 24 > $O/kernel_summary.txt
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc/p$i.log 2>&1
  rc=$?
  echo "PASS $i ($grp) EXIT $rc"
  [ $rc -eq 0 ] || exit 1
done
python3 tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json
python3 tools/pmc_mfma.py $O/pmc $O/pmc_mfma.json > $O/mfma_util.txt
head -12 $O/mfma_util.txt
cat $O/kernel_summary.txt | head -12
