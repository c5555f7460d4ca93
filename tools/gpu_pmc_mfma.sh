# MFMA-utilisation and issue-stall counters per kernel over a short bench run
# (one counter group per rocprofv3 pass, kernel trace only; no other trace domains).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcm}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1; echo "LIST EXIT $?"
i=0
for grp in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/p$i.log 2>&1
  rc=$?
  echo "PASS $i ($grp) EXIT $rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_mfma.py $OUT $OUT/pmc_mfma.json > $OUT/summary.txt && cat $OUT/summary.txt
