# LDS / issue-stall counters of the block kernels (one --pmc pass each, kernel trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ldspmc}
mkdir -p $OUT
i=0
for grp in "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/p$i.log 2>&1
  rc=$?
  echo "PASS $i EXIT $rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_kernels.py $OUT "${PAT:-}" > $OUT/summary.txt && cat $OUT/summary.txt
