# PMC passes (one group per pass) over a short bench run; summary of the ctn kernels
set -eo pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
i=0
for grp in "FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "WRITE_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/p$i.log 2>&1
  echo "PASS $i EXIT $?"
done
python tools/pmc_kern.py $O gemm_dual dw_bwd gemm_ws > $O/summary.txt
cat $O/summary.txt
