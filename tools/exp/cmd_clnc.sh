# combined cLN dual statistics: reproducibility screen (3 shapes, both norms), GPU suite,
# c4 A/B against build/ab/lib_prev.so with a c4 kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-clnc}
SHAPES="3 1000;32 3199;64 7999" NRUN=20 bash tools/gpu_det.sh $T lib:c lib || exit 1
AB_BENCH="--config c4 --steps 8 --warmup 2" bash tools/exp/cmd_ab.sh $T || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/profc4 -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/$T/profc4.log 2>&1 || exit 1
python tools/prof_summary.py $(ls gpurun_out/$T/profc4/*kernel_stats.csv | head -1) 4 10
