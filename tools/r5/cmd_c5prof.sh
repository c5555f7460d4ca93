# round 5: c5 kernel statistics (rocprofv3) of the c5 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5c5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 4 --warmup 2 --profile-steps 0 > $O/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv | head -1) 6 22 | tee $O/c5_kernel_summary.txt
python tools/step_sequence.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/c5_step_sequence.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/profc2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 4 --warmup 2 --profile-steps 0 > $O/profc2.log 2>&1 || exit 1
python tools/prof_summary.py $(ls $O/profc2/*kernel_stats.csv | head -1) 6 22 > $O/c2_kernel_summary.txt
grep -E "dec_|enc_|total" $O/c2_kernel_summary.txt
