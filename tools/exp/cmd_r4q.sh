# round 4: where a streaming call's 1 ms goes (kernel trace of 1-stream 1-frame pushes)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4q}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/sprof -o run --output-format csv -- python3 tools/bench_streaming.py --streams 1 --frames 1 > $O/sprof.log 2>&1 || { tail $O/sprof.log; exit 1; }
python tools/prof_summary.py $(ls $O/sprof/*kernel_stats.csv | head -1) 60 20 | tee $O/stream_kernels.txt
python tools/trace_gaps.py $(ls $O/sprof/*kernel_trace.csv | head -1) sc_set_pos > $O/stream_gaps.txt; head -8 $O/stream_gaps.txt
python tools/step_sequence.py $(ls $O/sprof/*kernel_trace.csv | head -1) sc_set_pos > $O/stream_seq.txt; head -12 $O/stream_seq.txt
