# c4 (causal cLN, L=16, 16 kHz, batch 64) and c5 (3 spk, N=512, 8 s, batch 16)
# train-step throughput on one MI355X, plus the default c2 line for comparison.
set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cfg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err
tail -1 $O/c2.json | cut -c1-160
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 > $O/c4.json 2> $O/c4.err
tail -1 $O/c4.json | cut -c1-160
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > $O/c5.json 2> $O/c5.err
tail -1 $O/c5.json | cut -c1-160
