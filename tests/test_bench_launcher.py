"""bench.py --gpus N without torchrun: the parent starts N rank processes itself
(bench.spawn_ranks).  Driven here with a stub worker over gloo on the CPU, so the
launcher's environment contract (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) and its
exit-code handling are checked without a GPU."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r"""
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"])
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
open(os.path.join(sys.argv[1], f"rank{r}"), "w").write(f"{w} {int(t)}")
dist.barrier()
dist.destroy_process_group()
"""


def test_spawn_ranks_starts_world_size_ranks(tmp_path):
    n = 3
    rc = bench.spawn_ranks(n, [sys.executable, "-c", STUB, str(tmp_path)])
    assert rc == 0
    got = sorted(os.listdir(tmp_path))
    assert got == [f"rank{r}" for r in range(n)]
    for r in range(n):
        w, total = (tmp_path / f"rank{r}").read_text().split()
        assert int(w) == n and int(total) == n * (n + 1) // 2


def test_spawn_ranks_reports_a_failing_rank():
    stub = "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"
    assert bench.spawn_ranks(2, [sys.executable, "-c", stub]) == 3


def test_bench_refuses_more_gpus_than_visible():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
